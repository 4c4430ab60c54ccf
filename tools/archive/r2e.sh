set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2e
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r2e/phase_cornell.json 2>&1 &&
timeout -k 10 120 python tools/phase_profile.py --scene blob70k quant=0 > gpurun_out/r2e/phase_blob.json 2>&1
