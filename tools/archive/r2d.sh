set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2d
timeout -k 10 200 bash tools/ab.sh cornell34 5 base nospill > gpurun_out/r2d/ab_cornell.txt 2>&1 &&
timeout -k 10 200 bash tools/ab.sh blob70k 3 base nospill > gpurun_out/r2d/ab_blob.txt 2>&1 &&
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r2d/phase_cornell.json 2>&1 &&
timeout -k 10 120 python tools/phase_profile.py --scene blob70k > gpurun_out/r2d/phase_blob.json 2>&1
