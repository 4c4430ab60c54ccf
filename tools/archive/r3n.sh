# r3n: phase profiles (counting builds) of blob70k and cornell34 on the current kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3n
timeout -k 10 200 python tools/phase_profile.py --scene blob70k > gpurun_out/r3n/blob.json 2>&1 && \
timeout -k 10 200 python tools/phase_profile.py --scene cornell34 > gpurun_out/r3n/cornell.json 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 2 --count > gpurun_out/r3n/blob_count.jsonl 2>&1
