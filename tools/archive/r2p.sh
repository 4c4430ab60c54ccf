set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2p
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 leafexit=15,17,18,19,20,22 > gpurun_out/r2p/blob.jsonl 2>&1 &&
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 leafexit=4,8,12,15,18 > gpurun_out/r2p/random.jsonl 2>&1 &&
timeout -k 10 300 python tools/sweep.py --blob 64,34 --steps 3 leafexit=6,9,12,15 > gpurun_out/r2p/blobsmall.jsonl 2>&1
