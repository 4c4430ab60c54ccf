# r3d: camera pool on global-memory trees with smaller LDS stacks (more LDS for the top)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 pool=0,1 stackcap=0,9,11 > gpurun_out/r3d/blob.jsonl 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 pool=0,1 stackcap=0,7,9 > gpurun_out/r3d/random.jsonl 2>&1
