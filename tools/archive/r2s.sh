# r2s: BVH build-parameter sweep (SAH traversal cost x100, max leaf size) on Cornell and blob70k
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2s
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 3 --count tcost=50,100,200,300,500 leaf=2,4,8,15 > gpurun_out/r2s/cornell.jsonl && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 2 --count tcost=70,100,150 leaf=2,4,6 > gpurun_out/r2s/blob.jsonl
