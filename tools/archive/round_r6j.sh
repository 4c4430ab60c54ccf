# r6j: camera pool on trees in global memory re-checked under the current kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6j
mkdir -p $T
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 pool=0,1,0,1 > $T/ab_blob_pool.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 pool=0,1,0,1 > $T/ab_random_pool.txt 2>&1
echo "r6j rc=$?"
