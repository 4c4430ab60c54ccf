# r6h: blob70k BVH build knobs re-swept under the current kernel (leaf size, SAH traversal cost,
# collapse) and its item order on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6h
mkdir -p $T
timeout -k 10 500 python tools/sweep.py --scene blob70k --steps 3 leaf=1,2,3 tcost=70,100,140 > $T/sweep_blob_build.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 collapse=0,1 > $T/sweep_blob_collapse.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 order=0,1,0,1 > $T/ab_blob_order.txt 2>&1
echo "r6h rc=$?"
