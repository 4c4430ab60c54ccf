# r6n: blob70k camera pool with 8-bit nodes (the same LDS then holds twice the top nodes)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6n
mkdir -p $T
bash tools/gpu_tests.sh r6n "lds_top or pool" && \
timeout -k 10 400 python tools/sweep.py --scene blob70k --steps 3 quant=0,1,0,1 pool=1 > $T/ab_blob_quant_pool.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 quant=1 pool=1 stackcap=8,10,13 > $T/sweep_quant_pool_cap.txt 2>&1
echo "r6n rc=$?"
