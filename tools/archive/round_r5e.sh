# r5e: top-first hybrid traversal (float LDS top, 8-bit nodes below; the two node formats never in
# one iteration): its parity tests, then the A/B against float and 8-bit nodes on blob70k
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5e
mkdir -p $T
bash tools/gpu_tests.sh r5e "lds_top or quantized or fuzz or headline" && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 5 quant=0,2,0,2,1 > $T/ab_hybrid_topfirst_blob.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --width 3840 --height 2160 --spp 16 --steps 3 quant=0,2,0,2 > $T/ab_hybrid_topfirst_blob4k.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 quant=2 leafexit=9,13,17,25 > $T/sweep_hybrid_exits.txt 2>&1
echo "r5e rc=$?"
