# r5w: runs handed out by an estimated sample length (longest first) instead of hit/sky —
# parity, full-size A/B against the hit/sky build (libv_prev) and order off, blob with the order
# forced on, 1/8-share rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5w
mkdir -p $T
V=qt-raytracer_amd/libv_prev.so
bash tools/gpu_tests.sh r5w "item_order or headline or pool or row_interleave" && \
for i in 1 2; do
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 order=-1,0 >> $T/ab_cornell.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 order=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
done && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 4 order=0,1,0,1 > $T/ab_blob.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell_mixed --steps 4 order=0,1,0,1 > $T/ab_mixed.txt 2>&1 && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_prev.jsonl 2>&1
echo "r5w rc=$?"
