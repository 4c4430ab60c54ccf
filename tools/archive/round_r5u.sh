# r5u: queue claims read the counter first (no atomics on a drained queue) — item-order parity
# test, 1/8-share rehearsal and launch-overhead points against the previous build (libv_prev),
# full-size A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5u
mkdir -p $T
V=qt-raytracer_amd/libv_prev.so
bash tools/gpu_tests.sh r5u "item_order or headline or row_interleave or split" && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_prev.jsonl 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_prev.jsonl 2>&1 && \
for i in 1 2; do
  timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 >> $T/spp4.jsonl 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 >> $T/spp4_prev.jsonl 2>&1 || exit 1
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
done
echo "r5u rc=$?"
