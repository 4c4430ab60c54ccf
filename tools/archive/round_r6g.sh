# r6g: loop exits scaled to the wave's live lanes (HIPPT_SCALED_EXITS) — parity subset, the 1/8
# share (every band) and full size against the unscaled build (libv_unscaled), timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6g
mkdir -p $T
V=qt-raytracer_amd/libv_unscaled.so
bash tools/gpu_tests.sh r6g "headline or pool or item_order or matches_oracle" && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_unscaled.jsonl 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_unscaled.jsonl 2>&1 && \
for i in 1 2; do
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  timeout -k 10 100 python tools/sweep.py --scene blob70k --steps 4 pool=-1 >> $T/ab_blob.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene blob70k --steps 4 pool=-1 >> $T/ab_blob.txt 2>&1 || exit 1
done && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 8 > $T/timeline_cornell_stride8.json 2>&1
echo "r6g rc=$?"
