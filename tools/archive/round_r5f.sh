# r5f: the launch's tail — exact claims near a queue's end (EXACT) and loop exits off for waves with
# few live lanes (SCALE): GPU suite, 4-way A/B at full size, every rank's 1/8 share of the strong-
# scaling job for each variant, the per-wave timeline of a 1/8 share
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5f
mkdir -p $T
bash tools/gpu_tests.sh r5f && \
bash tools/ab.sh cornell34 5 base exact scale both > $T/ab_tail_cornell.txt 2>&1 && \
bash tools/ab.sh blob70k 5 base exact scale both > $T/ab_tail_blob.txt 2>&1 && \
for v in base both; do
  HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_$v.jsonl 2>&1 || exit 1
  HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_$v.jsonl 2>&1 || exit 1
done && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 8 > $T/timeline_cornell_s8.json 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene blob70k --stride 8 > $T/timeline_blob_s8.json 2>&1
echo "r5f rc=$?"
