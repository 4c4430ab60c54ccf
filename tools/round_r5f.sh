# r5f: exact tail claims — GPU suite, A/B against 64-item tail chunks at full size and for the
# 1/8 shares of the strong-scaling job (every rank), the fixed per-launch cost, the timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5f
mkdir -p $T
bash tools/gpu_tests.sh r5f && \
bash tools/ab.sh cornell34 5 tail64 exact > $T/ab_tail_cornell.txt 2>&1 && \
bash tools/ab.sh blob70k 5 tail64 exact > $T/ab_tail_blob.txt 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tail64.so timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_tail64.jsonl 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_exact.so timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_exact.jsonl 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tail64.so timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_tail64.jsonl 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_exact.so timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_exact.jsonl 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 8 > $T/timeline_cornell_s8.json 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene blob70k --stride 8 > $T/timeline_blob_s8.json 2>&1
echo "r5f rc=$?"
