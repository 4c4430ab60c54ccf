# r5d: strong-scaling rehearsal on one GPU (every rank's interleaved share timed, N = 1, 2, 4, 8)
# for configs[1] and configs[2], the fixed per-launch cost, and the per-wave timeline of a 1/8 share
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5d
mkdir -p $T
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,2,4,8 > $T/scaling_cornell.jsonl 2> $T/scaling_cornell.err && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,2,4,8 > $T/scaling_blob.jsonl 2> $T/scaling_blob.err && \
timeout -k 10 120 python tools/launch_overhead.py --scene cornell34 > $T/overhead_cornell.json 2>&1 && \
timeout -k 10 120 python tools/launch_overhead.py --scene blob70k > $T/overhead_blob.json 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 8 > $T/timeline_cornell_s8.json 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_tl.so timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 1 > $T/timeline_cornell_s1.json 2>&1
echo "r5d rc=$?"
