# r5k: the camera-ray pool in the queue's tail generates only the lanes' shortfall
# (HIPPT_POOL_TAIL) — parity, strong-scaling rehearsal (every 1/8 share) and full-size A/B
# against the variant without it (libv_notail)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5k
mkdir -p $T
V=qt-raytracer_amd/libv_notail.so
bash tools/gpu_tests.sh r5k "pool or headline or row_interleave or matches_oracle or deferred" && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_tail.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_notail.jsonl 2>&1 && \
for i in 1 2; do
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
done
echo "r5k rc=$?"
