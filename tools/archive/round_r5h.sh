# r5h: primary candidate lists (HIPPT_OPT_PRIMARY_LISTS) — parity (lists on/off/auto, pool and
# one-by-one refill, interleaved rows, camera changes, the full-size headline goldens), in-process
# A/B at full size, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5h
mkdir -p $T
bash tools/gpu_tests.sh r5h "primary or camera_pool or headline or row_interleave or matches_oracle" && \
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 6 prim=0,1,0,1 > $T/ab_prim_cornell.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 6 prim=0,1,0,1 > $T/ab_prim_blob.txt 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline off > $T/bench_cornell.json 2> $T/bench_cornell.err && \
timeout -k 10 300 python bench.py --preset config3 --cpu-baseline off > $T/bench_blob.json 2> $T/bench_blob.err
echo "r5h rc=$?"
