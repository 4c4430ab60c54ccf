# r5g: overlapped batches on two trace streams (HIPPT_OPT_TRACE_STREAMS) — parity (the async/deferred
# suite in both modes), in-process A/B at full size, the strong-scaling rehearsal (every 1/8 share)
# and bench lines with it on
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5g
mkdir -p $T
bash tools/gpu_tests.sh r5g "deferred or switch or headline or present or batches" && \
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 6 streams=0,1,0,1 > $T/ab_streams_cornell.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 6 streams=0,1,0,1 > $T/ab_streams_blob.txt 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,2,4,8 29=1 > $T/scaling_cornell_streams.jsonl 2>&1 && \
timeout -k 10 300 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,2,4,8 29=1 > $T/scaling_blob_streams.jsonl 2>&1 && \
timeout -k 10 300 python bench.py --trace-streams 1 --cpu-baseline off > $T/bench_cornell_streams.json 2> $T/bench_cornell_streams.err && \
timeout -k 10 300 python bench.py --trace-streams 1 --preset config3 --cpu-baseline off > $T/bench_blob_streams.json 2> $T/bench_blob_streams.err && \
timeout -k 10 300 python bench.py --trace-streams 1 --preset config4 --steps 3 --warmup 1 --cpu-baseline off > $T/bench_blob4k_streams.json 2> $T/bench_blob4k_streams.err
echo "r5g rc=$?"
