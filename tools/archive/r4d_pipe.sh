# round 4: GPU suite with pipelined batches (HIPPT_OPT_PIPELINE automatic), then the pipeline A/B on
# the 1/N row shares (tools/band_scaling.py, wall time per step of 20 back-to-back steps)
set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d/pytest.log 2>&1 || exit 1
for i in 1 2; do
  for pipe in 0 1; do
    timeout -k 10 120 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,2,4,8 31=$pipe > gpurun_out/r4d/cornell_pipe${pipe}_$i.jsonl || exit 1
  done
done
for pipe in 0 1; do
  timeout -k 10 150 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,8 31=$pipe > gpurun_out/r4d/blob_pipe${pipe}.jsonl || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/r4d/bench_cornell.json 2> gpurun_out/r4d/bench_cornell.err || exit 1
