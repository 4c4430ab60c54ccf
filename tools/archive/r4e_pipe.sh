# round 4: pipeline A/B with the item order forced (28=1: its table built in the warm-up call)
set -o pipefail
mkdir -p gpurun_out/r4e
for i in 1 2; do
  for pipe in 0 1; do
    timeout -k 10 120 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 28=1 31=$pipe > gpurun_out/r4e/cornell_pipe${pipe}_$i.jsonl || exit 1
  done
done
for pipe in 0 1; do
  timeout -k 10 150 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,8 28=1 31=$pipe > gpurun_out/r4e/blob_pipe${pipe}.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4e/prof -o pipe1 -- python3 -u tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 31=1 > gpurun_out/r4e/prof_pipe1.log 2>&1 || exit 1
