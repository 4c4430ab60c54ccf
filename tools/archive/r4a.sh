# r4a: rebuilt tree (fresh container) — GPU suite + fuzz, smoke, default Cornell bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
bash tools/gpu_tests.sh r4a && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r4a/cornell.json 2> gpurun_out/r4a/cornell.err && \
timeout -k 10 300 python3 bench.py --scene blob70k --cpu-baseline off > gpurun_out/r4a/blob.json 2>> gpurun_out/r4a/err
