# r3j: full GPU parity suite + smoke + default bench with the fused combine
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3j
bash tools/gpu_tests.sh r3j && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r3j/cornell.json 2> gpurun_out/r3j/cornell.err && \
timeout -k 10 300 python3 bench.py --scene blob70k --cpu-baseline off > gpurun_out/r3j/blob.json 2>> gpurun_out/r3j/err
