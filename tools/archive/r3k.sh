# r3k: fresh-container re-check — full GPU parity suite + smoke + default bench (fused combine on)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3k
bash tools/gpu_tests.sh r3k && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3k/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r3k/cornell.json 2> gpurun_out/r3k/cornell.err
