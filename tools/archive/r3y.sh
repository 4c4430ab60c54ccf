# r3y: final-tree check — full GPU parity suite, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3y
bash tools/gpu_tests.sh r3y && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3y/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r3y/cornell.json 2> gpurun_out/r3y/cornell.err
