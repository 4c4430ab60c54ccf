# round 4, last tree: the GPU suite and smoke on the library built from the final sources
set -o pipefail
mkdir -p gpurun_out/r4w
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4w/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4w/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r4w/cornell.json 2> gpurun_out/r4w/cornell.err || exit 1
