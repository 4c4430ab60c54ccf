# round 4, the library as committed last: GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4y/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4y/smoke.log 2>&1 || exit 1
