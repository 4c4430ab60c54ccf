# round 4: GPU suite on the current tree, then every BASELINE config's bench line and the rocprof
# profiles of the two headline scenes (tools/run_round_bench.sh)
set -o pipefail
mkdir -p gpurun_out/r4j
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4j/smoke.log 2>&1 || exit 1
bash tools/run_round_bench.sh r4j > gpurun_out/r4j/round_bench.log 2>&1 || exit 1
