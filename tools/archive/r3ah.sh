# r3ah: final state (leaf size 2 default) — full GPU parity suite, smoke, then every bench line and
# the rocprof profiles of the two headline scenes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ah
bash tools/gpu_tests.sh r3ah && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ah/smoke.log 2>&1 && \
bash tools/run_round_bench.sh r3ah
