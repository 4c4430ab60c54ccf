# r5v: the full GPU suite, then every round-3 bench line, the rocprof kernel-trace + PMC
# profiles of the two headline workloads and the legacy-ABI timing (tools/round3_bench.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r5v && bash tools/round3_bench.sh r5v
