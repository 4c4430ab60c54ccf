set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2q && bash tools/run_round_bench.sh r2q > gpurun_out/r2q/round.log 2>&1
