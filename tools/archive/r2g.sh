set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2g && bash tools/run_round_bench.sh r2g > gpurun_out/r2g/round.log 2>&1
