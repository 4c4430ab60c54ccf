# r3au: final state of round 2 in one tag — GPU suite + fuzz, smoke, every bench line, both profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3au
bash tools/gpu_tests.sh r3au && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3au/smoke.log 2>&1 && \
bash tools/run_round_bench.sh r3au
