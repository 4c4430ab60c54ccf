# r4e: final tree of the round (rebuilt in a fresh container, HIPPT_REJECT_CAP off) — GPU suite + fuzz, smoke, every bench line, both profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4e
bash tools/gpu_tests.sh r4e && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e/smoke.log 2>&1 && \
bash tools/run_round_bench.sh r4e
