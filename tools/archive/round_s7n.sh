# s7n: the session's final tree: full GPU suite, smoke, headline line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7n
mkdir -p $O
bash tools/gpu_tests.sh s7n && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err
echo "s7n rc=$?"
