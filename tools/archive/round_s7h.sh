# s7h: final tree of the session: full GPU suite, smoke, the app-path timing and the headline line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7h
mkdir -p $O
bash tools/gpu_tests.sh s7h && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err && \
timeout -k 10 300 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err
echo "s7h rc=$?"
