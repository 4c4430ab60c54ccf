# s7r: zero-copy frames with the copy as fallback: full GPU suite, smoke, app-path timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7r
mkdir -p $O
bash tools/gpu_tests.sh s7r && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err
echo "s7r rc=$?"
