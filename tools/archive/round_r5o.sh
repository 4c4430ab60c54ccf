# r5o: full GPU suite + smoke + the default bench line after the payload-queue wavefront
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5o
mkdir -p $T
bash tools/gpu_tests.sh r5o && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $T/bench_default.json 2> $T/bench_default.err
echo "r5o rc=$?"
