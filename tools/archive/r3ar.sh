# r3ar: automatic collapse (SAH-optimal for LDS-sized scenes) — full GPU suite + fuzz, smoke, bench lines
# of the LDS scenes and blob (greedy, unchanged)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ar
B="timeout -k 10 300 python3 bench.py"
bash tools/gpu_tests.sh r3ar && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ar/smoke.log 2>&1 && \
$B > gpurun_out/r3ar/cornell.json 2> gpurun_out/r3ar/err && \
$B --scene cornell_mixed --cpu-baseline off > gpurun_out/r3ar/mixed.json 2>> gpurun_out/r3ar/err && \
$B --scene blob70k --cpu-baseline off > gpurun_out/r3ar/blob.json 2>> gpurun_out/r3ar/err && \
bash tools/profile.sh r3ar && python3 tools/prof_summary.py r3ar > /dev/null
