# s7q: the final commit of the session: full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh s7q && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s7q/smoke.log 2>&1
echo "s7q rc=$?"
