# round 6: random chained host-call sequences against one launch per batch, audited
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6v
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain_fuzz.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r6v/pytest.log 2>&1; rc=$?
grep "seed\|passed\|failed\|Error" gpurun_out/r6v/pytest.log
exit $rc
