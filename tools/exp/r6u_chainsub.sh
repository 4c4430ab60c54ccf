# round 6: the chained GPU subset with the automatic item order added (the production default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6u
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chain or deferred or held or closes" > gpurun_out/r6u/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r6u/pytest.log
exit $rc
