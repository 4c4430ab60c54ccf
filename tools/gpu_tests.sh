#!/bin/bash
# tools/gpu_tests.sh TAG [pytest -k expr] — GPU parity suite on the box (via gpurun), log under gpurun_out/TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-gputest}
mkdir -p gpurun_out/$TAG
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest.log
exit $rc
