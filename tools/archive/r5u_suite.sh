# round 5: the full GPU suite and smoke on the automatic chain / claim-size build
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5u
sha256sum qt-raytracer_amd/libhippt.so > gpurun_out/r5u/lib.sha256
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5u/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r5u/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5u/smoke.log 2>&1 || { tail -20 gpurun_out/r5u/smoke.log; exit 1; }
tail -1 gpurun_out/r5u/smoke.log
