# round 5: the 37-same-frame-batch failure of r5o — the test's own sequence on the default build
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5r3
mkdir -p $O
for io in -1 1 0; do
  timeout -k 10 200 python -u tools/exp/chain_debug3.py $io > $O/io$io.txt 2> $O/io$io.err || { tail -5 $O/io$io.err; exit 1; }
  echo "== item order $io"; grep -v " 0 px differ, 0 NaN" $O/io$io.txt; grep -c "0 px differ, 0 NaN" $O/io$io.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "chained" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
