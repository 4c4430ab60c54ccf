# round 5: chained batches with the single-claimer mailbox refresh: diagnostics, parity subset,
# kernel traces of 20 chained steps, chain on/off timing
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 200 python -u tools/exp/chain_debug.py cornell34 > $O/dbg_cornell.txt 2>&1 || { cat $O/dbg_cornell.txt; exit 1; }
grep -c " 0 px differ" $O/dbg_cornell.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread -k "chained or deferred_combine or async" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "8 30=8" "1 30=-1"; do
  set -- $cfg
  tag=r${1}_$(echo $2 | tr '=' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$tag -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks $1 28=1 $2 > $O/$tag.jsonl 2> $O/$tag.err || exit 1
done
for sc in cornell34 blob70k; do
  for ch in -1 0; do
    timeout -k 10 200 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,8 28=1 30=$ch > $O/${sc}_chain${ch}.jsonl || exit 1
  done
done
for f in $O/*.jsonl; do echo $f; cat $f; done
