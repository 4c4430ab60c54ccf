# round 5: chained batches with one querier per block, packed per-XCD copy, sleeping losers — diagnostics,
# parity subset, chain caps on the Cornell share / whole image and blob70k, kernel traces
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 200 python -u tools/exp/chain_debug.py cornell34 > $O/dbg_cornell.txt 2>&1 || { cat $O/dbg_cornell.txt; exit 1; }
grep -c " 0 px differ" $O/dbg_cornell.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread -k "chained or deferred_combine or async" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for sc in cornell34 blob70k; do
  for r in 8 1; do
    for ch in 0 3 8; do
      timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r 28=1 30=$ch > $O/${sc}_r${r}_chain${ch}.jsonl || exit 1
      echo "$sc r$r chain$ch $(cat $O/${sc}_r${r}_chain${ch}.jsonl)"
    done
  done
done
for ch in 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_r8_c$ch -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 30=$ch > $O/kt_r8_c$ch.jsonl 2>&1 || exit 1
done
