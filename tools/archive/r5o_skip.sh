# round 5: chained batches without combine-only launches (chain_batch skips the launch of a batch the
# run's not-yet-started last launch will take; a catch-up launch when a run closes) — parity, caps,
# A/B against the build without the skip, kernel traces
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 200 python -u tools/exp/chain_debug.py cornell34 > $O/dbg_cornell.txt 2>&1 || { cat $O/dbg_cornell.txt; exit 1; }
grep -c " 0 px differ" $O/dbg_cornell.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread -k "chained or deferred_combine or async or pool or skipped" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for lib in libhippt libv_noskip; do
  run ${lib}_cornell_share_c0 $lib cornell34 8 28=1 30=0
  run ${lib}_cornell_share_c8 $lib cornell34 8 28=1 30=8
  run ${lib}_cornell_share_c8_k512 $lib cornell34 8 28=1 30=8 4=512
  run ${lib}_cornell_whole_c0 $lib cornell34 1 28=1 30=0
  run ${lib}_cornell_whole_c2 $lib cornell34 1 28=1 30=2
  run ${lib}_cornell_whole_c3 $lib cornell34 1 28=1 30=3
  run ${lib}_cornell_whole_c3_k512 $lib cornell34 1 28=1 30=3 4=512
  run ${lib}_blob_share_c8 $lib blob70k 8 28=1 30=8
  run ${lib}_blob_whole_c3 $lib blob70k 1 28=1 30=3
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_share_c8 -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 30=8 > $O/kt_share_c8.jsonl 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_whole_c3 -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 30=3 > $O/kt_whole_c3.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/micro/wf_sort_cost > $O/wf_sort_cost.jsonl || exit 1
cat $O/wf_sort_cost.jsonl
