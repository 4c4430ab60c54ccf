# round 5: block-level drained-queue words (queue_fetch skips a queue a wave of its block found
# drained): parity subset, chained/unchained A/B against the build without them for unchained
# kernels, and the chained share's rate timeline
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 200 python -u tools/exp/chain_debug.py cornell34 > $O/dbg_cornell.txt 2>&1 || { cat $O/dbg_cornell.txt; exit 1; }
grep -c " 0 px differ" $O/dbg_cornell.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread -k "chained or deferred_combine or async or pool" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 200 python -u tools/rate_timeline.py --scene cornell34 \
    --jobs 1:64:1,8:64:8 --bucket-us 50 28=1 30=8 > $O/rate_chain8.jsonl || exit 1
for sc in cornell34 blob70k; do
  for lib in libhippt libv_nodrain; do
    for r in 8 1; do
      for ch in 0 8; do
        HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r 28=1 30=$ch > $O/${sc}_${lib}_r${r}_chain${ch}.jsonl || exit 1
        echo "$sc $lib r$r chain$ch $(cat $O/${sc}_${lib}_r${r}_chain${ch}.jsonl)"
      done
    done
  done
done
