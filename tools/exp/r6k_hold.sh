# round 6: hold the batches that arrive while the run's first launch runs (default) against the
# round-5 rule (libv_nohold.so): chained GPU subset first, then the 1/8 shares (every rank) and the
# chained whole images, two alternating passes, and the share burst's kernel trace -> gpurun_out/r6k/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chain or deferred or held or closes" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=qt-raytracer_amd/libv_nohold.so
for pass in 1 2; do
  for lib in default nohold; do
    if [ $lib = nohold ]; then export HIPPT_LIB=$V; else unset HIPPT_LIB; fi
    for sc in cornell34 blob70k; do
      timeout -k 10 200 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 8 --all-bands 28=1 > $O/share8_${sc}_${lib}_p$pass.jsonl || exit 1
      python3 -c "import json;rs=[json.loads(l) for l in open('$O/share8_${sc}_${lib}_p$pass.jsonl')];print('share8 $sc $lib $pass', max(r['ms_per_step'] for r in rs))"
    done
    for sc in blob70k cornell_mixed; do
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off > $O/bench_${sc}_${lib}_p$pass.json 2> $O/bench_${sc}_${lib}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/bench_${sc}_${lib}_p$pass.json'));print('bench $sc $lib $pass', d['value'], d['ms_per_step'])"
    done
  done
done
unset HIPPT_LIB
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_cornell34 -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 > $O/share8_trace.jsonl 2> $O/share8_trace.err || exit 1
echo HOLD_DONE
