# round 6: automatic chain cap up to 16 (libv_cap16.so) against 8 (default): chained GPU subset on the
# variant, then the 1/8 and 1/4 shares (every rank) of Cornell and blob70k, two alternating passes,
# and the 1/8 Cornell share's launch sequence under the variant -> gpurun_out/r6n/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6n
mkdir -p $O
V=qt-raytracer_amd/libv_cap16.so
HIPPT_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "(chain or deferred or held or closes) and not automatic_chain" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pass in 1 2; do
  for lib in default cap16; do
    if [ $lib = cap16 ]; then export HIPPT_LIB=$V; else unset HIPPT_LIB; fi
    for sc in cornell34 blob70k; do
      for n in 8 4; do
        timeout -k 10 200 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $n --all-bands 28=1 > $O/share${n}_${sc}_${lib}_p$pass.jsonl || exit 1
        python3 -c "import json;rs=[json.loads(l) for l in open('$O/share${n}_${sc}_${lib}_p$pass.jsonl')];print('share $n $sc $lib $pass', max(r['ms_per_step'] for r in rs))"
      done
    done
  done
done
export HIPPT_LIB=$V
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_cornell34 -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 > $O/share8_trace.jsonl 2> $O/share8_trace.err || exit 1
echo CAP16_DONE
