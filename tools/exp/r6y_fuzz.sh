# round 6: the chained-sequence fuzz over 256 seeds (pattern breaks now drawn), then the default bench
# line (CPU baseline with independent processes, median of 3) -> gpurun_out/r6y/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6y
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
HIPPT_FUZZ_SEEDS=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_fuzz.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/fuzz256.log 2>&1 || { tail -30 $O/fuzz256.log; exit 1; }
tail -2 $O/fuzz256.log
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/bench_cornell.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_cornell.json'));c=d['cpu_baseline'];print(d['value'], c['value'], c.get('per_thread'), c.get('independent_processes'))"
echo FUZZ_DONE
