# round 6: the chained-sequence fuzz over 256 seeds (every 8th at 320x180) on the exact final library
# -> gpurun_out/r6bi/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bi
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
HIPPT_FUZZ_SEEDS=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_fuzz.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/fuzz256.log 2>&1 || { tail -30 $O/fuzz256.log; exit 1; }
tail -2 $O/fuzz256.log
echo FUZZ_DONE
