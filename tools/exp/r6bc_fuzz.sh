# round 6: the chained-sequence fuzz with every 8th sequence at 320x180 (long launches), 128 seeds
# -> gpurun_out/r6bc/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bc
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
HIPPT_FUZZ_SEEDS=128 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_fuzz.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/fuzz128.log 2>&1 || { tail -30 $O/fuzz128.log; exit 1; }
tail -2 $O/fuzz128.log
echo FUZZ_DONE
