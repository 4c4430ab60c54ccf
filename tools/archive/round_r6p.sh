# r6p: packed child keys in the general kernel (cornell_mixed) re-tried under the current exits
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6p
mkdir -p $T
V=qt-raytracer_amd/libv_pfull.so
HIPPT_LIB=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed or fuzz or materials" > $T/pytest_pfull.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 100 python tools/sweep.py --scene cornell_mixed --steps 4 pool=-1 >> $T/ab_mixed.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell_mixed --steps 4 pool=-1 >> $T/ab_mixed.txt 2>&1 || exit 1
done
echo "r6p rc=$?"
