# r6v: packed-FMA (v_pk_fma_f32) child keys in the LDS-resident kernels — parity subset + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6v
mkdir -p $T
HIPPT_LIB=qt-raytracer_amd/libv_pk1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "parity or mixed or fuzz or headline" > $T/pytest_pk1.log 2>&1 && \
timeout -k 10 400 bash tools/ab.sh cornell34 5 pk0 pk1 > $T/ab_pk_cornell.txt 2>&1 && \
timeout -k 10 400 bash tools/ab.sh cornell_mixed 4 pk0 pk1 > $T/ab_pk_mixed.txt 2>&1
echo "r6v rc=$?"
