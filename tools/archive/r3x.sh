# r3x: packed slab FMAs (v_pk_fma_f32 with the axis terms broadcast by op_sel) in the LDS-scene node visit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3x
timeout -k 10 300 bash tools/ab.sh cornell34 8 base pk > gpurun_out/r3x/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh cornell_mixed 6 base pk > gpurun_out/r3x/ab_mixed.txt 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_pk.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mesh_matches or general or camera_pool or full_size or lds" > gpurun_out/r3x/pytest_pk.log 2>&1
