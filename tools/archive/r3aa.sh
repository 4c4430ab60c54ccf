# r3aa: wavefront — scattered rays appended grouped by direction octant within each 1024-ray block
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aa
for pass in 1 2; do for v in base wfsort; do
  printf '%s pass%s ' $v $pass
  HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 mode=1 || exit 1
done; done > gpurun_out/r3aa/ab.txt 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_wfsort.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k wavefront > gpurun_out/r3aa/pytest.log 2>&1
