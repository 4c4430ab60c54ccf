# r3ab: wavefront — wf_shade/wf_generate write whole 64-byte slot records (no partial lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ab
for pass in 1 2; do for v in base full; do
  printf '%s pass%s ' $v $pass
  HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 mode=1 || exit 1
done; done > gpurun_out/r3ab/ab.txt 2>&1 && \
true
