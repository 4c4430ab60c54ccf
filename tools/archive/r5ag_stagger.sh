# round 5: why a run's first launch is slower — its waves start together (no combine to stagger them)?
# The would-be combine waves held back 50 / 300 us when there is nothing to combine (experiment)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ag
mkdir -p $O
for lib in libhippt libv_st50 libv_st300; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$lib -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 30=3 > $O/$lib.jsonl 2>&1 || exit 1
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ktu_$lib -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 30=0 > $O/u_$lib.jsonl 2>&1 || exit 1
done
