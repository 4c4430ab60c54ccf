# round 5: where the share's per-segment rate goes — rate timelines (HIPPT_DEBUG_RATE build) of the
# whole image, one 1/8 share and 8 chained shares, chained and unchained kernels; the chain kernel
# without its per-round LDS segment count (A/B)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5k
mkdir -p $O
for ch in 0 8; do
  HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 200 python -u tools/rate_timeline.py --scene cornell34 \
      --jobs 1:64:1,8:64:1,8:64:8 --bucket-us 50 28=1 30=$ch > $O/rate_chain$ch.jsonl || exit 1
done
for lib in libhippt libv_nosegs; do
  for r in 8 1; do
    for ch in 0 3 8; do
      HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks $r 28=1 30=$ch > $O/${lib}_r${r}_chain${ch}.jsonl || exit 1
      echo "$lib r$r chain$ch $(cat $O/${lib}_r${r}_chain${ch}.jsonl)"
    done
  done
done
