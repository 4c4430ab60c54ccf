# round 5: the tail claim size under 512-item claims (HIPPT_TAIL_CHUNK 64 default / 128 / 256), three
# alternating passes, Cornell whole image and 1/8 share (chained), blob70k whole
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ak
mkdir -p $O
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2 3; do
  for lib in libhippt libv_tail128 libv_tail256; do
    run p${pass}_${lib}_cornell_whole $lib cornell34 1 28=1
    run p${pass}_${lib}_cornell_share $lib cornell34 8 28=1
    run p${pass}_${lib}_blob_whole $lib blob70k 1 28=1
  done
done
