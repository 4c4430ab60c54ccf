# round 5: static first chunks off (every claim dynamic) — Cornell/blob whole and 1/8 share,
# chained and unchained, kernel traces of the chained share; rate timelines
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5t
mkdir -p $O
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
for lib in libhippt libv_nostatic; do
  run p${pass}_${lib}_cornell_whole_c0 $lib cornell34 1 28=1 30=0
  run p${pass}_${lib}_cornell_share_c0 $lib cornell34 8 28=1 30=0
  run p${pass}_${lib}_cornell_share_c8 $lib cornell34 8 28=1 30=8
  run p${pass}_${lib}_blob_whole_c0 $lib blob70k 1 28=1 30=0
  run p${pass}_${lib}_blob_share_c0 $lib blob70k 8 28=1 30=0
  run p${pass}_${lib}_blob_share_c8 $lib blob70k 8 28=1 30=8
done
done
HIPPT_LIB=qt-raytracer_amd/libv_nostatic.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_share_c8_nostatic -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 30=8 > /dev/null 2>&1 || exit 1
