# round 5: the share's per-batch deficit inside a chained launch — claim sizes (chunk, tail chunk)
# and the item order, Cornell 1/8 share chained (cap 8) and unchained, whole image unchained
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5m
mkdir -p $O
run() {  # name lib ranks opts...
  local name=$1 lib=$2 r=$3; shift 3
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for ck in 256 512 1024; do
  run share_c8_chunk$ck libhippt 8 28=1 30=8 4=$ck
  run share_c0_chunk$ck libhippt 8 28=1 30=0 4=$ck
  run whole_c0_chunk$ck libhippt 1 28=1 30=0 4=$ck
done
run share_c8_order0 libhippt 8 28=0 30=8
run share_c0_order0 libhippt 8 28=0 30=0
run whole_c0_order0 libhippt 1 28=0 30=0
run share_c8_tail256 libv_tail256 8 28=1 30=8
run share_c0_tail256 libv_tail256 8 28=1 30=0
run whole_c0_tail256 libv_tail256 1 28=1 30=0
