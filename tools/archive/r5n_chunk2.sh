# round 5: claim size sweep (HIPPT_OPT_CHUNK) around 512, two passes, Cornell and blob70k, whole image
# unchained and chained, 1/8 share chained
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5n
mkdir -p $O
run() {  # name scene ranks opts...
  local name=$1 sc=$2 r=$3; shift 3
  timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for ck in 256 384 512 768; do
    run p${pass}_cornell_whole_c0_chunk$ck cornell34 1 28=1 30=0 4=$ck
    run p${pass}_cornell_whole_c3_chunk$ck cornell34 1 28=1 30=3 4=$ck
    run p${pass}_cornell_share_c8_chunk$ck cornell34 8 28=1 30=8 4=$ck
  done
done
for ck in 256 512; do
  run blob_whole_c0_chunk$ck blob70k 1 28=1 30=0 4=$ck
  run blob_whole_c3_chunk$ck blob70k 1 28=1 30=3 4=$ck
  run blob_share_c8_chunk$ck blob70k 8 28=1 30=8 4=$ck
  run blob_share_c0_chunk$ck blob70k 8 28=1 30=0 4=$ck
done
