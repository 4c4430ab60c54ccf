# round 5: the whole-image claim size around 512 (Cornell unchained, two passes), and the general
# kernel's whole image chained (cornell_mixed) against one launch per batch
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5x
mkdir -p $O
run() {  # name scene ranks opts...
  local name=$1 sc=$2 r=$3; shift 3
  timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for ck in 256 384 448 512 576 640 768; do
    run p${pass}_cornell_whole_k$ck cornell34 1 28=1 30=0 4=$ck
  done
  run p${pass}_mixed_whole_c0 cornell_mixed 1 28=1 30=0
  run p${pass}_mixed_whole_c3 cornell_mixed 1 28=1 30=3
  run p${pass}_blob_whole_c3_k256 blob70k 1 28=1 30=3 4=256
  run p${pass}_blob_whole_c3_k512 blob70k 1 28=1 30=3 4=512
done
