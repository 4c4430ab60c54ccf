# round 5: claim size for chained 1/8 shares (automatic: 256), three alternating passes
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ab
mkdir -p $O
run() {  # name scene ranks opts...
  local name=$1 sc=$2 r=$3; shift 3
  timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2 3; do
  for ck in 256 384 512; do
    run p${pass}_cornell_share_k$ck cornell34 8 28=1 4=$ck
    run p${pass}_blob_share_k$ck blob70k 8 28=1 4=$ck
    run p${pass}_mixed_share_k$ck cornell_mixed 8 28=1 4=$ck
  done
done
