# round 5: the wave threshold (HIPPT_OPT_WAVE_THRESHOLD) for the Cornell whole image under 512-item
# claims, and the leaf/node exits around their defaults (two passes)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z
mkdir -p $O
run() {  # name scene ranks opts...
  local name=$1 sc=$2 r=$3; shift 3
  timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for thr in 16 20 24 28 32; do
    run p${pass}_cornell_thr$thr cornell34 1 28=1 2=$thr
  done
  for le in 8 16; do run p${pass}_cornell_leaf$le cornell34 1 28=1 14=$le; done
  for ne in 4 12; do run p${pass}_cornell_node$ne cornell34 1 28=1 15=$ne; done
  for thr in 16 32; do run p${pass}_share_thr$thr cornell34 8 28=1 2=$thr; done
  run p${pass}_share_thr24 cornell34 8 28=1 2=24
done
