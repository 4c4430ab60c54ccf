# round 5: with group launches, does chaining pay for the Cornell whole image (automatic: off)?
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5af
mkdir -p $O
run() {  # name scene ranks opts...
  local name=$1 sc=$2 r=$3; shift 3
  timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for ch in 0 2 3 4; do
    run p${pass}_cornell_whole_c$ch cornell34 1 28=1 30=$ch
  done
  run p${pass}_cornell_half_c0 cornell34 2 28=1 30=0
  run p${pass}_cornell_half_auto cornell34 2 28=1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_whole_c3 -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 30=3 > /dev/null 2>&1 || exit 1
