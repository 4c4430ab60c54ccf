# round 5: where the chained launches' time goes — rocprofv3 kernel traces of 20 chained steps
# (1/8 Cornell share at cap 8; whole Cornell image automatic), chain off for reference
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5d
for cfg in "8 30=8" "8 30=0" "1 30=-1" "1 30=0"; do
  set -- $cfg
  tag=r${1}_$(echo $2 | tr '=' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r5d/$tag -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks $1 28=1 $2 > gpurun_out/r5d/$tag.jsonl 2> gpurun_out/r5d/$tag.err || exit 1
  cat gpurun_out/r5d/$tag.jsonl
done
