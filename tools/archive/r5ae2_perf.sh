# round 5: held batches launched as one group (MeshParams::chainGroup) — parity (chain_debug
# sequences with the decision trace, the chained GPU subset), then A/B against the previous library
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ae2
mkdir -p $O
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for lib in libhippt libv_prev; do
    run p${pass}_${lib}_cornell_share $lib cornell34 8 28=1
    run p${pass}_${lib}_cornell_quarter $lib cornell34 4 28=1
    run p${pass}_${lib}_blob_share $lib blob70k 8 28=1
    run p${pass}_${lib}_blob_whole $lib blob70k 1 28=1
    run p${pass}_${lib}_mixed_whole $lib cornell_mixed 1 28=1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_share -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 > /dev/null 2>&1 || exit 1
