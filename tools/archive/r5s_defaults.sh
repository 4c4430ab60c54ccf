# round 5: defaults — claim size 512 against 256 chained and unchained on the four scenes (whole
# image and 1/8 share), the non-temporal radiance store (blob70k's DRAM writes), and the rate probe
# of the small batch's interior phase (r5q)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s
mkdir -p $O
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for sc in cornell34 blob70k random_scene cornell_mixed; do
  for ck in 256 512; do
    run ${sc}_whole_c0_k$ck libhippt $sc 1 28=1 30=0 4=$ck
    run ${sc}_whole_c3_k$ck libhippt $sc 1 28=1 30=3 4=$ck
    run ${sc}_share_c0_k$ck libhippt $sc 8 28=1 30=0 4=$ck
    run ${sc}_share_c8_k$ck libhippt $sc 8 28=1 30=8 4=$ck
    run ${sc}_half_c0_k$ck libhippt $sc 2 28=1 30=0 4=$ck
    run ${sc}_half_c6_k$ck libhippt $sc 2 28=1 30=6 4=$ck
  done
done
for lib in libhippt libv_ntrad; do
  run blob_whole_$lib $lib blob70k 1 28=1 30=0
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_$lib -o run -- \
      python3 tools/band_scaling.py --scene blob70k --steps 3 --ranks 1 28=1 30=0 > /dev/null 2>&1 || exit 1
done
bash tools/exp/r5q_rate2.sh
