# round 6: the item order's pixel tiles on the final library's chained whole images (cap 8): automatic
# (8x8) against rows and 16x4, Cornell and blob70k, two alternating passes -> gpurun_out/r6bd/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bd
mkdir -p $O
for pass in 1 2; do
  for sc in cornell34 blob70k; do
    for t in auto 0 16; do
      A=""; [ $t != auto ] && A="--option PIXEL_TILE=$t"
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off $A > $O/${sc}_t${t}_p$pass.json 2> $O/${sc}_t${t}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${sc}_t${t}_p$pass.json'));print('$sc tile $t pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
    done
  done
done
echo TILE_DONE
