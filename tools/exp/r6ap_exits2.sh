# round 6: blob70k's wave threshold x leaf exit x node exit around (40, 22, 56) (r6ao: +1.6% over the
# defaults 40/17/48): bench.py A/B, three alternating passes -> gpurun_out/r6ap/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ap
mkdir -p $O
for pass in 1 2 3; do
  for e in 40_22_56 40_22_64 40_24_64 40_26_64 40_28_64 44_22_56 44_24_64 48_24_64; do
    IFS=_ read w l n <<< "$e"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off --wave-threshold $w --option LEAF_EXIT=$l --option NODE_EXIT=$n > $O/blob_${e}_p$pass.json 2> $O/blob_${e}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_${e}_p$pass.json'));print('blob70k $e pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
  done
done
echo EXITS2_DONE
