# round 6: the general megakernel's thresholds over a tree in global memory (random_scene, the
# reference app's scene; automatic 24 / 12 / 16) at the final library, bench.py A/B, two alternating
# passes -> gpurun_out/r6bf/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bf
mkdir -p $O
for pass in 1 2; do
  for e in auto 32_12_16 24_17_32 24_12_24 32_17_48 40_22_56; do
    A=""; [ $e != auto ] && { IFS=_ read w l n <<< "$e"; A="--wave-threshold $w --option LEAF_EXIT=$l --option NODE_EXIT=$n"; }
    timeout -k 10 200 python3 bench.py --scene random_scene --cpu-baseline off $A > $O/random_${e}_p$pass.json 2> $O/random_${e}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/random_${e}_p$pass.json'));print('random $e pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
  done
done
echo RANDOM_DONE
