# round 6: cap 8 for whole images (r6aw: Cornell chained at 8 +0.5% over unchained, blob70k 8 +0.5% over
# 3) on the general-kernel scenes and again on the headline ones; bench.py A/B, two alternating passes
# -> gpurun_out/r6ax/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ax
mkdir -p $O
for pass in 1 2; do
  for sc in random_scene cornell_mixed cornell34 blob70k; do
    for c in auto 8; do
      A=""; [ $c != auto ] && A="--option CHAIN=$c"
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off $A > $O/${sc}_c${c}_p$pass.json 2> $O/${sc}_c${c}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${sc}_c${c}_p$pass.json'));print('$sc chain $c pass $pass', d['value'], d['ms_per_step'], d['config']['chain']['applied_cap'], d['config'].get('image_crc32'))"
    done
  done
done
echo CAP2_DONE
