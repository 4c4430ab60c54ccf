# round 6: blob70k's wave threshold 40 / 48 against the automatic one (r6ad's sweep: 40 +0.5%), the
# bench's own timing, three alternating passes -> gpurun_out/r6aj/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6aj
mkdir -p $O
for pass in 1 2 3; do
  for w in auto 40 48; do
    A=""; [ $w != auto ] && A="--wave-threshold $w"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off $A > $O/blob_w${w}_p$pass.json 2> $O/blob_w${w}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_w${w}_p$pass.json'));print('blob70k wave $w pass $pass', d['value'], d['ms_per_step'], d['config']['wave_threshold'], d['config'].get('image_crc32'))"
  done
done
echo WAVE_DONE
