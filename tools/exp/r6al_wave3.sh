# round 6: Cornell's wave threshold (automatic 24 for LDS scenes) against 28 / 32 on the whole image,
# three alternating passes, and the 1/8 shares at 24 and 32 -> gpurun_out/r6al/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6al
mkdir -p $O
for pass in 1 2 3; do
  for w in auto 28 32; do
    A=""; [ $w != auto ] && A="--wave-threshold $w"
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off $A > $O/cornell_w${w}_p$pass.json 2> $O/cornell_w${w}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/cornell_w${w}_p$pass.json'));print('cornell wave $w pass $pass', d['value'], d['ms_per_step'])"
  done
done
for w in auto 32; do
  A=""; [ $w != auto ] && A="2=$w"
  timeout -k 10 300 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 --all-bands 28=1 $A > $O/rehearsal_cornell_w$w.jsonl || exit 1
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/rehearsal_cornell_w$w.jsonl') if l.startswith('{')]
r8=[r for r in rows if r.get('ranks')==8 and 'rank' in r]
print('cornell share wave $w', max(r['ms_per_step'] for r in r8), min(r['efficiency'] for r in r8))"
done
echo WAVE3_DONE
