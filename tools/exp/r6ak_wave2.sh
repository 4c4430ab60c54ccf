# round 6: blob70k's wave threshold around 40 (whole image: auto = 32, 36, 40, 44, two alternating
# passes), configs[3] (4K/256 spp) and the 1/8 shares at auto and 40 -> gpurun_out/r6ak/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ak
mkdir -p $O
for pass in 1 2; do
  for w in auto 36 40 44; do
    A=""; [ $w != auto ] && A="--wave-threshold $w"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off $A > $O/blob_w${w}_p$pass.json 2> $O/blob_w${w}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_w${w}_p$pass.json'));print('blob70k wave $w pass $pass', d['value'], d['ms_per_step'])"
  done
done
for w in auto 40; do
  A=""; [ $w != auto ] && A="--wave-threshold $w"
  timeout -k 10 300 python3 bench.py --preset config4 --steps 5 --warmup 1 --cpu-baseline off $A > $O/blob4k_w$w.json 2> $O/blob4k_w$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/blob4k_w$w.json'));print('blob4k wave $w', d['value'], d['ms_per_step'])"
done
for w in auto 40; do
  A=""; [ $w != auto ] && A="2=$w"
  timeout -k 10 300 python -u tools/band_scaling.py --scene blob70k --steps 20 --ranks 1,8 --all-bands 28=1 $A > $O/rehearsal_blob_w$w.jsonl || exit 1
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/rehearsal_blob_w$w.jsonl') if l.startswith('{')]
r8=[r for r in rows if r.get('ranks')==8 and 'rank' in r]
print('blob share wave $w', max(r['ms_per_step'] for r in r8), min(r['efficiency'] for r in r8))"
done
echo WAVE2_DONE
