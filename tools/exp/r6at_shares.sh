# round 6: blob70k's 1/8 and 1/4 row shares (chained, 2^24-sample batches, automatic 32 / 17 / 48) with
# the big-batch thresholds and mixes (band_scaling, every rank, 20 steps) -> gpurun_out/r6at/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6at
mkdir -p $O
for pass in 1 2; do
  for e in auto 40_22_56 32_22_56 36_20_52 40_17_48; do
    A=""; [ $e != auto ] && { IFS=_ read w l n <<< "$e"; A="2=$w 14=$l 15=$n"; }
    timeout -k 10 300 python -u tools/band_scaling.py --scene blob70k --steps 20 --ranks 4,8 --all-bands 28=1 $A > $O/share_${e}_p$pass.jsonl || exit 1
    python3 -c "
import json
rows=[json.loads(l) for l in open('$O/share_${e}_p$pass.jsonl') if l.startswith('{')]
for n in (4,8):
    r=[x for x in rows if x.get('ranks')==n and 'rank' in x]
    print('blob share $e pass $pass N', n, max(x['ms_per_step'] for x in r))"
  done
done
echo SHARES_DONE
