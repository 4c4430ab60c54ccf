# round 6: configs[3]'s row shares (4K, 256 spp, blob70k) on the final library: the one-GPU rehearsal
# of every rank's share at N = 1, 2, 4, 8 -> gpurun_out/r6bh/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bh
mkdir -p $O
timeout -k 10 600 python -u tools/band_scaling.py --scene blob70k --width 3840 --height 2160 --spp 256 --steps 5 --ranks 1,2,4,8 --all-bands 28=1 > $O/rehearsal_4k.jsonl || exit 1
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/rehearsal_4k.jsonl') if l.startswith('{')]
for n in (1,2,4,8):
    r=[x for x in rows if x.get('ranks')==n and 'rank' in x]
    print(n, max(x['ms_per_step'] for x in r), min(x['efficiency'] for x in r))"
echo R4K_DONE
