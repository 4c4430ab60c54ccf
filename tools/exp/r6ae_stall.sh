# round 6: the sweep's slow settings, every host call timed (tools/exp/r6ae_stall.py) -> gpurun_out/r6ae/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ae
mkdir -p $O
REPS=4 timeout -k 10 400 python3 -u tools/exp/r6ae_stall.py blob70k > $O/stall_blob.jsonl 2> $O/stall_blob.err || { tail -20 $O/stall_blob.err; exit 1; }
python3 -c "
import json
for l in open('$O/stall_blob.jsonl'):
    d=json.loads(l)
    if d['slow'] or d['msamples_s'] < 15000: print(d['rep'], d['leafexit'], d['nodeexit'], d['msamples_s'], d['trace_ms_step'], d['slow'])
"
echo STALL_DONE
