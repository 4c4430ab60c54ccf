# round 6: kept work buffers across re-initialization (State::spare): the GPU suite on the new library,
# then the re-initialization sequence of r6ae with every host call timed -> gpurun_out/r6ag/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ag
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
bash tools/gpu_tests.sh r6ag || exit 1
REPS=4 timeout -k 10 400 python3 -u tools/exp/r6ae_stall.py blob70k > $O/stall_blob.jsonl 2> $O/stall_blob.err || { tail -20 $O/stall_blob.err; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/stall_blob.jsonl')]
print('settings', len(rows), 'max call s', max(max(d['call_ms']) for d in rows)/1e3, 'slow', [ (d['rep'],d['leafexit'],d['nodeexit'],d['slow']) for d in rows if any(x['s']>0.2 for x in d['slow'])])
print('initialize ms', sorted(d['call_ms'][0] for d in rows)[-5:], 'first async ms', sorted(d['call_ms'][2] for d in rows)[-5:])
"
echo SPARE_DONE
