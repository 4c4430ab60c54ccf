# round 6: the seconds-long host calls after a re-initialization (r6ae), under the HIP runtime trace:
# which runtime call takes the time -> gpurun_out/r6af/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6af
mkdir -p $O
REPS=4 timeout -k 10 500 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/tr -o run -- \
  python3 -u tools/exp/r6ae_stall.py blob70k > $O/stall_blob.jsonl 2> $O/stall_blob.err || { tail -20 $O/stall_blob.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections, json
O = "gpurun_out/r6af"
api = glob.glob(f"{O}/tr/**/run_hip_api_trace.csv", recursive=True)
kt = glob.glob(f"{O}/tr/**/run_kernel_trace.csv", recursive=True)
out = {}
for path, key in ((api, "Function"), (kt, "Kernel_Name")):
    if not path: continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path[0])):
        agg[r[key]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    top = sorted(((max(v), k, len(v), sum(v)) for k, v in agg.items()), reverse=True)[:15]
    out[key] = [{"name": k[:60], "max_ms": round(m, 2), "calls": n, "total_ms": round(t, 1)} for m, k, n, t in top]
print(json.dumps(out, indent=1))
json.dump(out, open(f"{O}/top_calls.json", "w"), indent=1)
PY
python3 -c "
import json
for l in open('gpurun_out/r6af/stall_blob.jsonl'):
    d=json.loads(l)
    if any(x['s']>1 for x in d['slow']): print(d['rep'], d['leafexit'], d['nodeexit'], d['slow'])
"
echo TRACE_DONE
