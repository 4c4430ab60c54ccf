# round 6: the 1/8 Cornell share's launch sequence over longer bursts (36 steps, caps 8 and 4): is only
# the first group slow? -> gpurun_out/r6p/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6p
mkdir -p $O
for cap in 8 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_cap$cap -o run -- \
    python3 tools/band_scaling.py --scene cornell34 --steps 36 --ranks 8 28=1 30=$cap > $O/share8_cap$cap.jsonl 2> $O/share8_cap$cap.err || exit 1
  python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/kt_cap$cap/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
i=max(k for k,r in enumerate(rows) if r['Kernel_Name'].startswith('__amd_rocclr_fill'))
prev=None
for r in rows[i+1:]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    print('cap $cap', r['Kernel_Name'][:20], round((e-s)/1e6,3), round((s-prev)/1e3,1) if prev else 0)
    prev=e
PY
done
echo GROUPS_DONE
