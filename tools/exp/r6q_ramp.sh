# round 6: is the share burst's slow start a clock/power ramp?  The whole image's 20-step burst after
# one warmup step and a sync (Cornell, unchained), and the 1/8 share's 36-step burst at cap 4 after a
# 2-second idle -> gpurun_out/r6q/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6q
mkdir -p $O
show() {
  python3 - "$1" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
i=max(k for k,r in enumerate(rows) if r['Kernel_Name'].startswith('__amd_rocclr_fill'))
print(' '.join(f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6:.3f}" for r in rows[i+1:] if r['Kernel_Name'].startswith('mesh')))
PY
}
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_whole -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 > $O/whole.jsonl 2> $O/whole.err || exit 1
echo whole; show $O/kt_whole/run_kernel_trace.csv
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_share -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 36 --ranks 8 28=1 30=4 > $O/share.jsonl 2> $O/share.err || exit 1
echo share cap4; show $O/kt_share/run_kernel_trace.csv
echo RAMP_DONE
