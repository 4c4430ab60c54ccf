# round 6: with the clock prewarm (bench.py / band_scaling --prewarm-ms 200): the whole image's and the
# 1/8 share's launch durations, the rehearsal (every rank), and the bench lines at N = 1, 2, 4
# (the N > 1 ones on the one GPU) -> gpurun_out/r6r/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6r
mkdir -p $O
show() {
  python3 - "$1" "$2" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
m=[r for r in rows if r['Kernel_Name'].startswith('mesh')]
print(' '.join(f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6:.3f}" for r in m[-int(sys.argv[2]):]))
PY
}
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_whole -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1 28=1 > $O/whole.jsonl 2> $O/whole.err || exit 1
echo whole; show $O/kt_whole/run_kernel_trace.csv 22
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_share -o run -- \
  python3 tools/band_scaling.py --scene cornell34 --steps 36 --ranks 8 28=1 30=4 > $O/share.jsonl 2> $O/share.err || exit 1
echo share cap4; show $O/kt_share/run_kernel_trace.csv 11
for sc in cornell34 blob70k; do
  timeout -k 10 300 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,2,4,8 --all-bands 28=1 > $O/rehearsal_$sc.jsonl || exit 1
  python3 - <<PY
import json
rows=[json.loads(l) for l in open('$O/rehearsal_$sc.jsonl') if l.strip().startswith('{')]
by={}
for r in rows: by.setdefault(r['ranks'],[]).append(r)
full=by[1][0]['ms_per_step']
print('$sc', ' '.join(f"N={n}: {max(r['ms_per_step'] for r in rs):.3f} eff {full/n/max(r['ms_per_step'] for r in rs):.3f}" for n,rs in sorted(by.items())))
PY
done
for n in 1 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 --cpu-baseline off > $O/bench_${n}.json 2> $O/bench_${n}.err || { tail -20 $O/bench_${n}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_${n}.json').read().strip().splitlines()[-1]);print('bench', $n, d['value'], d['ms_per_step'], d['config'].get('image_crc32'), d['prewarm'])"
done
echo PREWARM_DONE
