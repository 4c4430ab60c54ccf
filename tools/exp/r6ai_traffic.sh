# round 6: the final library's headline lines with the committed r6ah profiles in place (roofline.traffic
# filled from profiles/pmc_summary.json and profiles/round6/*_r6ah_pmc.json) -> gpurun_out/r6ai/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/cornell.err || exit 1
timeout -k 10 400 python3 bench.py --scene blob70k --cpu-baseline off > $O/bench_blob.json 2> $O/blob.err || exit 1
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['frac'], r['traffic'], r.get('limiter'), r.get('pmc_refused'))"; done
echo TRAFFIC_DONE
