# round 6: the default bench line with the CPU baseline's independent-process figure (the reference's
# threads against the same sample split over separate 1-thread processes) -> gpurun_out/r6x/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/bench_cornell.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_cornell.json'));c=d['cpu_baseline'];print(d['value'], c['value'], c['runs'], c.get('per_thread'), c.get('independent_processes'))"
echo CPU_DONE
