# round 5: headline lines with roofline.traffic (profiles of this library committed), 20 steps as the
# driver runs them; then the wave-threshold sweep
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_cornell_20.json 2> $O/cornell.err || exit 1
cat $O/bench_cornell_20.json
timeout -k 10 300 python3 bench.py --scene blob70k --steps 20 --warmup 5 > $O/bench_blob_20.json 2> $O/blob.err || exit 1
bash tools/exp/r5z_thr.sh
