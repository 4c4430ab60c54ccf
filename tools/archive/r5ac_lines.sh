# round 5: the headline lines again with roofline.traffic from this library's committed profiles
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_cornell.json 2> $O/cornell.err || exit 1
timeout -k 10 300 python3 bench.py --scene blob70k --steps 20 --warmup 5 > $O/bench_blob.json 2> $O/blob.err || exit 1
cat $O/bench_cornell.json $O/bench_blob.json
