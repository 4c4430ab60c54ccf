# r5l: per-kernel times of the wavefront step (config 5) from a rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=gpurun_out/r5l
mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o wf -- python3 bench.py --preset config5 --steps 3 --warmup 1 --cpu-baseline off > $T/bench_wf.json 2> $T/bench_wf.err
echo "r5l rc=$?"
find $T/prof -name "*kernel_stats.csv" | head -3
