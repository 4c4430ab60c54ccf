# r5n: the payload-queue wavefront — config 5 bench line, per-kernel times (rocprofv3 kernel
# trace) and the extend kernel's node format (8-bit vs float) re-measured
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=gpurun_out/r5n
mkdir -p $T
timeout -k 10 300 python bench.py --preset config5 --cpu-baseline off > $T/bench_config5.json 2> $T/bench_config5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $T/prof -o wf -- python3 bench.py --preset config5 --steps 3 --warmup 1 --cpu-baseline off > $T/bench_wf_prof.json 2> $T/bench_wf_prof.err && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 4 mode=1 quant=-1,0,-1,0 > $T/sweep_quant_wf.txt 2>&1
echo "r5n rc=$?"
