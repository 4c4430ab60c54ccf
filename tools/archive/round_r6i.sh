# r6i: final round-3 state — full GPU suite, every bench line, rocprof kernel-trace + PMC profiles
# of the two headline workloads, legacy-ABI timing, 1/8-share rehearsal of both headline scenes
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6i
mkdir -p $T
bash tools/gpu_tests.sh r6i && bash tools/round3_bench.sh r6i && \
timeout -k 10 250 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,2,4,8 > $T/scaling_cornell.jsonl 2>&1 && \
timeout -k 10 300 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,2,4,8 > $T/scaling_blob.jsonl 2>&1
echo "r6i rc=$?"
