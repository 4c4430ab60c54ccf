# r6q: final state after packed keys in the general kernel and the camera pool for the
# Lambertian kernel over global trees — full GPU suite, every bench line, profiles, 1/8 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6q
mkdir -p $T
timeout -k 10 60 tools/micro/ta_cost > $T/ta_cost.txt 2>&1 && bash tools/gpu_tests.sh r6q && bash tools/round3_bench.sh r6q && \
timeout -k 10 250 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,2,4,8 > $T/scaling_cornell.jsonl 2>&1 && \
timeout -k 10 300 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,2,4,8 > $T/scaling_blob.jsonl 2>&1
echo "r6q rc=$?"
