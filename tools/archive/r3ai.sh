# r3ai: builder re-sweep around the new leaf default (leaf 1/2, SAH traversal cost), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ai
S="timeout -k 10 300 python tools/sweep.py --steps 4"
$S --scene blob70k leaf=2,1,2,1 > gpurun_out/r3ai/b_leaf1.jsonl 2>&1 && \
$S --scene blob70k tcost=100,70,140,100,70,140 > gpurun_out/r3ai/b_tcost.jsonl 2>&1 && \
$S --scene cornell34 leaf=2,1,2,1 > gpurun_out/r3ai/c_leaf1.jsonl 2>&1 && \
$S --scene cornell34 tcost=100,70,140,100,70,140 > gpurun_out/r3ai/c_tcost.jsonl 2>&1
