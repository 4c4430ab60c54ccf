# r3aq: SAH-optimal collapse vs greedy on the leaf-2 trees, global-memory scenes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aq
S="timeout -k 10 300 python tools/sweep.py --steps 3"
$S --scene blob70k collapse=0,1,0,1 > gpurun_out/r3aq/b.jsonl 2>&1 && \
$S --scene random_scene collapse=0,1,0,1 > gpurun_out/r3aq/r.jsonl 2>&1 && \
$S --scene cornell34 collapse=0,1,0,1 > gpurun_out/r3aq/c.jsonl 2>&1
