# r3ap: SAH-optimal 4-wide collapse vs greedy on the leaf-2 trees (LDS scenes), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ap
S="timeout -k 10 300 python tools/sweep.py --steps 4"
$S --scene cornell34 collapse=0,1,0,1 > gpurun_out/r3ap/c.jsonl 2>&1 && \
$S --scene cornell_mixed collapse=0,1,0,1 > gpurun_out/r3ap/m.jsonl 2>&1 && \
$S --scene cornell34 collapse=1 leaf4=2,3,4,6 > gpurun_out/r3ap/c_leaf4.jsonl 2>&1
