# r3as: SAH-optimal collapse node cost (LDS scenes), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3as
S="timeout -k 10 300 python tools/sweep.py --steps 4"
$S --scene cornell34 ncost=200,100,300,450,200,100,300,450 > gpurun_out/r3as/c.jsonl 2>&1 && \
$S --scene cornell_mixed ncost=200,100,300,450,200,100,300,450 > gpurun_out/r3as/m.jsonl 2>&1
