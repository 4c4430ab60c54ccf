# r2zb: SAH-optimal 4-wide collapse (node cost x leaf size) vs the greedy collapse
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2zb
timeout -k 10 300 python tools/sweep.py --scene cornell34 --steps 3 --count collapse=1 ncost=100,150,200,300,400 leaf4=4,8,15 > gpurun_out/r2zb/cornell.jsonl && \
timeout -k 10 60 python tools/sweep.py --scene cornell34 --steps 3 --count collapse=0 > gpurun_out/r2zb/cornell0.jsonl && \
timeout -k 10 400 python tools/sweep.py --scene blob70k --steps 2 --count collapse=1 ncost=100,200,300 leaf4=4,8 > gpurun_out/r2zb/blob.jsonl && \
timeout -k 10 60 python tools/sweep.py --scene blob70k --steps 2 --count collapse=0 > gpurun_out/r2zb/blob0.jsonl
