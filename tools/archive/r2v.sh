# r2v: float (128 B) vs 8-bit (64 B) nodes for blob70k with the LDS top of the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2v
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 quant=0,1 stackcap=19,13 top=0,-1 > gpurun_out/r2v/blob.jsonl
