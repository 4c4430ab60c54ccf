# r2w: float nodes + LDS top of the tree: stack cap vs top size (blob70k, random_scene)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2w
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 quant=0 stackcap=15,13,11,9,7,5 top=-1 > gpurun_out/r2w/blob.jsonl && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 quant=0 stackcap=13 top=21,40,52 > gpurun_out/r2w/blob_top.jsonl && \
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 stackcap=19,15,13,11,9 top=-1 > gpurun_out/r2w/random.jsonl
