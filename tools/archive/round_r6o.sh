# r6o: random_scene (the reference app's scene) — item order on/off, stack cap, top nodes, chunk
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6o
mkdir -p $T
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 order=0,1,0,1 > $T/ab_order.txt 2>&1 && \
timeout -k 10 400 python tools/sweep.py --scene random_scene --steps 3 stackcap=8,10,13 chunk=256,512 > $T/sweep_cap_chunk.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene random_scene --steps 3 quant=0,1 > $T/sweep_quant.txt 2>&1
echo "r6o rc=$?"
