# r6c: loop exits re-swept for trees in global memory (blob70k, random_scene) under the item order
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6c
mkdir -p $T
timeout -k 10 500 python tools/sweep.py --scene blob70k --steps 3 leafexit=12,17,24 nodeexit=16,32,48 wave=28,32,36 > $T/sweep_blob.txt 2>&1 && \
timeout -k 10 400 python tools/sweep.py --scene random_scene --steps 3 leafexit=8,12,17 nodeexit=16,48 wave=24,32 > $T/sweep_random.txt 2>&1
echo "r6c rc=$?"
