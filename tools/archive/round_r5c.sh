# r5c: GPU suite with the 40-byte triangle records; their A/B on blob70k (1080p and 4K) and the
# leaf/node loop exits re-swept with them
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5c
mkdir -p $T
bash tools/gpu_tests.sh r5c && \
timeout -k 10 150 python tools/sweep.py --scene blob70k --steps 5 tris40=1,0,1,0 > $T/ab_tris40_blob.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --width 3840 --height 2160 --spp 16 --steps 3 tris40=1,0,1,0 > $T/ab_tris40_blob4k.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 leafexit=13,17,21 nodeexit=40,48,56 > $T/sweep_exits_blob.txt 2>&1 && \
timeout -k 10 150 python tools/sweep.py --scene random_scene --steps 5 tris40=1,0,1,0 > $T/ab_tris40_random.txt 2>&1
echo "r5c rc=$?"
