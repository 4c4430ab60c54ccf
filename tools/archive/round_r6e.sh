# r6e: work chunk 256 vs 512, alternating, at full size and on the 1/8 share
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6e
mkdir -p $T
timeout -k 10 300 python tools/sweep.py --scene cornell34 --steps 6 chunk=256,512,256,512,256,512 > $T/ab_cornell.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 4 chunk=256,512,256,512 > $T/ab_blob.txt 2>&1 && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_256.jsonl 2>&1 && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 4=512 > $T/scaling_512.jsonl 2>&1
echo "r6e rc=$?"
