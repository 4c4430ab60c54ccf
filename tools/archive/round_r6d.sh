# r6d: build and layout knobs re-swept under the new loop exits and item order
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6d
mkdir -p $T
timeout -k 10 400 python tools/sweep.py --scene cornell34 --steps 5 ncost=100,200,300 leaf4=2,4 > $T/sweep_cornell_build.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene cornell34 --steps 5 chunk=256,512,1024 > $T/sweep_cornell_chunk.txt 2>&1 && \
timeout -k 10 400 python tools/sweep.py --scene blob70k --steps 3 stackcap=8,10,13 chunk=256,512 > $T/sweep_blob_cap_chunk.txt 2>&1
echo "r6d rc=$?"
