# r5p: the payload-queue wavefront's extend knobs re-swept on blob70k 1080p (wave threshold,
# fetch chunk, loop exits)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5p
mkdir -p $T
timeout -k 10 280 python tools/sweep.py --scene blob70k --steps 3 mode=1 wave=-1,16,48 chunk=64,256,1024 > $T/sweep_wave_chunk.txt 2>&1 && \
timeout -k 10 250 python tools/sweep.py --scene blob70k --steps 3 mode=1 leafexit=-1,8,24 nodeexit=-1,32 > $T/sweep_exits.txt 2>&1
echo "r5p rc=$?"
