# r5x: Cornell knobs re-swept under the sample-length order (chunk, wave threshold, loop exits)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5x
mkdir -p $T
timeout -k 10 280 python tools/sweep.py --scene cornell34 --steps 5 chunk=128,256,512 wave=12,16,20 > $T/sweep_chunk_wave.txt 2>&1 && \
timeout -k 10 250 python tools/sweep.py --scene cornell34 --steps 5 leafexit=2,4,8 nodeexit=40,48,56 > $T/sweep_exits.txt 2>&1
echo "r5x rc=$?"
