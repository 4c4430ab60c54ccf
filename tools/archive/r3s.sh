# r3s: wavefront extend knobs after the launch trims: node format (float vs 8-bit), wave threshold, stack cap
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3s
S="timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3"
$S mode=1 quant=0,1 > gpurun_out/r3s/quant.jsonl 2>&1 && \
$S mode=1 wave=16,32,48 > gpurun_out/r3s/wave.jsonl 2>&1 && \
$S mode=1 stackcap=8,10,13 > gpurun_out/r3s/cap.jsonl 2>&1
