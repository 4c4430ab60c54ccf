# r3ao: work-queue chunk and wave threshold re-sweep on the final trees (alternating, two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ao
S="timeout -k 10 300 python tools/sweep.py --steps 3"
for p in 1 2; do
$S --scene blob70k chunk=256,128,512 >> gpurun_out/r3ao/b_chunk.jsonl 2>&1 && \
$S --scene blob70k wave=32,28,36 >> gpurun_out/r3ao/b_wave.jsonl 2>&1 && \
$S --scene cornell34 chunk=256,128,512 >> gpurun_out/r3ao/c_chunk.jsonl 2>&1 && \
$S --scene cornell34 wave=16,12,20 >> gpurun_out/r3ao/c_wave.jsonl 2>&1 || exit 1
done
