# r3u: 8- and 12-wave blocks (6 waves per SIMD, one top-of-tree copy per block) vs 4-wave blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3u
S="timeout -k 10 200 python tools/sweep.py"
$S --scene blob70k --steps 4 bw=4,12,8,4 > gpurun_out/r3u/b_bw.jsonl 2>&1 && \
$S --scene random_scene --steps 4 bw=4,12,8,4 > gpurun_out/r3u/r_bw.jsonl 2>&1 && \
$S --scene blob70k --steps 4 bw=12 stackcap=8,10,13 > gpurun_out/r3u/b_cap12.jsonl 2>&1
