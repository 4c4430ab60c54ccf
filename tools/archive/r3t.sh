# r3t: per-wave LDS stack regions + larger persistent-grid blocks for global-memory trees
# (HIPPT_OPT_BLOCK_WAVES 4/7/14): parity suite, then blob70k / random_scene / 4K sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3t
S="timeout -k 10 200 python tools/sweep.py"
bash tools/gpu_tests.sh r3t && \
$S --scene blob70k --steps 4 bw=4,14,7,4 > gpurun_out/r3t/b_bw.jsonl 2>&1 && \
$S --scene random_scene --steps 4 bw=4,14,7,4 > gpurun_out/r3t/r_bw.jsonl 2>&1 && \
$S --scene cornell34 --steps 4 > gpurun_out/r3t/c.jsonl 2>&1
