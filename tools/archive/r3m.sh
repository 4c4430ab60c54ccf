# r3m: Cornell/blob re-sweeps of the SAH cost, leaf size and loop-exit knobs on the current kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3m
S="timeout -k 10 200 python tools/sweep.py"
$S --scene cornell34 --steps 5 tcost=60,100,150,250 leaf=2,4,8 > gpurun_out/r3m/c_sah.jsonl 2>&1 && \
$S --scene cornell34 --steps 5 wave=8,16,24,32 > gpurun_out/r3m/c_wave.jsonl 2>&1 && \
$S --scene cornell34 --steps 5 leafexit=2,4,8 nodeexit=24,48,56 > gpurun_out/r3m/c_exit.jsonl 2>&1 && \
$S --scene blob70k --steps 3 wave=16,24,32,40 > gpurun_out/r3m/b_wave.jsonl 2>&1 && \
$S --scene cornell_mixed --steps 5 tcost=60,100,150,250 > gpurun_out/r3m/m_sah.jsonl 2>&1
