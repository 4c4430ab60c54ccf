# r3at: 2-wide build knobs under the automatic (SAH-optimal) collapse on LDS scenes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3at
S="timeout -k 10 300 python tools/sweep.py --steps 4"
$S --scene cornell34 tcost=100,60,150,100,60,150 > gpurun_out/r3at/c_tcost.jsonl 2>&1 && \
$S --scene cornell34 sah=1,0,1,0 > gpurun_out/r3at/c_sah.jsonl 2>&1 && \
$S --scene cornell34 leaf=2,3,2,3 > gpurun_out/r3at/c_leaf.jsonl 2>&1 && \
$S --scene cornell_mixed tcost=100,60,150,100,60,150 > gpurun_out/r3at/m_tcost.jsonl 2>&1
