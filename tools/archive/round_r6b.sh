# r6b: new loop-exit defaults for LDS scenes (wave 24, leaf exit 12, node exit 8) — the full GPU
# suite, then the general kernel (cornell_mixed) and the wavefront's LDS case checked around them
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6b
mkdir -p $T
bash tools/gpu_tests.sh r6b && \
timeout -k 10 300 python tools/sweep.py --scene cornell_mixed --steps 4 nodeexit=-1,16,48 wave=-1,16 leafexit=-1,4 > $T/sweep_mixed.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 4 mode=1 nodeexit=-1,48 wave=-1,16 leafexit=-1,4 > $T/sweep_cornell_wf.txt 2>&1 && \
timeout -k 10 120 python tools/sweep.py --scene cornell34 --steps 6 wave=-1,-1 > $T/cornell_default.txt 2>&1
echo "r6b rc=$?"
