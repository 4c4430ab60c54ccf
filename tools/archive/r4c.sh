# r4c: -O2, no loop unrolling, iterative ILP / min-register schedulers, no high-pressure
# reschedule (-mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1) vs the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
V="base o2 nounroll iterilp iterminreg noresched"
bash tools/ab.sh cornell34 5 $V > gpurun_out/r4c/ab_cornell.txt 2>&1 && \
bash tools/ab.sh blob70k 4 $V > gpurun_out/r4c/ab_blob.txt 2>&1 && \
bash tools/ab.sh cornell_mixed 4 $V > gpurun_out/r4c/ab_mixed.txt 2>&1 && \
bash tools/ab.sh random_scene 4 $V > gpurun_out/r4c/ab_random.txt 2>&1
python3 tools/ab_summary.py gpurun_out/r4c/ab_*.txt
