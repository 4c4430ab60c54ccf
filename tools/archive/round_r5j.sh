# r5j: wavefront shade blocks partitioned by material kind (HIPPT_OPT_SHADE_SORT) — parity, then
# in-process A/B on the general-kernel scenes at 1080p
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5j
mkdir -p $T
bash tools/gpu_tests.sh r5j "shade_sort or wavefront" && \
timeout -k 10 250 python tools/sweep.py --scene random_scene --steps 4 mode=1 ssort=0,1,0,1 > $T/ab_ssort_random.txt 2>&1 && \
timeout -k 10 250 python tools/sweep.py --scene cornell_mixed --steps 4 mode=1 ssort=0,1,0,1 > $T/ab_ssort_mixed.txt 2>&1
echo "r5j rc=$?"
