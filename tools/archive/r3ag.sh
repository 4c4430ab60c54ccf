# r3ag: max BVH leaf size 2 vs 4 (alternating, one process per scene) on the four bench scenes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ag
for sc in blob70k cornell34 random_scene cornell_mixed; do
  timeout -k 10 300 python tools/sweep.py --scene $sc --steps 4 leaf=4,2,4,2,4,2 > gpurun_out/r3ag/$sc.jsonl 2>&1 || exit 1
done
