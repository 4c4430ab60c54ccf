set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2n || exit 1
for s in blob70k random_scene; do
timeout -k 10 300 bash tools/ab.sh $s 3 noslp pairsg > gpurun_out/r2n/ab_$s.txt 2>&1 || exit 1
done
