set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2l || exit 1
for s in cornell34 blob70k cornell_mixed; do
timeout -k 10 300 bash tools/ab.sh $s 3 noslp w8 > gpurun_out/r2l/ab_$s.txt 2>&1 || exit 1
done
