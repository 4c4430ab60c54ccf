set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2k
for s in cornell34 blob70k random_scene cornell_mixed; do
timeout -k 10 300 bash tools/ab.sh $s 3 lds0 noslp > gpurun_out/r2k/ab_$s.txt 2>&1 || exit 1
done
