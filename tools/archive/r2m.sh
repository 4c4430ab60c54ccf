set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2m
for s in blob70k cornell34 cornell_mixed; do
timeout -k 10 300 bash tools/ab.sh $s 3 noslp leafpairs > gpurun_out/r2m/ab_$s.txt 2>&1 || exit 1
done
