# r3ak: leaf loop in pairs for LDS-resident scenes too (leaves now hold <= 2 primitives)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ak
timeout -k 10 300 bash tools/ab.sh cornell34 8 base ldspairs > gpurun_out/r3ak/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh cornell_mixed 6 base ldspairs > gpurun_out/r3ak/ab_mixed.txt 2>&1
