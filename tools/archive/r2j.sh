set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2j || exit 1
timeout -k 10 300 bash tools/ab.sh cornell34 5 r2opt lds0 > gpurun_out/r2j/ab_cornell.txt 2>&1 &&
timeout -k 10 300 bash tools/ab.sh cornell_mixed 3 r2opt lds0 > gpurun_out/r2j/ab_mixed.txt 2>&1
