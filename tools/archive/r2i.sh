set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2i || exit 1
timeout -k 10 300 bash tools/ab.sh cornell34 5 nospill r2opt > gpurun_out/r2i/ab_cornell.txt 2>&1 &&
timeout -k 10 300 bash tools/ab.sh blob70k 3 nospill r2opt > gpurun_out/r2i/ab_blob.txt 2>&1 &&
timeout -k 10 300 bash tools/ab.sh random_scene 3 nospill r2opt > gpurun_out/r2i/ab_random.txt 2>&1
