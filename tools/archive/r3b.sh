# r3b: exhaustive rounding self-test + parity suite with the short sqrt/rcp sequences; A/B vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 100 python -u -m pytest tests/test_gpu_rounding.py -x -v --timeout 90 --timeout-method thread > gpurun_out/r3b/rounding.log 2>&1 && \
bash tools/gpu_tests.sh r3b && \
timeout -k 10 300 bash tools/ab.sh cornell34 5 base rsq > gpurun_out/r3b/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh random_scene 3 base rsq > gpurun_out/r3b/ab_random.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh cornell_mixed 3 base rsq > gpurun_out/r3b/ab_mixed.txt 2>&1 && \
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r3b/phase_cornell.json 2>&1
