# r2x: full GPU parity suite after the LDS top of the tree; default-option timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2x
bash tools/gpu_tests.sh r2x && \
timeout -k 10 120 python tools/sweep.py --scene blob70k --steps 5 > gpurun_out/r2x/blob.jsonl && \
timeout -k 10 120 python tools/sweep.py --scene random_scene --steps 5 > gpurun_out/r2x/random.jsonl && \
timeout -k 10 120 python tools/sweep.py --scene cornell34 --steps 5 > gpurun_out/r2x/cornell.jsonl && \
timeout -k 10 120 python tools/sweep.py --scene blob70k --width 3840 --height 2160 --spp 256 --steps 1 > gpurun_out/r2x/blob4k.jsonl
