# r3g: the previous batch's combine inside the next megakernel launch: parity + A/B vs r3f
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
bash tools/gpu_tests.sh r3g && \
timeout -k 10 300 bash tools/ab.sh cornell34 5 fresh fuse > gpurun_out/r3g/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh blob70k 3 fresh fuse > gpurun_out/r3g/ab_blob.txt 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r3g/cornell.json 2> gpurun_out/r3g/cornell.err
