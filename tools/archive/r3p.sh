# r3p: A/B of the pixel-major work-item order (64 consecutive items = 64 frames of one pixel) vs frame-major
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3p
timeout -k 10 300 bash tools/ab.sh cornell34 6 base pixmaj > gpurun_out/r3p/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh blob70k 4 base pixmaj > gpurun_out/r3p/ab_blob.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh random_scene 4 base pixmaj > gpurun_out/r3p/ab_random.txt 2>&1
