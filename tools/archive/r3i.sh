# r3i: fused combine code size / placement A/B vs r3f (fresh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3i
timeout -k 10 400 bash tools/ab.sh blob70k 5 fresh noun combl > gpurun_out/r3i/ab_blob.txt 2>&1 && \
timeout -k 10 400 bash tools/ab.sh cornell34 8 fresh noun combl > gpurun_out/r3i/ab_cornell.txt 2>&1
