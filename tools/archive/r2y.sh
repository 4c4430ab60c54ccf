# r2y: 8 waves per SIMD (80 SGPRs, 64 VGPRs, a few spills) vs 7
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2y
bash tools/ab.sh cornell34 5 base w8 > gpurun_out/r2y/cornell.txt && bash tools/ab.sh blob70k 3 base w8 > gpurun_out/r2y/blob.txt
