# round 4: kernel trace of chained batches against one launch per batch (1/8 Cornell share, 10 steps)
set -o pipefail
mkdir -p gpurun_out/r4s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4s/share1 -o run -- python3 $GRAFT_REPO_ROOT/tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 30=1 > $GRAFT_REPO_ROOT/gpurun_out/r4s/share1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4s/share0 -o run -- python3 $GRAFT_REPO_ROOT/tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 30=0 > $GRAFT_REPO_ROOT/gpurun_out/r4s/share0.log 2>&1 || exit 1
