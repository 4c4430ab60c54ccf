set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2f
timeout -k 10 300 bash tools/ab.sh blob70k 3 nospill latecodes > gpurun_out/r2f/ab_blob.txt 2>&1
