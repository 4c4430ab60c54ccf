set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u tools/exp/chain_debug.py cornell34 > gpurun_out/r5c/dbg_cornell.txt 2>&1; rc=$?
cat gpurun_out/r5c/dbg_cornell.txt
exit $rc
