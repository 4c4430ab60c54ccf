set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2o
timeout -k 10 300 python tools/sweep.py --scene cornell34 --steps 3 wave=8,16,24,32 leafexit=2,4,8 > gpurun_out/r2o/cornell_we.jsonl 2>&1 &&
timeout -k 10 300 python tools/sweep.py --scene cornell34 --steps 3 nodeexit=32,40,48,56,64 > gpurun_out/r2o/cornell_ne.jsonl 2>&1 &&
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 2 wave=24,32,40 leafexit=12,15,18 > gpurun_out/r2o/blob_we.jsonl 2>&1 &&
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 2 nodeexit=32,48,56 chunk=128,256,512 > gpurun_out/r2o/blob_ne.jsonl 2>&1
