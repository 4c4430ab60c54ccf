set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 120 tools/micro/valu_cost > gpurun_out/r2c/valu.txt 2>&1 &&
timeout -k 10 120 tools/micro/ta_cost > gpurun_out/r2c/ta.txt 2>&1 &&
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 3 --count leaf=1,2,3,4,6,8 tcost=100,200 > gpurun_out/r2c/sweep_cornell.jsonl 2>&1
