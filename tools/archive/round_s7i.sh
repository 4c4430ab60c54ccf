# s7i: the driver's multi-rank bench launch rehearsed on one GPU (2 and 4 ranks share device 0):
# strong scaling of configs[1], the gathered image's CRC against the N=1 line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7i
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 2 > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 20 --warmup 2 > $O/rehearsal_4ranks.json 2> $O/rehearsal_4ranks.err
echo "s7i rc=$?"
