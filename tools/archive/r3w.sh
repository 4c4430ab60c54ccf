# r3w: multi-rank rehearsal of the driver's N>1 bench launch on one GPU (both ranks on device 0):
# --scaling strong renders the same 64 frames, so the gathered image CRC must equal the N=1 run's
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3w
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r3w/n1.json 2> gpurun_out/r3w/n1.err && \
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 2 --warmup 1 --scaling strong > gpurun_out/r3w/n2_strong.json 2> gpurun_out/r3w/n2_strong.err && \
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
    bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r3w/n2_weak.json 2> gpurun_out/r3w/n2_weak.err
