# round 4: strong-scaling rehearsal on one GPU (every rank's share, tools/band_scaling.py) and the
# driver's launch with 2 and 4 ranks on the one GPU (torch.distributed.run)
set -o pipefail
mkdir -p gpurun_out/r4k
timeout -k 10 300 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,2,4,8 --all-bands 28=1 > gpurun_out/r4k/strong_scaling_rehearsal_cornell34.jsonl || exit 1
timeout -k 10 400 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,2,4,8 --all-bands 28=1 > gpurun_out/r4k/strong_scaling_rehearsal_blob70k.jsonl || exit 1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $n --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r4k/rehearsal_${n}ranks_1gpu_strong.json 2> gpurun_out/r4k/rehearsal_${n}ranks.err || exit 1
done
