# r5a: first GPU pass of round 3 — GPU suite (new headline/config-4/hybrid/flush tests), hybrid-node
# A/B on blob70k, legacy-ABI timing, default bench line, 2-rank strong-scaling rehearsal on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5a
mkdir -p $T
bash tools/gpu_tests.sh r5a && \
timeout -k 10 150 python tools/sweep.py --scene blob70k --steps 5 quant=0,2,0,2,1 > $T/sweep_blob.txt 2>&1 && \
timeout -k 10 150 python tools/sweep.py --scene blob70k --width 3840 --height 2160 --spp 16 --steps 3 quant=0,2,0,2 > $T/sweep_blob4k.txt 2>&1 && \
bash tools/ab.sh cornell34 5 nopack pack > $T/ab_pack_cornell.txt 2>&1 && \
bash tools/ab.sh cornell_mixed 5 nopack pack > $T/ab_pack_mixed.txt 2>&1 && \
timeout -k 10 200 python tools/legacy_abi_bench.py > $T/legacy.json 2> $T/legacy.err && \
timeout -k 10 300 python bench.py > $T/bench.json 2> $T/bench.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline off > $T/n2_strong.json 2> $T/n2_strong.err
echo "r5a rc=$?"
