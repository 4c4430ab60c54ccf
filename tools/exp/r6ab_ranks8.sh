# round 6: the driver's own multi-rank command at N = 8 (torch.distributed.run, 8 ranks) on the one
# GPU of the box (every rank's share on device 0; rank -> device is local_rank % devices): the 8-rank
# path end to end, one JSON line, gathered image CRC -> gpurun_out/r6ab/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab
mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --steps 20 --warmup 5 > $O/bench_8ranks.json 2> $O/bench_8ranks.err || { tail -30 $O/bench_8ranks.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_8ranks.json'));print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('image_crc32'), d['config'].get('rank_imbalance'), d.get('cpu_baseline'))"
echo RANKS8_DONE
