# round 5: the multi-rank path on one GPU with the final library — bench.py --gpus 2 / 4 starts its own
# ranks (torch.distributed.run, 127.0.0.1), every rank's share chained; the gathered image's CRC
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5aj
mkdir -p $O
for n in 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 --cpu-baseline off > $O/bench_${n}ranks.json 2> $O/bench_${n}ranks.err || { tail -20 $O/bench_${n}ranks.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_${n}ranks.json').read().strip().splitlines()[-1]); c=d['config']
print($n, d['value'], d['ms_per_step'], 'crc', c.get('image_crc32'), 'chain', c['chain'].get('applied_cap'), 'chunk', c['chunk'].get('applied'), 'ranks', d.get('ranks', {}).get('trace_ms_per_step'))"
done
