# round 6: the driver's own round-end sequence on the final tree, as it runs it: the GPU suite without
# this repo's per-test flags, smoke(), bench.py with no flags (N = 1 defaults), and the 2-rank launch
# -> gpurun_out/r6ba/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ba
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > $O/pytest_q.log 2>&1 || { tail -30 $O/pytest_q.log; exit 1; }
  tail -2 $O/pytest_q.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
t1=$(date +%s.%N)
python3 -c "print('bench.py wall s', round($t1 - $t0, 1))"
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['steps'], d['warmup'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2ranks.json 2> $O/bench_2ranks.err || { tail -20 $O/bench_2ranks.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_2ranks.json'));print(d['n_gpus'], d['value'], d['config']['image_crc32'])"
echo DRIVER_DONE
