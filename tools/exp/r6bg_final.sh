# round 6, the final library (kept work buffers, a failed allocation leaving the size at 0; thresholds
# 40 / 22 / 56 for Lambertian scenes over global trees; every asynchronous batch chained, cap 8 for whole
# images): GPU suite, smoke, every BASELINE bench line, the rehearsal, --gpus 2 / 4 and the 8-rank command,
# the headline profiles and the headline lines again with them in place -> gpurun_out/r6bg/, prof_r6bg*/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6bg
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
bash tools/gpu_tests.sh r6bg || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
B="timeout -k 10 400 python3 bench.py"
S="--steps 20 --warmup 5"
$B $S > $O/bench_cornell.json 2> $O/cornell.err || exit 1
$B $S --scene blob70k > $O/bench_blob.json 2> $O/blob.err || exit 1
$B --preset config4 --steps 5 --warmup 1 --cpu-baseline off > $O/bench_blob4k.json 2> $O/blob4k.err || exit 1
$B $S --preset config5 --cpu-baseline off > $O/bench_blob_wf.json 2> $O/wf.err || exit 1
$B $S --scene random_scene --cpu-baseline off > $O/bench_random.json 2> $O/random.err || exit 1
$B $S --scene cornell_mixed --cpu-baseline off > $O/bench_mixed.json 2> $O/mixed.err || exit 1
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
for sc in cornell34 blob70k; do
  timeout -k 10 300 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,2,4,8 --all-bands 28=1 > $O/rehearsal_$sc.jsonl || exit 1
done
for n in 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 --cpu-baseline off > $O/bench_${n}ranks.json 2> $O/bench_${n}ranks.err || { tail -20 $O/bench_${n}ranks.err; exit 1; }
done
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --steps 20 --warmup 5 > $O/bench_8ranks.json 2> $O/bench_8ranks.err || { tail -30 $O/bench_8ranks.err; exit 1; }
bash tools/profile.sh r6bg || exit 1
bash tools/profile.sh r6bg_blob --scene blob70k || exit 1
python3 tools/prof_summary.py r6bg --name cornell_1080p_64spp_r6bg --out profiles/round6 > /dev/null || exit 1
python3 tools/prof_summary.py r6bg_blob --name blob70k_1080p_64spp_r6bg --out profiles/round6 > /dev/null || exit 1
$B $S > $O/bench_cornell_with_traffic.json 2> $O/cornell_t.err || exit 1
$B $S --scene blob70k --cpu-baseline off > $O/bench_blob_with_traffic.json 2> $O/blob_t.err || exit 1
for f in $O/bench_*with_traffic.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['frac'], r['traffic'], r.get('limiter'), r.get('pmc_refused'))"; done
echo FINAL_DONE
