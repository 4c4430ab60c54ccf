# round 5 final: bench lines of every BASELINE config and the extra scenes, and the one-GPU strong-
# scaling rehearsal (every rank's row share, N = 1, 2, 4, 8) -> gpurun_out/r5w/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5w
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
B="timeout -k 10 300 python3 bench.py"
S="--steps 20 --warmup 5"
$B $S > $O/bench_cornell.json 2> $O/cornell.err || exit 1
cat $O/bench_cornell.json
$B $S --scene blob70k > $O/bench_blob.json 2> $O/blob.err || exit 1
$B --scene blob70k --width 3840 --height 2160 --spp 256 --steps 5 --warmup 1 --cpu-baseline off > $O/bench_blob4k.json 2> $O/blob4k.err || exit 1
$B $S --scene blob70k --path-mode wavefront --cpu-baseline off > $O/bench_blob_wf.json 2> $O/wf.err || exit 1
$B $S --scene random_scene --cpu-baseline off > $O/bench_random.json 2> $O/random.err || exit 1
$B $S --scene cornell_mixed --cpu-baseline off > $O/bench_mixed.json 2> $O/mixed.err || exit 1
for sc in cornell34 blob70k; do
  timeout -k 10 300 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,2,4,8 --all-bands 28=1 > $O/rehearsal_$sc.jsonl || exit 1
done
echo BENCH_DONE
