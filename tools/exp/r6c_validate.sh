# round 6: the fixed chained path's speed and multi-rank images — headline bench lines, the one-GPU
# strong-scaling rehearsal (every rank's row share, N = 1, 2, 4, 8) and bench.py --gpus 2 / 4 (its own
# ranks on one GPU, gathered image CRC) -> gpurun_out/r6c/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6c
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
B="timeout -k 10 300 python3 bench.py"
S="--steps 20 --warmup 5 --cpu-baseline off"
$B $S > $O/bench_cornell.json 2> $O/cornell.err || exit 1
$B $S --scene blob70k > $O/bench_blob.json 2> $O/blob.err || exit 1
for sc in cornell34 blob70k; do
  timeout -k 10 300 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,2,4,8 --all-bands 28=1 > $O/rehearsal_$sc.jsonl || exit 1
done
for n in 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 --cpu-baseline off > $O/bench_${n}ranks.json 2> $O/bench_${n}ranks.err || { tail -20 $O/bench_${n}ranks.err; exit 1; }
done
echo VALIDATE_DONE
