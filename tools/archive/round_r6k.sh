# r6k: camera pool automatic for the Lambertian kernel over global trees — parity (pool, headline,
# fuzz), bench lines of configs[2]/[3] and the 1/8-share rehearsal of blob70k
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6k
mkdir -p $T
bash tools/gpu_tests.sh r6k "pool or headline or fuzz or split or lds_top or matches_oracle" && \
timeout -k 10 300 python bench.py --preset config3 > $T/config3_blob.json 2> $T/config3_blob.err && \
timeout -k 10 400 python bench.py --preset config4 --steps 2 --warmup 1 --cpu-baseline off > $T/config4_blob4k.json 2> $T/config4_blob4k.err && \
timeout -k 10 300 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,2,4,8 > $T/scaling_blob.jsonl 2>&1
echo "r6k rc=$?"
