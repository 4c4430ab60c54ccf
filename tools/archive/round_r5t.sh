# r5t: launch counters spread over 64 copies (one cache line per 1/64 of the blocks) — parity
# (counting mode, legacy scene, headline), 1/8-share rehearsal, launch-overhead points, the
# legacy ABI frame, full-size A/B against the previous build (libv_head)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5t
mkdir -p $T
V=qt-raytracer_amd/libv_head.so
bash tools/gpu_tests.sh r5t "counting or legacy or sphere or headline or pool or stats or matches_oracle" && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell.jsonl 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob.jsonl 2>&1 && \
timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 > $T/spp4.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 > $T/spp4_head.jsonl 2>&1 && \
timeout -k 10 200 python tools/legacy_abi_bench.py > $T/legacy_abi.json 2> $T/legacy_abi.err && \
HIPPT_LIB=$V timeout -k 10 200 python tools/legacy_abi_bench.py > $T/legacy_abi_head.json 2> $T/legacy_abi_head.err && \
for i in 1 2; do
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 order=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
done
echo "r5t rc=$?"
