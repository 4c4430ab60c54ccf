# s7g: blocking single-frame mesh batches combined by the lanes that finish the samples (direct):
# full GPU suite, per-frame cost with and without zero-copy/direct, headline bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7g
mkdir -p $O
bash tools/gpu_tests.sh s7g && \
for pass in 1 2; do
  for v in zc0 zc1; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_${v}_p$pass.json 2> $O/legacy_${v}_p$pass.err || exit 1
  done
done && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err && \
timeout -k 10 300 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err && \
timeout -k 10 300 python -u bench.py --preset config3 --cpu-baseline off > $O/bench_config3.json 2> $O/bench_config3.err
echo "s7g rc=$?"
