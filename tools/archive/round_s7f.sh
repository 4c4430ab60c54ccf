# s7f: blocking frames written into the pinned host frame by the kernel that makes them (legacy
# kernel; the mesh combine): full GPU suite, then per-frame cost with and without, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7f
mkdir -p $O
bash tools/gpu_tests.sh s7f && \
for pass in 1 2; do
  for v in zc0 zc1; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_${v}_p$pass.json 2> $O/legacy_${v}_p$pass.err || exit 1
  done
done && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err && \
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "s7f rc=$?"
