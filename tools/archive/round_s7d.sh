# s7d: chunked blocking legacy frames (copy of chunk k behind the kernel of chunk k+1): legacy
# parity tests, then the app's per-frame cost with 1 / 4 / 8 chunks, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7d
mkdir -p $O
bash tools/gpu_tests.sh s7d "legacy" && \
for pass in 1 2; do
  for v in chunks1 chunks4 chunks8; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes sphere4 > $O/legacy_${v}_p$pass.json 2> $O/legacy_${v}_p$pass.err || exit 1
  done
done && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err
echo "s7d rc=$?"
