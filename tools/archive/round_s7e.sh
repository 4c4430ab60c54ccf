# s7e: legacy frames written by the kernel straight into the pinned host frame (zero copy):
# legacy parity tests, then the app's per-frame cost with and without, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7e
mkdir -p $O
bash tools/gpu_tests.sh s7e "legacy or present or interleave or multi or devices" && \
for pass in 1 2; do
  for v in zc0 zc1; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes sphere4 > $O/legacy_${v}_p$pass.json 2> $O/legacy_${v}_p$pass.err || exit 1
  done
done && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err
echo "s7e rc=$?"
