# s7o: the app's 1-spp Cornell frame (cudaPathTracerRender) under camera pool / item order /
# work chunk settings, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7o
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes cornell34 > $O/default_p$pass.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes cornell34 --opt 26=0 > $O/pool0_p$pass.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes cornell34 --opt 28=0 > $O/order0_p$pass.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/legacy_abi_bench.py --scenes cornell34 --opt 4=64 > $O/chunk64_p$pass.json 2>&1 || exit 1
done
echo "s7o rc=$?"
