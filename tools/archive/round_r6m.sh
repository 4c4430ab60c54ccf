# r6m: the legacy 1-spp frame and a 1/8 share at 4 spp against the persistent grid's blocks per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6m
mkdir -p $T
for b in 0 5 3 2; do
  timeout -k 10 120 python tools/legacy_abi_bench.py --scenes cornell34 --frames 100 --opt 5=$b > $T/legacy_bpc$b.json 2>/dev/null || exit 1
  timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 5=$b > $T/spp4_bpc$b.jsonl 2>&1 || exit 1
  timeout -k 10 100 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 64 5=$b > $T/spp64_bpc$b.jsonl 2>&1 || exit 1
done
echo "r6m rc=$?"
