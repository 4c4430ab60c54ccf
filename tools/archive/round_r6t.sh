# r6t: the item order's effect against job size (Cornell full image 16/32/64 spp, alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6t
mkdir -p $T
for i in 1 2; do
  timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 16,32,64 28=0 >> $T/slope_stride1_noorder.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 16,32,64 >> $T/slope_stride1_order.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 16,32,64 --scene blob70k 28=0 >> $T/slope_blob_noorder.jsonl 2>&1 && \
timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 16,32,64 --scene blob70k >> $T/slope_blob_order.jsonl 2>&1
echo "r6t rc=$?"
