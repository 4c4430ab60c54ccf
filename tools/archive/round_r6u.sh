# r6u: item-order variants — cost buckets (image order within a bucket) and run-major ties
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6u
mkdir -p $T
S="timeout -k 10 200 python tools/sweep.py --steps 5"
for i in 1 2; do
  $S --scene cornell34 order=0,1,4,8,16,128,132,136,144 >> $T/sweep_cornell64.txt 2>&1 || exit 1
  $S --scene cornell34 --spp 32 order=0,1,4,8,16,128,132,136,144 >> $T/sweep_cornell32.txt 2>&1 || exit 1
  $S --scene blob70k --steps 3 order=0,1,4,8,136 >> $T/sweep_blob64.txt 2>&1 || exit 1
done
for v in 0 1 8 136 0 1 8 136; do
  timeout -k 10 100 python tools/launch_overhead.py --stride 8 --spp 64,128 28=$v >> $T/share_order_$v.jsonl 2>&1 || exit 1
done
echo "r6u rc=$?"
