# round 6: blob70k's LDS top of the tree and stack cap at the new big-batch defaults (tools/sweep.py,
# 200 ms warm-up, 5 timed steps, two passes) -> gpurun_out/r6ar/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ar
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 top=-1,21,48,64,85,128 stackcap=0,8 > $O/blob_top_p$pass.jsonl 2> $O/blob_top_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 tile=-1,0,16 chunk=256,512 > $O/blob_tile_p$pass.jsonl 2> $O/blob_tile_p$pass.err || exit 1
done
echo TOP_DONE
