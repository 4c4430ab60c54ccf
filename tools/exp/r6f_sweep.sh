# round 6: blob70k occupancy / LDS top / stack cap around the defaults with 8x8 tile runs, and the 1/8
# row shares at tile widths 0 / 8 / 16 (every rank) -> gpurun_out/r6f/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 400 python -u tools/sweep.py --scene blob70k --steps 10 tile=8 bpc=0,4,5,6 stackcap=0,8,10,13 > $O/sweep_blob.jsonl || exit 1
for sc in cornell34 blob70k; do
  for t in 0 8 16; do
    timeout -k 10 200 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 8 --all-bands 28=1 32=$t > $O/share8_${sc}_t$t.jsonl || exit 1
  done
done
echo SWEEP_DONE
