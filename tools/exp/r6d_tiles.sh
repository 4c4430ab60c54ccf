# round 6: pixel-tile runs for the item order (HIPPT_OPT_PIXEL_TILE) — blob70k (a tree in global memory,
# TA-bound) and Cornell whole images at tile widths 0 (rows) / 8 / 16 / 32, two alternating passes, and
# the 1/8 row shares (band_scaling, every rank) -> gpurun_out/r6d/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6d
mkdir -p $O
B="timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off"
for pass in 1 2; do
  for t in 0 8 16 32; do
    $B --scene blob70k --option PIXEL_TILE=$t > $O/blob_t${t}_p$pass.json 2> $O/blob_t${t}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_t${t}_p$pass.json'));print('blob tile $t pass $pass', d['value'], d['ms_per_step'])"
  done
  for t in 0 8; do
    $B --option PIXEL_TILE=$t > $O/cornell_t${t}_p$pass.json 2> $O/cornell_t${t}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/cornell_t${t}_p$pass.json'));print('cornell tile $t pass $pass', d['value'], d['ms_per_step'])"
  done
done
for t in 0 16 32; do
  timeout -k 10 200 python -u tools/band_scaling.py --scene blob70k --steps 20 --ranks 8 --all-bands 28=1 32=$t > $O/share8_blob_t$t.jsonl || exit 1
  tail -1 $O/share8_blob_t$t.jsonl
done
echo TILES_DONE
