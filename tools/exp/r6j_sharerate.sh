# round 6: is the 1/8 share slower per sample than the whole image at equal work (one launch of
# 132.7 M samples)?  Interleaved share and contiguous band at 512 spp, the whole image at 64 spp with
# row runs and with 8x8 tiles, the 1/2 share at 128 spp -> gpurun_out/r6j/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6j
mkdir -p $O
BS="timeout -k 10 200 python -u tools/band_scaling.py --scene cornell34 --steps 6"
for pass in 1 2; do
  $BS --spp 512 --ranks 8 28=1 > $O/share8_512_p$pass.jsonl || exit 1
  $BS --spp 512 --ranks 8 --split bands 28=1 > $O/band8_512_p$pass.jsonl || exit 1
  $BS --spp 128 --ranks 2 28=1 > $O/share2_128_p$pass.jsonl || exit 1
  $BS --ranks 1 28=1 32=0 > $O/whole_rows_p$pass.jsonl || exit 1
  $BS --ranks 1 28=1 > $O/whole_tiles_p$pass.jsonl || exit 1
done
tail -n 1 $O/*.jsonl
