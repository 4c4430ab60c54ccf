# round 6: where the 1/8 Cornell share's time goes — the share's pixels as one 512-spp launch, the
# whole image as one 64-spp launch, the 20-step burst at caps 8 / 1 / 0 and 256-item claims
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6i
mkdir -p $O
BS="timeout -k 10 200 python -u tools/band_scaling.py --scene cornell34"
$BS --steps 4 --spp 512 --ranks 8 28=1 > $O/share8_512spp.jsonl || exit 1
$BS --steps 20 --ranks 1 28=1 30=0 > $O/whole_64spp_unchained.jsonl || exit 1
$BS --steps 20 --ranks 1 28=1 30=8 > $O/whole_64spp_cap8.jsonl || exit 1
for opt in "30=8" "30=1" "30=0" "30=8 4=256" "30=4"; do
  tag=$(echo $opt | tr ' =' '_-')
  $BS --steps 20 --ranks 8 28=1 $opt > $O/share8_$tag.jsonl || exit 1
done
tail -n 1 $O/*.jsonl
echo SHARE_DONE
