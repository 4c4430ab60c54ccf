# round 4: what one launch per several steps would buy the 1/8 share: the share at 64 spp per launch
# against 128 / 256 / 640 spp per launch (per-64-spp time = ms_per_step * 64 / spp)
set -o pipefail
mkdir -p gpurun_out/r4q
for scene in cornell34 blob70k; do
  for spp in 64 128 256 640; do
    steps=$(( 640 / spp )); [ $steps -lt 2 ] && steps=2
    timeout -k 10 200 python -u tools/band_scaling.py --scene $scene --spp $spp --steps $steps --ranks 1,8 28=1 > gpurun_out/r4q/${scene}_spp$spp.jsonl || exit 1
  done
done
