# round 5: every 1/2, 1/4, 1/8 interleaved share of BASELINE configs[3]
# (blob70k 3840x2160, 256 spp, 8 bounces) timed on one GPU, 5 steps each, item order forced as in
# bench.py; plus the Cornell 1080p shares on the same box for reference
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 500 python -u tools/band_scaling.py --scene blob70k --width 3840 --height 2160 --spp 256 --steps 5 --ranks 1,2,4,8 --all-bands 28=1 > gpurun_out/r5a/strong_scaling_rehearsal_blob70k_4k.jsonl || exit 1
timeout -k 10 200 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 --all-bands 28=1 > gpurun_out/r5a/strong_scaling_rehearsal_cornell34.jsonl || exit 1
