# r6s: why a 1/8 share's marginal cost per spp exceeds 1/8 of the full image's — per-spp slopes
# at stride 1 and 8 (item order on / off) and the phase profile of both
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6s
mkdir -p $T
timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 8,16,32,64 > $T/slope_stride1.json 2>&1 && \
timeout -k 10 200 python tools/launch_overhead.py --stride 8 --spp 16,32,64,128 > $T/slope_stride8.json 2>&1 && \
timeout -k 10 200 python tools/launch_overhead.py --stride 8 --spp 16,32,64,128 28=0 > $T/slope_stride8_noorder.json 2>&1 && \
timeout -k 10 200 python tools/launch_overhead.py --stride 1 --spp 8,16,32,64 28=0 > $T/slope_stride1_noorder.json 2>&1 && \
timeout -k 10 200 python tools/phase_profile.py --spp 64 > $T/phase_full.json 2>&1
echo "r6s rc=$?"
