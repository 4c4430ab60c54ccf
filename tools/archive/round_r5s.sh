# r5s: is the per-wave end-of-launch counter atomics (2 x 7168 on one cache line) the launch's
# fixed cost?  1/8-share rehearsal and launch-overhead fit with and without them (libv_noatom)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5s
mkdir -p $T
V=qt-raytracer_amd/libv_noatom.so
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_base.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_noatom.jsonl 2>&1 && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 > $T/spp4_base.jsonl 2>&1 && \
HIPPT_LIB=$V timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --ranks 8 --spp 4 > $T/spp4_noatom.jsonl 2>&1
echo "r5s rc=$?"
