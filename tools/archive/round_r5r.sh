# r5r: queues hand out, within each XCD queue, the scene-hitting runs of all its frames first and the sky runs last
# (HIPPT_OPT_ITEM_ORDER) — parity, strong-scaling rehearsal (every 1/8 share), full-size A/B
# (order 0/1 in one process, and against the previous build, libv_head)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5r
mkdir -p $T
V=qt-raytracer_amd/libv_head.so
bash tools/gpu_tests.sh r5r "pool or headline or row_interleave or matches_oracle or deferred or split" && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $T/scaling_cornell_order.jsonl 2>&1 && \
timeout -k 10 200 python tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 28=0 > $T/scaling_cornell_noorder.jsonl 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 > $T/scaling_blob_order.jsonl 2>&1 && \
timeout -k 10 250 python tools/band_scaling.py --scene blob70k --all-bands --ranks 1,8 28=0 > $T/scaling_blob_noorder.jsonl 2>&1 && \
timeout -k 10 150 python tools/sweep.py --scene cornell34 --steps 6 order=0,1,0,1 > $T/ab_cornell.txt 2>&1 && \
HIPPT_LIB=$V timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 4 order=0,1,0,1 > $T/ab_blob.txt 2>&1
echo "r5r rc=$?"
