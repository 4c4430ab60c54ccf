# r6f: per-wave timeline of the 1/8 share and the full image (debug build libv_tl): what the
# waves do after the queues drain
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6f
mkdir -p $T
V=qt-raytracer_amd/libv_tl.so
HIPPT_LIB=$V timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 8 > $T/timeline_cornell_stride8.json 2>&1 && \
HIPPT_LIB=$V timeout -k 10 120 python tools/timeline.py --scene cornell34 --stride 1 > $T/timeline_cornell_stride1.json 2>&1 && \
HIPPT_LIB=$V timeout -k 10 120 python tools/timeline.py --scene blob70k --stride 8 > $T/timeline_blob_stride8.json 2>&1
echo "r6f rc=$?"
