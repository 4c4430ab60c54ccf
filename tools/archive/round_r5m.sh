# r5m: wavefront ray queues carrying the paths' state (no slot indirection) — the wavefront
# parity suite, then config 5 A/B against the slot-pool variant (libv_wfold)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5m
mkdir -p $T
V=qt-raytracer_amd/libv_wfold.so
bash tools/gpu_tests.sh r5m "wavefront or counting or switch or deferred" && \
for i in 1 2; do
  timeout -k 10 120 python tools/sweep.py --scene blob70k --steps 4 mode=1 >> $T/ab_wf_blob.txt 2>&1 || exit 1
  HIPPT_LIB=$V timeout -k 10 120 python tools/sweep.py --scene blob70k --steps 4 mode=1 >> $T/ab_wf_blob.txt 2>&1 || exit 1
done && \
timeout -k 10 120 python tools/sweep.py --scene cornell34 --steps 4 mode=1 >> $T/ab_wf_cornell.txt 2>&1 && \
HIPPT_LIB=$V timeout -k 10 120 python tools/sweep.py --scene cornell34 --steps 4 mode=1 >> $T/ab_wf_cornell.txt 2>&1
echo "r5m rc=$?"
