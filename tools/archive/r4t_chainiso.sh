# round 4: which part of the chained-batch kernel costs: its 6-wave occupancy only (ce1: plain queue
# and camera code), plus the chained queue (ce2), the full kernel (libhippt), one launch per batch (30=0)
set -o pipefail
mkdir -p gpurun_out/r4t
for i in 1 2; do
  for lib in libv_ce1 libv_ce2 libhippt; do
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 30=1 > gpurun_out/r4t/${lib}_$i.jsonl || exit 1
  done
  timeout -k 10 150 python -u tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 30=0 > gpurun_out/r4t/plain_$i.jsonl || exit 1
done
