# round 4: the item order with the sky-only runs first (libv_sky.so, -DHIPPT_SKY_FIRST=1) against the
# default (longest first, sky last): whole image and every 1/8 share, alternating
set -o pipefail
mkdir -p gpurun_out/r4x
for i in 1 2; do
  for lib in libhippt libv_sky; do
    for scene in cornell34 blob70k; do
      HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene $scene --steps 10 --ranks 1,8 --all-bands 28=1 > gpurun_out/r4x/${scene}_${lib}_$i.jsonl || exit 1
    done
  done
done
