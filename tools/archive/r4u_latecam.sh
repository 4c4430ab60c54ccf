# round 4: camera-sample and item-order arguments loaded where camera rays are made (libv_late.so,
# -DHIPPT_LATE_CAM=1) against the default library; parity subset first, then alternating A/B
set -o pipefail
mkdir -p gpurun_out/r4u
HIPPT_LIB=qt-raytracer_amd/libv_late.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not rgba8 and not legacy and not present and not rng_table" > gpurun_out/r4u/pytest_late.log 2>&1 || exit 1
for i in 1 2; do
  for lib in libhippt libv_late; do
    for scene in cornell34 blob70k random_scene cornell_mixed; do
      HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene $scene --steps 10 --ranks 1 28=1 > gpurun_out/r4u/${scene}_${lib}_$i.jsonl || exit 1
    done
  done
done
