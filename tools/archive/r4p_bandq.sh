# round 4: queue g takes image band g's runs (libv_bandq.so, -DHIPPT_BAND_QUEUES=1) against the
# default table (each queue 8 frames of the whole image); parity subset first
set -o pipefail
mkdir -p gpurun_out/r4p
HIPPT_LIB=qt-raytracer_amd/libv_bandq.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not rgba8 and not legacy and not present and not rng_table" > gpurun_out/r4p/pytest_bandq.log 2>&1 || exit 1
for i in 1 2; do
  for lib in libhippt libv_bandq; do
    for scene in blob70k random_scene cornell34; do
      HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene $scene --steps 10 --ranks 1,8 28=1 > gpurun_out/r4p/${scene}_${lib}_$i.jsonl || exit 1
    done
  done
done
