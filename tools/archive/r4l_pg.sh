# round 4: packed child keys over global trees (libv_pg.so, -DHIPPT_PACKED_GLOBAL=1): parity with the
# variant library, then the A/B against the default library
set -o pipefail
mkdir -p gpurun_out/r4l
HIPPT_LIB=qt-raytracer_amd/libv_pg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not wavefront and not rgba8 and not legacy and not present and not rng_table" > gpurun_out/r4l/pytest_pg.log 2>&1 || exit 1
for i in 1 2; do
  for lib in libhippt libv_pg; do
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,8 28=1 > gpurun_out/r4l/blob_${lib}_$i.jsonl || exit 1
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene random_scene --steps 10 --ranks 1 28=1 > gpurun_out/r4l/random_${lib}_$i.jsonl || exit 1
  done
done
