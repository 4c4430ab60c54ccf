# round 4: the closest-hit update without branches (libv_bf.so) and the triangle test without any
# branch (libv_flat.so, -DHIPPT_FLAT_TRI=1): parity of both, then the A/B against the round's
# default library (libv_base.so) on the four scene kinds, alternating
set -o pipefail
mkdir -p gpurun_out/r4n
for lib in libv_bf libv_flat; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not rgba8 and not legacy and not present and not rng_table" > gpurun_out/r4n/pytest_$lib.log 2>&1 || exit 1
done
for i in 1 2; do
  for lib in libv_base libv_bf libv_flat; do
    for scene in cornell34 blob70k random_scene cornell_mixed; do
      HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene $scene --steps 10 --ranks 1 28=1 > gpurun_out/r4n/${scene}_${lib}_$i.jsonl || exit 1
    done
  done
done
