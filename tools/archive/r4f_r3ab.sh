# round 4: the current library against round 3's (libv_r3.so, built from e76396a) on the same box
set -o pipefail
mkdir -p gpurun_out/r4f
for i in 1 2; do
  for lib in libhippt libv_r3; do
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 120 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 28=1 > gpurun_out/r4f/cornell_${lib}_$i.jsonl || exit 1
  done
done
for lib in libhippt libv_r3; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,8 28=1 > gpurun_out/r4f/blob_${lib}.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in libhippt libv_r3; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f/prof_$lib -o kt -- python3 -u tools/band_scaling.py --scene cornell34 --steps 5 --ranks 1 28=1 > gpurun_out/r4f/prof_$lib.log 2>&1 || exit 1
done
