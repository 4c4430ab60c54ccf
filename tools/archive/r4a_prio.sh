# round 4: GPU suite, then the wave-priority A/B (libv_prio1/2 against the default library) on the
# 1/8 row share and the whole image, alternating libraries
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1 || exit 1
for i in 1 2; do
  for lib in libhippt libv_prio1 libv_prio2; do
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/drain_export_ab.py --scene cornell34 --strides 8,1 --passes 1 --settings 0:0 > gpurun_out/r4a/cornell_${lib}_$i.jsonl || exit 1
  done
done
for lib in libhippt libv_prio1 libv_prio2; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/drain_export_ab.py --scene blob70k --strides 8,1 --passes 1 --steps 3 --settings 0:0 > gpurun_out/r4a/blob_${lib}.jsonl || exit 1
done
