# round 4: GPU suite, the tail chunk (kTailChunk 64 default / 128 / 256) A/B, the wavefront sort A/B
set -o pipefail
mkdir -p gpurun_out/r4g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g/pytest.log 2>&1 || exit 1
for i in 1 2; do
  for lib in libhippt libv_tc128 libv_tc256; do
    HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 120 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 28=1 > gpurun_out/r4g/cornell_${lib}_$i.jsonl || exit 1
  done
done
for lib in libhippt libv_tc128 libv_tc256; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 150 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1,8 28=1 > gpurun_out/r4g/blob_${lib}.jsonl || exit 1
done
for i in 1 2; do
  for k in 0 3 6; do
    timeout -k 10 200 python -u bench.py --preset config5 --steps 5 --warmup 1 --cpu-baseline off --option WAVEFRONT_SORT=$k > gpurun_out/r4g/wf_sort${k}_$i.json 2> gpurun_out/r4g/wf_sort${k}_$i.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for k in 0 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g/prof_wf$k -o wf -- python3 -u bench.py --preset config5 --steps 2 --warmup 1 --cpu-baseline off --option WAVEFRONT_SORT=$k > gpurun_out/r4g/prof_wf$k.log 2>&1 || exit 1
done
timeout -k 10 1000 bash tools/profile.sh r4g_cornell > gpurun_out/r4g/profile.log 2>&1 || exit 1
