# round 4: overlapped batches (measurement only) without fill/write kernels between the launches
set -o pipefail
mkdir -p gpurun_out/r4i
for i in 1 2; do
  for mode in seq pipe; do
    if [ $mode = pipe ]; then export HIPPT_PIPE=1; else unset HIPPT_PIPE; fi
    HIPPT_LIB=qt-raytracer_amd/libv_pipe.so timeout -k 10 120 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks 1,8 28=1 > gpurun_out/r4i/cornell_${mode}_$i.jsonl || exit 1
  done
done
unset HIPPT_PIPE
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
HIPPT_PIPE=1 HIPPT_LIB=qt-raytracer_amd/libv_pipe.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4i/prof -o pipe -- python3 -u tools/band_scaling.py --scene cornell34 --steps 10 --ranks 8 28=1 > gpurun_out/r4i/prof.log 2>&1 || exit 1
