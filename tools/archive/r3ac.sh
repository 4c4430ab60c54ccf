# r3ac: kernel traces of the wavefront path, partial (base) vs whole (full) 64-byte slot record writes
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ac
for v in base full base full; do
  HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r3ac/kt_$v -o run -- \
      python3 bench.py --scene blob70k --path-mode wavefront --steps 3 --warmup 1 --cpu-baseline off >> gpurun_out/r3ac/$v.json 2>> gpurun_out/r3ac/$v.err || exit 1
  cp gpurun_out/r3ac/kt_$v/run_kernel_stats.csv gpurun_out/r3ac/stats_$v.$RANDOM.csv
done
