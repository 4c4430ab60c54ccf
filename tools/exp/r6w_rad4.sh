# round 6: the partial-line write-back A/B: radiance as one aligned 16-byte store per
# sample (libv_rad4, -DHIPPT_RAD_FLOATS=4) against the 12-byte store; blob70k and Cornell whole
# images, two alternating passes, then a WRITE_SIZE and a FETCH_SIZE pass of each on blob70k -> gpurun_out/r6w/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6w
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so qt-raytracer_amd/libv_rad4.so > $O/libs.sha256
for pass in 1 2; do
  for lib in default rad4; do
    if [ $lib = default ]; then unset HIPPT_LIB; else export HIPPT_LIB=qt-raytracer_amd/libv_$lib.so; fi
    for sc in blob70k cornell34; do
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off > $O/${sc}_${lib}_p$pass.json 2> $O/${sc}_${lib}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${sc}_${lib}_p$pass.json'));print('$sc $lib $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
    done
  done
done
for lib in default rad4; do
  if [ $lib = default ]; then unset HIPPT_LIB; else export HIPPT_LIB=qt-raytracer_amd/libv_$lib.so; fi
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d $O/pmc_${lib}_$c -o run -- \
      python3 bench.py --scene blob70k --steps 3 --warmup 1 --cpu-baseline off > $O/pmc_${lib}_$c.json 2> $O/pmc_${lib}_$c.err || exit 1
  done
done
echo RAD4_DONE
