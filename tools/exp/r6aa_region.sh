# round 6: XCD region queues (libv_region, -DHIPPT_EXP_REGION_QUEUES: queue g hands out the g-th band
# of runs over every frame) against the default (queue g = every run over its own frames); blob70k,
# Cornell, random_scene whole images, two alternating passes; then the item-order parity tests on the
# variant -> gpurun_out/r6aa/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6aa
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so qt-raytracer_amd/libv_region.so > $O/libs.sha256
for pass in 1 2; do
  for lib in default region; do
    if [ $lib = default ]; then unset HIPPT_LIB; else export HIPPT_LIB=qt-raytracer_amd/libv_$lib.so; fi
    for sc in blob70k cornell34 random_scene; do
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off > $O/${sc}_${lib}_p$pass.json 2> $O/${sc}_${lib}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${sc}_${lib}_p$pass.json'));print('$sc $lib $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
    done
  done
done
export HIPPT_LIB=qt-raytracer_amd/libv_region.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "order or tile or chain or headline" > $O/pytest_region.log 2>&1 || { tail -20 $O/pytest_region.log; exit 1; }
tail -2 $O/pytest_region.log
echo REGION_DONE
