# round 6: compiler-flag variants of the kernels (libv_{unclhrp,cluslo,bias0,bias100,nounroll}: LLVM
# AMDGPU rescheduling stages off, the occupancy/latency metric bias 0 and 100, -fno-unroll-loops)
# against the default; Cornell and blob70k whole images, two alternating passes -> gpurun_out/r6ac/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ac
mkdir -p $O
for pass in 1 2; do
  for lib in default unclhrp cluslo bias0 bias100 nounroll; do
    if [ $lib = default ]; then unset HIPPT_LIB; else export HIPPT_LIB=qt-raytracer_amd/libv_$lib.so; fi
    for sc in cornell34 blob70k; do
      timeout -k 10 200 python3 bench.py --scene $sc --steps 20 --warmup 5 --cpu-baseline off > $O/${sc}_${lib}_p$pass.json 2> $O/${sc}_${lib}_p$pass.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${sc}_${lib}_p$pass.json'));print('$sc $lib $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
    done
  done
done
echo FLAGS_DONE
