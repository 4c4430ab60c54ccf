# r3h: fused combine on/off, with and without non-temporal scratch traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
for v in fuse2 fusent; do
  for sc in blob70k cornell34; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python tools/sweep.py --scene $sc --steps 10 fuse=0,1 fuse=0,1 > gpurun_out/r3h/${v}_$sc.jsonl 2>&1 || exit 1
  done
done
