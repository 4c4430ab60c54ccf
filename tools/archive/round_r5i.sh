# r5i: is the lists-off kernel slower than HEAD's (r5h: Cornell 44.2 G vs 48.1 G in r5b)?  Same box,
# alternating libraries, both scenes
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5i
mkdir -p $T
for i in 1 2; do
  HIPPT_LIB=qt-raytracer_amd/libv_head.so timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 pool=-1 >> $T/ab_cornell.txt 2>&1 || exit 1
  timeout -k 10 100 python tools/sweep.py --scene cornell34 --steps 6 prim=0,1 >> $T/ab_cornell.txt 2>&1 || exit 1
done
for i in 1 2; do
  HIPPT_LIB=qt-raytracer_amd/libv_head.so timeout -k 10 100 python tools/sweep.py --scene blob70k --steps 6 pool=-1 >> $T/ab_blob.txt 2>&1 || exit 1
  timeout -k 10 100 python tools/sweep.py --scene blob70k --steps 6 prim=0,1 >> $T/ab_blob.txt 2>&1 || exit 1
done
echo "r5i done"
