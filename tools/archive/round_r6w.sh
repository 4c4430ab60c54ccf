# r6w: work-chunk size and wave threshold at a 1/8 Cornell share (the strong-scaling step)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6w
mkdir -p $T
L="timeout -k 10 100 python tools/launch_overhead.py --stride 8 --spp 32,64"
for i in 1 2; do
  for o in "4=256" "4=64" "4=128" "4=512" "2=16" "2=32" "2=8"; do
    echo "$o $($L $o 2>&1)" >> $T/share_knobs.txt || exit 1
  done
done
echo "r6w rc=$?"
