# r5z: Cornell node exit x wave threshold x leaf exit around the new optimum (order on)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5z
mkdir -p $T
timeout -k 10 500 python tools/sweep.py --scene cornell34 --steps 5 nodeexit=16,20,24,28,32 wave=20,24,28,32 leafexit=4,8 > $T/sweep_cornell.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 5 order=0 nodeexit=32,48 wave=16,24 > $T/sweep_cornell_noorder.txt 2>&1
echo "r5z rc=$?"
