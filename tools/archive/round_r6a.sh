# r6a: Cornell loop exits continued (node exit down to 0 = leaf loop until no lane holds a leaf)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6a
mkdir -p $T
timeout -k 10 500 python tools/sweep.py --scene cornell34 --steps 5 nodeexit=0,4,8,12,16 wave=20,24,28 leafexit=8,12,16 > $T/sweep_cornell.txt 2>&1
echo "r6a rc=$?"
