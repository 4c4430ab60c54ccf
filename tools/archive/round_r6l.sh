# r6l: blob70k knobs with its camera pool on (the top of the tree is smaller now)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6l
mkdir -p $T
timeout -k 10 400 python tools/sweep.py --scene blob70k --steps 3 stackcap=8,10,12 wave=28,32,36 > $T/sweep_cap_wave.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 leafexit=12,17,22 nodeexit=32,48 > $T/sweep_exits.txt 2>&1
echo "r6l rc=$?"
