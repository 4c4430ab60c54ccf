# r5y: Cornell node exit x wave threshold x chunk, finer, under the sample-length order
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r5y
mkdir -p $T
timeout -k 10 400 python tools/sweep.py --scene cornell34 --steps 5 nodeexit=32,36,40,44 wave=16,20,24 chunk=256,512 > $T/sweep_cornell.txt 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 nodeexit=32,40,48 wave=24,32,40 > $T/sweep_blob.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell_mixed --steps 4 nodeexit=40,48 wave=16,20 > $T/sweep_mixed.txt 2>&1
echo "r5y rc=$?"
