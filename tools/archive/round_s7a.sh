# s7a: GPU suite with the half-plane node cases, then half (quant 3) against float nodes (quant 0)
# on blob70k and random_scene, node visits per segment of both, and the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7a
mkdir -p $O
bash tools/gpu_tests.sh s7a && \
timeout -k 10 200 python -u tools/sweep.py --scene blob70k --steps 3 quant=0,3,0,3 > $O/ab_half_blob70k.txt 2>&1 && \
timeout -k 10 200 python -u tools/sweep.py --scene random_scene --steps 3 quant=0,3,0,3 > $O/ab_half_random.txt 2>&1 && \
timeout -k 10 200 python -u tools/sweep.py --scene blob70k --steps 1 --count quant=0,3 > $O/count_half_blob70k.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "s7a rc=$?"
