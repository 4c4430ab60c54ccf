# s7b: half-plane nodes with aligned per-octant rows: parity cases, then A/B against float nodes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7b
mkdir -p $O
bash tools/gpu_tests.sh s7b "lds_top_of_tree or bvh_width_and_stack or fuzz_scene_matches_oracle" && \
timeout -k 10 200 python -u tools/sweep.py --scene blob70k --steps 3 quant=0,3,0,3 > $O/ab_half_blob70k.txt 2>&1 && \
timeout -k 10 200 python -u tools/sweep.py --scene random_scene --steps 3 quant=0,3,0,3 > $O/ab_half_random.txt 2>&1
echo "s7b rc=$?"
