# s7p: half-precision nodes built and uploaded on first use: the tests that use them
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh s7p "lds_top_of_tree or bvh_width_and_stack or fuzz_scene or wavefront_node_formats"
echo "s7p rc=$?"
