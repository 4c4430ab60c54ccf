# r3af: blob70k leaf-size sweep on the final kernels (max primitives per BVH leaf)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3af
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 --count leaf=4,2,3,6,4 > gpurun_out/r3af/b_leaf.jsonl 2>&1
