# r3aj: loop-exit re-sweep with the leaf-2 trees (leaf exit x node exit), two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aj
S="timeout -k 10 300 python tools/sweep.py --steps 3"
for p in 1 2; do
$S --scene cornell34 leafexit=4,2,8 nodeexit=48,40,56 >> gpurun_out/r3aj/c.jsonl 2>&1 && \
$S --scene blob70k leafexit=17,12,22 nodeexit=48,40,56 >> gpurun_out/r3aj/b.jsonl 2>&1 || exit 1
done
