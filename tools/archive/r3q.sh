# r3q: blob70k / random_scene LDS stack cap sweep (the rest of the LDS budget goes to the top of the tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3q
S="timeout -k 10 200 python tools/sweep.py"
$S --scene blob70k --steps 3 stackcap=6,8,10,13,16 > gpurun_out/r3q/b_cap.jsonl 2>&1 && \
$S --scene random_scene --steps 3 stackcap=6,8,10,13,16 > gpurun_out/r3q/r_cap.jsonl 2>&1
