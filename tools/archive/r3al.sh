# r3al: LDS stack cap of spilling global-memory trees, 13 (default) vs 10/11, alternating, leaf-2 trees
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3al
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 4 stackcap=13,10,11,13,10,11,13,10,11 > gpurun_out/r3al/b.jsonl 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --width 3840 --height 2160 --spp 64 --steps 2 stackcap=13,10,13,10 > gpurun_out/r3al/b4k.jsonl 2>&1
