# r3am: spill-tree stack cap 10 — full GPU suite, then the global-memory-tree bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3am
B="timeout -k 10 300 python3 bench.py"
bash tools/gpu_tests.sh r3am && \
$B --scene blob70k > gpurun_out/r3am/blob.json 2> gpurun_out/r3am/err && \
$B --scene blob70k --width 3840 --height 2160 --spp 256 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r3am/blob4k.json 2>> gpurun_out/r3am/err && \
$B --scene blob70k --path-mode wavefront --cpu-baseline off > gpurun_out/r3am/blob_wf.json 2>> gpurun_out/r3am/err && \
$B --scene random_scene --cpu-baseline off > gpurun_out/r3am/random.json 2>> gpurun_out/r3am/err && \
bash tools/profile.sh r3am_blob --scene blob70k && python3 tools/prof_summary.py r3am_blob > /dev/null
