# round 4: the launch's fixed cost (tiny jobs, events and rocprof kernel trace) and configs[0] on the
# reference CPU tracer
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 120 python -u tools/launch_floor.py > gpurun_out/r4b/floor.jsonl 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof -o floor -- python3 -u tools/launch_floor.py --calls 10 > gpurun_out/r4b/floor_prof.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ref_cpu_config0.py > gpurun_out/r4b/ref_cpu_config0.jsonl 2>&1 || exit 1
