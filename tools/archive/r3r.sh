# r3r: wavefront launch trims (exact iteration count when the pool holds the batch; empty blocks of
# wf_shade / wf_generate leave before the block appends) — wavefront parity tests, bench, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3r
bash tools/gpu_tests.sh r3r "wavefront or counting or present or deferred" && \
timeout -k 10 300 python3 bench.py --scene blob70k --path-mode wavefront --cpu-baseline off > gpurun_out/r3r/wf.json 2> gpurun_out/r3r/wf.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r3r/kt -o run -- \
    python3 bench.py --scene blob70k --path-mode wavefront --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r3r/wf_kt.json 2> gpurun_out/r3r/wf_kt.err
