# r3o: kernel trace of the wavefront path (blob70k 1080p/64 spp): per-kernel time split
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r3o/kt -o run -- \
    python3 bench.py --scene blob70k --path-mode wavefront --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r3o/wf.json 2> gpurun_out/r3o/wf.err
