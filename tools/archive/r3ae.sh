# r3ae: per-dispatch PMC of the wavefront path (blob70k 1080p/64 spp): VALU / VMEM instructions and
# waves per wf_extend launch, to see why late (small) iterations cost more per ray
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ae
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T --output-format csv -d gpurun_out/r3ae/pmc -o run -- \
    python3 bench.py --scene blob70k --path-mode wavefront --steps 1 --warmup 0 --cpu-baseline off > gpurun_out/r3ae/wf.json 2> gpurun_out/r3ae/wf.err
