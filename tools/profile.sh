#!/bin/bash
# tools/profile.sh TAG [bench args...] — run ON THE GPU BOX (via gpurun).
#
# 1. rocprofv3 --kernel-trace --stats over the driver's bench run (20 steps after 5) -> gpurun_out/prof_TAG/kt
# 2. separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ counters) -> gpurun_out/prof_TAG/pmc*
#    (one TCC counter group per pass: FETCH_SIZE and WRITE_SIZE do not fit together)
# Every step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
shift
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
ARGS=(--steps 20 --warmup 5 --cpu-baseline off "$@")
sha256sum qt-raytracer_amd/libhippt.so > "$OUT/lib.sha256"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -T --output-format csv -d "$OUT/pmc_sq" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/pmc_sq.json" 2> "$OUT/pmc_sq.err"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/pmc_sq2" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/pmc_sq2.json" 2> "$OUT/pmc_sq2.err" || echo "pmc_sq2 pass failed (counter set)" >&2
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/pmc_ta" -o run -- \
    python3 bench.py "${ARGS[@]}" > "$OUT/pmc_ta.json" 2> "$OUT/pmc_ta.err" || echo "pmc_ta pass failed (counter set)" >&2
echo "profile $TAG done"
