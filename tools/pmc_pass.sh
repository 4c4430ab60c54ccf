#!/bin/bash
# tools/pmc_pass.sh NAME "COUNTERS" [bench args...] — one extra rocprofv3 --pmc pass over a short
# bench run, ON THE GPU BOX; output in gpurun_out/pmc_NAME/.  Counter limits per pass: 8 SQ,
# 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM.
set -euo pipefail
NAME=${1:?name}
CTRS=${2:?counters}
shift 2
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_$NAME
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -T --output-format csv -d "$OUT" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "pmc $NAME done"
