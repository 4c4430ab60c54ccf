#!/bin/bash
# tools/micro/pmc_bytes.sh TAG — ON THE GPU BOX: the calibration program under one FETCH_SIZE and one
# WRITE_SIZE rocprofv3 pass (one TCC counter group each), then the factors -> gpurun_out/TAG/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:?tag}
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run -- \
    ./tools/micro/pmc_bytes > "$OUT/bytes.jsonl" || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run -- \
    ./tools/micro/pmc_bytes > /dev/null || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o run -- \
    ./tools/micro/pmc_bytes > /dev/null || exit 1
python3 tools/micro/pmc_bytes.py "$OUT" > "$OUT/factors.json" && cat "$OUT/factors.json"
