# round 5: the app's own path (cudaPathTracerRender per frame, hipptRenderFramesPresent) on the
# final library
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ai
mkdir -p $O
timeout -k 10 300 python3 tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy.err || { tail -5 $O/legacy.err; exit 1; }
cat $O/legacy_abi_1080p.json
