# s7k: hand-off frames of hipptRenderFramesPresent written by the frame's kernel (zero copy):
# full GPU suite, then both app paths' per-frame cost
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7k
mkdir -p $O
bash tools/gpu_tests.sh s7k && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy_abi_1080p.err && \
timeout -k 10 120 python -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p_p2.json 2> $O/legacy_abi_1080p_p2.err
echo "s7k rc=$?"
