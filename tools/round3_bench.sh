# tools/round3_bench.sh TAG — ON THE GPU BOX: rocprof kernel-trace + PMC profiles of the two
# headline workloads (BASELINE configs[1], configs[2]) and every BASELINE bench line
# (configs[1..4] via bench.py --preset, plus the reference app's random_scene and cornell_mixed)
# and the legacy-ABI timing, into gpurun_out/TAG/ and gpurun_out/prof_TAG_*/.  Summaries are
# made locally afterwards: python tools/prof_summary.py TAG_cornell (and TAG_blob).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
T=gpurun_out/$TAG
mkdir -p $T
B="timeout -k 10 300 python3 bench.py"
bash tools/profile.sh ${TAG}_cornell && \
bash tools/profile.sh ${TAG}_blob --preset config3 && \
$B > $T/config2_cornell.json 2> $T/config2_cornell.err && \
$B --preset config3 > $T/config3_blob.json 2> $T/config3_blob.err && \
$B --preset config4 --steps 2 --warmup 1 --cpu-baseline off > $T/config4_blob4k.json 2> $T/config4_blob4k.err && \
$B --preset config5 --cpu-baseline off > $T/config5_blob_wavefront.json 2> $T/config5_blob_wavefront.err && \
$B --scene random_scene --cpu-baseline off > $T/random_scene.json 2> $T/random_scene.err && \
$B --scene cornell_mixed --cpu-baseline off > $T/cornell_mixed.json 2> $T/cornell_mixed.err && \
timeout -k 10 200 python3 tools/legacy_abi_bench.py > $T/legacy_abi.json 2> $T/legacy_abi.err
echo "round3_bench $TAG rc=$?"
