# round 6: the GPU suite once more on the final library, on another box (the round-5 failure was
# box-dependent) -> gpurun_out/r6bj/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6bj
sha256sum qt-raytracer_amd/libhippt.so > gpurun_out/r6bj/lib.sha256
bash tools/gpu_tests.sh r6bj
