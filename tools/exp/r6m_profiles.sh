# round 6 final library, part 2: headline profiles (Cornell configs[1], blob70k configs[2]) -> gpurun_out/prof_r6m*/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh r6m || exit 1
bash tools/profile.sh r6m_blob --scene blob70k || exit 1
echo PROFILES_DONE
