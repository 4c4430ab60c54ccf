# round 6 final library, part 2 (prewarm, cap 16 for global trees): headline profiles (Cornell configs[1], blob70k configs[2]) -> gpurun_out/prof_r6t*/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh r6t || exit 1
bash tools/profile.sh r6t_blob --scene blob70k || exit 1
echo PROFILES_DONE
