# round 6: headline profiles on the library with automatic 8x8 tile runs (Cornell configs[1], blob70k
# configs[2]) and blob70k with row runs (the TA / FETCH_SIZE pair for the tile A/B) -> gpurun_out/prof_r6g*/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh r6g || exit 1
bash tools/profile.sh r6g_blob --scene blob70k || exit 1
bash tools/profile.sh r6g_blob_rows --scene blob70k --option PIXEL_TILE=0 || exit 1
echo PROFILES_DONE
