# round 5 final: rocprofv3 kernel trace + PMC passes of the headline bench lines (Cornell configs[1],
# blob70k configs[2]) on the final library -> gpurun_out/prof_r5v{,_blob}/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh r5v || exit 1
bash tools/profile.sh r5v_blob --scene blob70k || exit 1
echo PROFILES_DONE
