# round 5 final library: GPU suite + smoke, then the profiles, then the bench lines and rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/exp/r5u_suite.sh && bash tools/exp/r5v_profiles.sh && bash tools/exp/r5w_bench.sh
