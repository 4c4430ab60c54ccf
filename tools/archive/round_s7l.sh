# s7l: rocprof kernel trace + PMC passes of the headline (configs[1]) on the session's final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh s7l_cornell
echo "s7l rc=$?"
