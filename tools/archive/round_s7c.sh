# s7c: rocprof kernel trace + PMC passes of blob70k (configs[2]) with half-precision planes
# (HIPPT_OPT_BVH_QUANT 3), to compare TA busy / VALU issue with the float-node profile (r6q)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh s7c_blob_half --preset config3 --option BVH_QUANT=3
echo "s7c rc=$?"
