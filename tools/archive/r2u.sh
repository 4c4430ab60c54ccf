# r2u: share of node visits served by the LDS top of the tree (counting builds), blob70k
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2u
for k in 5 21 85 341; do
  timeout -k 10 60 python tools/phase_profile.py --scene blob70k --spp 4 top=$k stackcap=13 > gpurun_out/r2u/top$k.json || exit 1
done
timeout -k 10 60 python tools/phase_profile.py --scene random_scene --spp 4 top=28 > gpurun_out/r2u/random_top28.json
