# round 6: blob70k's tree build at the final traversal thresholds (tools/sweep.py; build options take
# effect at the re-upload): 4-wide collapse greedy / SAH-optimal x node cost x 4-wide leaf size, and the
# SAH traversal cost; two passes -> gpurun_out/r6av/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6av
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 400 python3 -u tools/sweep.py --scene blob70k --steps 5 collapse=0,1 ncost=150,200,300 leaf4=2,4 > $O/blob_collapse_p$pass.jsonl 2> $O/blob_collapse_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 tcost=70,100,140 leaf=2,3 > $O/blob_sah_p$pass.jsonl 2> $O/blob_sah_p$pass.err || exit 1
done
echo BUILD_DONE
