# round 6: the final library's headline lines on one more box (box-to-box spread; run once per gpurun
# call, each call a fresh box) -> gpurun_out/r6be_$TAG/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6be_${TAG:-x}
mkdir -p $O
for sc in cornell34 blob70k; do
  timeout -k 10 200 python3 bench.py --scene $sc --cpu-baseline off > $O/$sc.json 2> $O/$sc.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$sc.json'));print('$sc', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
done
echo BOX_DONE
