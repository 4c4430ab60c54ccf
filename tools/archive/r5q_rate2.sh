# round 5: the small batch's interior rate — rate timelines (HIPPT_DEBUG_RATE build)
# of the whole image (64 spp), the 1/8 share in one launch of 512 spp (the same samples), the share
# at 64 spp, and 8 chained 64-spp share batches (cap 8); whole image at 8 spp (the share's samples,
# contiguous rows)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5q
mkdir -p $O
HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 300 python -u tools/rate_timeline.py --scene cornell34 \
    --jobs 1:64:1,8:512:1,8:64:1,8:64:8,1:8:1 --bucket-us 50 28=1 30=8 > $O/rate.jsonl || exit 1
python3 - <<'PY'
import json
for line in open("gpurun_out/r5q/rate.jsonl"):
    j = json.loads(line)
    b = j["buckets"]
    n = len(b)
    lo, hi = int(n * 0.1), int(n * 0.8)
    r = [x["segs_per_us"] for x in b[lo:hi]]
    u = [x["lane_util"] for x in b[lo:hi]]
    w = [x["waves"] for x in b[lo:hi]]
    print(j["stride"], j["spp"], j["batches"], "trace_ms", j["trace_ms"], "gseg/s", j["gseg_per_s"],
          "interior seg/us %.2f lane %.3f waves %.0f" % (sum(r) / len(r), sum(u) / len(u), sum(w) / len(w)))
PY
