# round 5: the interior rate inside a group launch — 10 share batches (the first
# launch takes 2, then one group of 8), buckets 2.5-6.5 ms belong to the group alone; against the
# whole image and the share as one 512-spp batch
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ah
mkdir -p $O
HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 300 python -u tools/rate_timeline.py --scene cornell34 \
    --jobs 1:64:1,8:512:1,8:64:10 --bucket-us 50 28=1 > $O/rate.jsonl || exit 1
python3 - <<'PY'
import json
for line in open("gpurun_out/r5ah/rate.jsonl"):
    j = json.loads(line)
    b = j["buckets"]
    n = len(b)
    if j["batches"] > 1:
        win = [x for x in b if 2500 <= x["t_us"] < 6500]
        tag = "group window 2.5-6.5 ms"
    else:
        win = b[int(n * 0.1):int(n * 0.8)]
        tag = "10-80%"
    r = sum(x["segs_per_us"] for x in win) / len(win)
    u = sum(x["lane_util"] for x in win) / len(win)
    print(j["stride"], j["spp"], j["batches"], tag, "segs/us %.2f lane %.3f" % (r, u), "trace_ms", j["trace_ms"])
PY
