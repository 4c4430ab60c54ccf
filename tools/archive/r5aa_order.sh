# round 5: is the small batch's interior deficit the item order's? rate timelines with the order off
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5aa
mkdir -p $O
for io in 0 1; do
  HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 300 python -u tools/rate_timeline.py --scene cornell34 \
      --jobs 1:64:1,8:512:1,8:64:1,1:8:1 --bucket-us 50 28=$io 30=0 > $O/rate_io$io.jsonl || exit 1
done
python3 - <<'PY'
import json
for io in (0, 1):
    for line in open(f"gpurun_out/r5aa/rate_io{io}.jsonl"):
        j = json.loads(line)
        b = j["buckets"]
        n = len(b)
        lo, hi = int(n * 0.1), int(n * 0.8)
        r = [x["segs_per_us"] for x in b[lo:hi]]
        u = [x["lane_util"] for x in b[lo:hi]]
        print("order", io, j["stride"], j["spp"], "trace_ms", j["trace_ms"], "gseg/s", j["gseg_per_s"],
              "interior %.2f lane %.3f" % (sum(r) / len(r), sum(u) / len(u)))
PY
