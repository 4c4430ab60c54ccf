# round 5: the small batch's deficit — a big batch whose item order walks the cost spectrum 8 times
# (as a chain of 8 small batches does) against the default order walked once
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ad
mkdir -p $O
for lib in libv_rate libv_ratecyc; do
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 300 python -u tools/rate_timeline.py --scene cornell34 \
      --jobs 1:64:1,8:512:1 --bucket-us 50 28=1 30=0 > $O/rate_$lib.jsonl || exit 1
done
python3 - <<'PY'
import json
for lib in ("libv_rate", "libv_ratecyc"):
    for line in open(f"gpurun_out/r5ad/rate_{lib}.jsonl"):
        j = json.loads(line)
        b = j["buckets"]
        n = len(b)
        lo, hi = int(n * 0.1), int(n * 0.8)
        r = [x["segs_per_us"] for x in b[lo:hi]]
        u = [x["lane_util"] for x in b[lo:hi]]
        print(lib, j["stride"], j["spp"], "trace_ms", j["trace_ms"], "gseg/s", j["gseg_per_s"],
              "interior %.2f lane %.3f" % (sum(r) / len(r), sum(u) / len(u)))
PY
run() {  # name lib scene ranks opts...
  local name=$1 lib=$2 sc=$3 r=$4; shift 4
  HIPPT_LIB=qt-raytracer_amd/$lib.so timeout -k 10 100 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks $r "$@" > $O/$name.jsonl || exit 1
  echo "$name $(cat $O/$name.jsonl)"
}
for pass in 1 2; do
  for lib in libhippt libv_cyc8; do
    run p${pass}_${lib}_whole cornell34 1 28=1
    run p${pass}_${lib}_share512 cornell34 8 --spp 512 28=1 30=0
  done
done
