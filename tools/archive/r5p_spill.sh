# round 5: blob70k's spilled stack bottoms — the LDS stack cap (HIPPT_OPT_STACK_CAP)
# against time and DRAM write bytes (WRITE_SIZE per mesh_kernel launch; the 12-B/lane radiance
# stores are 1.59 GB of it, factor 1.0 per profiles/round5/pmc_bytes_factors.json)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p
mkdir -p $O
for cap in 10 13 16 19 24; do
  timeout -k 10 100 python -u tools/band_scaling.py --scene blob70k --steps 10 --ranks 1 28=1 18=$cap > $O/blob_cap$cap.jsonl || exit 1
  echo "cap $cap $(cat $O/blob_cap$cap.jsonl)"
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_cap$cap -o run -- \
      python3 tools/band_scaling.py --scene blob70k --steps 3 --ranks 1 28=1 18=$cap > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for cap in (10, 13, 16, 19, 24):
    vals = []
    for f in glob.glob(f"gpurun_out/r5p/pmc_cap{cap}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("mesh_kernel") and r["Counter_Name"] == "WRITE_SIZE":
                vals.append(float(r["Counter_Value"]) * 1024)
    print(cap, "launches", len(vals), "write GB per launch (last 3)", [round(v / 1e9, 3) for v in vals[-3:]])
PY
