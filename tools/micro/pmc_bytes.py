#!/usr/bin/env python3
"""Per-width factors of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 (tools/micro/pmc_bytes.hip).

usage: tools/micro/pmc_bytes.py DIR  (DIR holds bytes.jsonl = the program's stdout, and the
rocprofv3 --pmc runs fetch/ and write/; tools/micro/pmc_bytes.sh makes them on the GPU box)

factor = bytes the kernel moves / counter bytes (KiB x 1024): multiply a counter by the factor of
its access width to get bytes.  Prints one JSON object with the factors per kernel."""
import csv
import glob
import json
import os
import sys

READS = {"ld_f3": 1.0, "ld_f3_fr": 1.0, "ld_f4": 1.0, "ld_row": 1.0, "rmw_f4": 0.5}
WRITES = {"st_f3": 1.0, "st_f4": 1.0, "rmw_f4": 0.5}


def counters(path, name):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out[r["Kernel_Name"].split("(")[0].strip()] = float(r["Counter_Value"]) * 1024
    return out


def main():
    d = sys.argv[1]
    moved = {}
    for line in open(os.path.join(d, "bytes.jsonl")):
        if line.startswith("{"):
            j = json.loads(line)
            moved[j["kernel"]] = j
    fetch = counters(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(d, "write"), "WRITE_SIZE")
    res = {}
    for k, j in moved.items():
        r = {"what": j["what"], "bytes": j["bytes"]}
        if k in READS and fetch.get(k):
            r["fetch_counter_bytes"] = fetch[k]
            r["fetch_factor"] = round(j["bytes"] * READS[k] / fetch[k], 4)
        if k in WRITES and write.get(k):
            r["write_counter_bytes"] = write[k]
            r["write_factor"] = round(j["bytes"] * WRITES[k] / write[k], 4)
        res[k] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
