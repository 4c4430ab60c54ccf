#!/usr/bin/env python3
"""Summarise tools/ab.sh output files: mean Msamples/s per variant and the change vs the first.
usage: python tools/ab_summary.py gpurun_out/TAG/ab_*.txt"""
import json
import sys

for path in sys.argv[1:]:
    runs = {}
    for line in open(path):
        parts = line.split(" ", 2)
        if len(parts) < 3 or not parts[2].startswith("{"):
            continue
        runs.setdefault(parts[0], []).append(json.loads(parts[2])["msamples_s"])
    if not runs:
        print(path, "no results")
        continue
    names = list(runs)
    base = sum(runs[names[0]]) / len(runs[names[0]])
    out = []
    for n in names:
        m = sum(runs[n]) / len(runs[n])
        out.append(f"{n} {m:.0f} ({(m / base - 1) * 100:+.2f}%)")
    print(path.rsplit("/", 1)[-1], " | ".join(out))
