#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / scratch bytes from a hipcc -S device assembly file (spill check)."""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.match(r"\s*\.amdhsa_kernel\s+(\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    if cur is None:
        continue
    for key in ("private_segment_fixed_size", "next_free_vgpr", "next_free_sgpr"):
        m = re.match(rf"\s*\.amdhsa_{key}\s+(\d+)", line)
        if m:
            cur[key] = int(m.group(1))
    if re.match(r"\s*\.end_amdhsa_kernel", line):
        rows.append(cur)
        cur = None
for r in rows:
    n = re.sub(r"_ZN5hippt12_GLOBAL__N_1", "", r["name"])
    print(f"{r.get('next_free_vgpr', '?'):>4} vgpr {r.get('next_free_sgpr', '?'):>4} sgpr "
          f"{r.get('private_segment_fixed_size', '?'):>5} scratch  {n}")
