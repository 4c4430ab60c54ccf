#!/usr/bin/env python3
"""Spill census of one kernel in a hipcc -S device assembly file: SGPR lane spills (v_writelane),
their reloads (v_readlane), VGPR scratch spills/reloads (with the loop depth of the block each sits
in, from LLVM's '; in Loop: ... Depth=N' block comments) and the static instruction count.
usage: tools/kspill.py build_hippt_kernels.s PATTERN [PATTERN ...]  (substring of the mangled name)"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(text) if re.match(r"^_Z\S+:", l)]
for pat in sys.argv[2:]:
    for i, name in starts:
        if pat not in name:
            continue
        j = i
        while not text[j].strip().startswith(".Lfunc_end"):
            j += 1
        depth = 0
        ins = []
        for l in text[i:j]:
            s = l.strip()
            m = re.search(r"Depth=(\d+)", s)
            if re.match(r"^(\.LBB|; %bb)", s):
                depth = int(m.group(1)) if m else 0
                continue
            if s and not s.startswith((".", ";")) and not s.endswith(":"):
                ins.append((s, depth))
        c = lambda p: sum(1 for s, _ in ins if s.startswith(p))
        sd = Counter(d for s, d in ins if s.startswith("scratch_"))
        print(f"{name[-48:]}: {len(ins)} instr, writelane {c('v_writelane')}, readlane {c('v_readlane')}, "
              f"scratch {c('scratch_store')}st/{c('scratch_load')}ld by loop depth {dict(sorted(sd.items()))}")
