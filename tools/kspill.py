#!/usr/bin/env python3
"""Spill census of one kernel in a hipcc -S device assembly file: SGPR lane spills (v_writelane),
their reloads (v_readlane), VGPR scratch spills/reloads, and the static instruction count.
usage: tools/kspill.py build_hippt_kernels.s PATTERN [PATTERN ...]  (substring of the mangled name)"""
import re
import sys

text = open(sys.argv[1]).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(text) if re.match(r"^_Z\S+:", l)]
for pat in sys.argv[2:]:
    for i, name in starts:
        if pat not in name:
            continue
        j = i
        while not text[j].strip().startswith(".Lfunc_end"):
            j += 1
        body = [l.strip() for l in text[i:j]]
        ins = [l for l in body if l and not l.startswith((".", ";")) and not l.endswith(":")]
        c = lambda p: sum(1 for l in ins if l.startswith(p))
        print(f"{name[-60:]}: {len(ins)} instr, writelane {c('v_writelane')}, readlane {c('v_readlane')}, "
              f"scratch_store {c('scratch_store')}, scratch_load {c('scratch_load')}, v_ {c('v_')}, s_ {c('s_')}")
