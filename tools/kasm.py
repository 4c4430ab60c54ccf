#!/usr/bin/env python3
"""One kernel's body from a hipcc -S device assembly file, with instruction counts per class.

usage: python tools/kasm.py ASM.s SUBSTRING [--out body.s]
SUBSTRING picks the kernel by its mangled name, e.g. 'mesh_kernelILb0ELb1ELb0ELb1ELb0ELb0ELb1ELb0ELb0E'
(the Cornell kernel: LDS scene, packed keys, camera pool).
"""
import argparse
import collections
import re


def body(path, sub):
    out, name, inside = [], None, False
    for line in open(path):
        m = re.match(r"^(\S+):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and sub in m.group(1):
            name, inside = m.group(1), True
            continue
        if inside:
            if re.match(r"\s*s_endpgm", line) or re.match(r"^\.Lfunc_end", line):
                out.append(line)
                break
            out.append(line)
    return name, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("sub")
    ap.add_argument("--out")
    a = ap.parse_args()
    name, lines = body(a.asm, a.sub)
    if name is None:
        raise SystemExit(f"no kernel matching {a.sub}")
    cls = collections.Counter()
    for line in lines:
        m = re.match(r"\s+([a-z_0-9]+)", line)
        if not m or line.lstrip().startswith(";"):
            continue
        op = m.group(1)
        if op.startswith("v_"):
            cls["valu"] += 1
        elif op.startswith("s_"):
            cls["salu/smem/branch"] += 1
        elif op.startswith("ds_"):
            cls["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cls["vmem"] += 1
        cls["total"] += 1
    print(name)
    print(dict(cls))
    if a.out:
        open(a.out, "w").writelines(lines)


if __name__ == "__main__":
    main()
