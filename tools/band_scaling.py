#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: time the row band an N-GPU run gives each rank
(rows [0, H/N)) and compare with 1/N of the full-image time.  Prints one JSON line per N.

usage: python tools/band_scaling.py [--scene cornell34] [--steps 5] [--ranks 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402
from hippt.distributed import row_band  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--all-bands", action="store_true", help="time every rank's rows (max = the N-GPU step)")
    ap.add_argument("--split", default="interleave", choices=["interleave", "bands"])
    ap.add_argument("--prewarm-ms", type=float, default=200.0, help="untimed GPU clock warm-up per job")
    ap.add_argument("opts", nargs="*", help="KEY=VALUE hipptSetOption pairs (numeric keys)")
    a = ap.parse_args()
    sc = scenes.get_scene(a.scene)
    full_ms = None
    jobs = [(n, r) for n in [int(x) for x in a.ranks.split(",")] for r in (range(n) if a.all_bands else [0])]
    for n, rank in jobs:
        pt = hippt.PathTracer()
        pt.setDevices([0])
        for o in a.opts:
            k, v = o.split("=")
            pt.setOption(int(k), int(v))
        if a.split == "interleave":
            pt.setRowInterleave(rank, n)
            nrows = len(range(rank, a.height, n))
        else:
            y0, y1 = row_band(rank, n, a.height)
            pt.setRowRange(y0, y1)
            nrows = y1 - y0
        pt.uploadMesh(sc)
        assert pt.initialize(a.width, a.height)
        lib = pt._lib
        # clock warm-up (as bench.py --prewarm-ms): whole steps for a.prewarm_ms of wall time
        t_warm = time.perf_counter()
        lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
        while (time.perf_counter() - t_warm) * 1e3 < a.prewarm_ms:
            for _ in range(4):
                lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
            pt.synchronize()
        pt.synchronize()
        pt.resetStats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
        pt.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        st = pt.stats()
        if full_ms is None:
            full_ms = ms * n
        print(json.dumps({"ranks": n, "rank": rank, "rows": nrows, "ms_per_step": round(ms, 3),
                          "trace_ms": round(st["traceMs"] / a.steps, 3), "combine_ms": round(st["combineMs"] / a.steps, 3),
                          "ideal_ms": round(full_ms / n, 3), "efficiency": round(full_ms / n / ms, 3)}), flush=True)
        pt.setRowRange(0, 0)  # also clears the interleave


if __name__ == "__main__":
    main()
