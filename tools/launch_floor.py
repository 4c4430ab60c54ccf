#!/usr/bin/env python3
"""Fixed cost of one megakernel launch: kernel time (events, traceMs per launch) of tiny jobs, from one
sample to a few image rows, at the automatic grid and at one block per CU, against the legacy
sphere4 kernel on one pixel (a plain launch).  One JSON line per job.

usage: python tools/launch_floor.py [--scenes cornell34,blob70k] [--calls 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402


def timed(pt, calls, spp, depth, legacy=False):
    lib = pt._lib
    for _ in range(3):
        (pt.renderFrame(depth) if legacy else lib.hipptRenderFramesAsync(0, spp, depth, None))
    pt.synchronize()
    pt.resetStats()
    for _ in range(calls):
        (pt.renderFrame(depth) if legacy else lib.hipptRenderFramesAsync(0, spp, depth, None))
    pt.synchronize()
    st = pt.stats()
    return st["traceMs"] / max(1, st["traceLaunches"]), st["segments"] // calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="cornell34,blob70k")
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--option", action="append", default=[], help="KEY=VALUE library option")
    a = ap.parse_args()
    pt = hippt.PathTracer()
    pt.setDevices([0])
    for kv in a.option:
        k, v = kv.split("=")
        pt.setOption(getattr(hippt, "OPT_" + k.upper()), int(v))
    pt.useBuiltinScene(hippt.SCENE_SPHERE4)
    assert pt.initialize(1, 1)
    ms, _ = timed(pt, a.calls, 1, 8, legacy=True)
    print(json.dumps({"job": "sphere4 1x1 1spp", "kernel_ms": round(ms, 4)}), flush=True)
    for name in a.scenes.split(","):
        pt.uploadMesh(scenes.get_scene(name))
        for bpc in (0, 1):
            pt.setOption(hippt.OPT_BLOCKS_PER_CU, bpc)
            for w, h, spp in ((1, 1, 1), (64, 1, 1), (1920, 1, 1), (1920, 8, 1), (1920, 8, 8), (1920, 135, 8)):
                assert pt.initialize(w, h), pt.lastError()
                ms, segs = timed(pt, a.calls, spp, 8)
                print(json.dumps({"job": f"{name} {w}x{h} {spp}spp", "blocks_per_cu": bpc,
                                  "active_blocks_per_cu": pt._lib.hipptGetOption(101),
                                  "kernel_ms": round(ms, 4), "segments": segs}), flush=True)
        pt.setOption(hippt.OPT_BLOCKS_PER_CU, 0)


if __name__ == "__main__":
    main()
