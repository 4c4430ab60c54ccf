#!/usr/bin/env python3
"""Fixed cost per launch of the mesh megakernel: kernel time of a 1/N-image row set against spp;
the intercept of the linear fit is the per-launch overhead (ramp-up + tail).

usage: python tools/launch_overhead.py [--scene cornell34] [--stride 8] [--spp 4,8,16,32,64]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--stride", type=int, default=8)
    ap.add_argument("--spp", default="4,8,16,32,64")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("opts", nargs="*", help="KEY=VALUE hipptSetOption pairs (numeric keys)")
    a = ap.parse_args()
    pt = hippt.PathTracer()
    pt.setDevices([0])
    for o in a.opts:
        k, v = o.split("=")
        pt.setOption(int(k), int(v))
    pt.setRowInterleave(0, a.stride)
    pt.uploadMesh(scenes.get_scene(a.scene))
    assert pt.initialize(1920, 1080)
    xs, ys = [], []
    for spp in [int(x) for x in a.spp.split(",")]:
        pt._lib.hipptRenderFramesAsync(0, spp, 8, None)
        pt.synchronize()
        pt.resetStats()
        for _ in range(a.steps):
            pt._lib.hipptRenderFramesAsync(0, spp, 8, None)
        pt.synchronize()
        ms = pt.stats()["traceMs"] / a.steps
        xs.append(spp)
        ys.append(ms)
    slope, icpt = np.polyfit(xs, ys, 1)
    print(json.dumps({"scene": a.scene, "stride": a.stride, "spp": xs, "trace_ms": [round(y, 4) for y in ys],
                      "ms_per_spp": round(slope, 5), "overhead_ms": round(icpt, 4)}))


if __name__ == "__main__":
    main()
