#!/usr/bin/env python3
"""Latency floor of the launch's tail: kernel time of tiny jobs (one image row, a few frames), where
the launch lasts as long as its longest path, against the segments of that path's row."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell34"
opts = [tuple(int(x) for x in o.split("=")) for o in sys.argv[2:]]
pt = hippt.PathTracer()
pt.setDevices([0])
for k, v in opts:
    pt.setOption(k, v)
pt.setRowRange(540, 541)
pt.uploadMesh(scenes.get_scene(scene))
assert pt.initialize(1920, 1080)
for spp in (1, 1, 2, 4, 8, 16):
    pt.resetStats()
    for _ in range(5):
        pt._lib.hipptRenderFramesAsync(0, spp, 8, None)
    pt.synchronize()
    st = pt.stats()
    print(json.dumps({"scene": scene, "rows": 1, "spp": spp, "trace_ms": round(st["traceMs"] / 5, 4),
                      "segments": st["segments"] // 5, "samples": st["pixelSamples"] // 5}), flush=True)
