#!/usr/bin/env python3
"""Per-phase SIMD efficiency of the mesh megakernel (counting build), GPU box.

usage: python tools/phase_profile.py [--scene S] [--spp N] [KEY=v ...]
Prints one JSON object: wave-level / lane-level passes per phase and per segment.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))

import hippt  # noqa: E402
from hippt import scenes  # noqa: E402

KEYS = {"wave": hippt.OPT_WAVE_THRESHOLD, "chunk": hippt.OPT_CHUNK, "lds": hippt.OPT_LDS_SCENE,
        "width": hippt.OPT_BVH_WIDTH, "stackcap": hippt.OPT_STACK_CAP, "leafexit": hippt.OPT_LEAF_EXIT,
        "nodeexit": hippt.OPT_NODE_EXIT, "quant": hippt.OPT_BVH_QUANT,
        "top": hippt.OPT_LDS_TOP_NODES, "collapse": hippt.OPT_BVH_COLLAPSE,
        "ncost": hippt.OPT_BVH_NODE_COST, "pool": hippt.OPT_CAMERA_POOL}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("opts", nargs="*")
    a = ap.parse_args()
    pt = hippt.PathTracer()
    pt.setDevices([0])
    for o in a.opts:
        k, v = o.split("=")
        pt.setOption(KEYS[k], int(v))
    pt.uploadMesh(scenes.get_scene(a.scene))
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 1)
    if not pt.initialize(a.width, a.height):
        raise SystemExit(pt.lastError())
    pt.resetStats()
    pt.renderFrames(a.spp, a.depth, copy=False)
    c = pt.counters()
    segs = c["segments"]
    for name in hippt.PathTracer.PHASES:
        c[name]["wave_per_seg"] = round(c[name]["wave"] / segs, 4)
        c[name]["lane_per_seg"] = round(c[name]["lane"] / segs, 4)
    print(json.dumps({"scene": a.scene, "opts": a.opts, **c}, indent=1))


if __name__ == "__main__":
    main()
