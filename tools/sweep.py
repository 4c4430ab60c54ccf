#!/usr/bin/env python3
"""Option sweep in one process (GPU box): Msamples/s per libhippt option setting.

usage: python tools/sweep.py [--scene cornell34] [--steps 3] KEY=v1,v2 [KEY=...]
keys: wave (HIPPT_OPT_WAVE_THRESHOLD), chunk, scratch (MB), bpc (blocks per CU), lds, mode, slots,
      leaf (max primitives per BVH leaf), tcost (SAH traversal cost x100)
Each combination: one warmup step, then `steps` timed steps; prints one JSON line each.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))

import hippt  # noqa: E402
from hippt import scenes  # noqa: E402

KEYS = {"wave": hippt.OPT_WAVE_THRESHOLD, "chunk": hippt.OPT_CHUNK, "scratch": hippt.OPT_SCRATCH_MB,
        "bpc": hippt.OPT_BLOCKS_PER_CU, "lds": hippt.OPT_LDS_SCENE, "mode": hippt.OPT_PATH_MODE,
        "slots": hippt.OPT_WAVEFRONT_SLOTS, "leaf": hippt.OPT_BVH_LEAF, "tcost": hippt.OPT_BVH_TRAVERSAL_COST,
        "depth": hippt.OPT_BVH_MAX_DEPTH, "leafexit": hippt.OPT_LEAF_EXIT,
        "nodeexit": hippt.OPT_NODE_EXIT, "sah": hippt.OPT_BVH_SAH,
        "width": hippt.OPT_BVH_WIDTH, "stackcap": hippt.OPT_STACK_CAP,
        "quant": hippt.OPT_BVH_QUANT, "top": hippt.OPT_LDS_TOP_NODES,
        "collapse": hippt.OPT_BVH_COLLAPSE, "ncost": hippt.OPT_BVH_NODE_COST, "leaf4": hippt.OPT_BVH_LEAF4,
        "rngtab": hippt.OPT_RNG_TABLE, "pool": hippt.OPT_CAMERA_POOL, "fuse": hippt.OPT_FUSE_COMBINE,
        "order": hippt.OPT_ITEM_ORDER, "tile": hippt.OPT_PIXEL_TILE, "chain": hippt.OPT_CHAIN}
REUPLOAD = {"leaf", "tcost", "depth", "sah", "collapse", "ncost", "leaf4"}  # build parameters: take effect at the next upload


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--blob", default=None, help="NU,NV: blob70k's walls + a blob of NU x NV quads")
    ap.add_argument("--count", action="store_true", help="report node visits / primitive tests per segment")
    ap.add_argument("--prewarm-ms", type=float, default=200.0,
                    help="untimed whole steps first (the GPU's clocks ramp over ~20 ms, DESIGN.md §6)")
    ap.add_argument("grid", nargs="*")
    a = ap.parse_args()
    axes = []
    for g in a.grid:
        k, vs = g.split("=")
        axes.append([(k, int(v)) for v in vs.split(",")])
    pt = hippt.PathTracer()
    pt.setDevices([0])
    sc = scenes.get_scene(a.scene)
    if a.blob:
        nu, nv = map(int, a.blob.split(","))
        sc = scenes.blob_scene(nu, nv)
        a.scene = f"blob{nu}x{nv}"
    pt.uploadMesh(sc)
    if a.prewarm_ms > 0:
        if not pt.initialize(a.width, a.height):
            raise SystemExit(pt.lastError())
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < a.prewarm_ms:
            pt.renderFrames(a.spp, a.depth, copy=False)
    for combo in itertools.product(*axes) if axes else [()]:
        for k, v in combo:
            pt.setOption(KEYS[k], v)
        if any(k in REUPLOAD for k, _ in combo):
            pt.uploadMesh(sc)
        if not pt.initialize(a.width, a.height):
            raise SystemExit(pt.lastError())
        pt.renderFrames(a.spp, a.depth, copy=False)
        extra = {}
        if a.count:
            pt.resetStats()
            pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 1)
            pt.renderFrames(a.spp, a.depth, copy=False)
            pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 0)
            c = pt.stats()
            extra = {"visits_per_seg": round(c["nodeVisits"] / c["segments"], 3),
                     "tests_per_seg": round(c["triTests"] / c["segments"], 3), "triangles": int(sc.num_tris)}
        pt.resetStats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            pt._lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
        pt.synchronize()
        dt = time.perf_counter() - t0
        st = pt.stats()
        print(json.dumps({"scene": a.scene, **dict(combo), "msamples_s": round(st["segments"] / dt / 1e6, 1),
                          "trace_ms_step": round(st["traceMs"] / a.steps, 3),
                          "combine_ms_step": round(st["combineMs"] / a.steps, 3),
                          "launches_step": st["traceLaunches"] // a.steps, "bvh_nodes": st["bvhNodes"],
                          "bvh_depth": st["bvhDepth"],
                          "lds_top_bytes": pt._lib.hipptGetOption(hippt.INFO_LDS_TOP_BYTES),
                          "blocks_per_cu": pt._lib.hipptGetOption(hippt.INFO_BLOCKS_PER_CU), **extra}), flush=True)


if __name__ == "__main__":
    main()
