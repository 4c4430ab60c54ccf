#!/usr/bin/env python3
"""Times the path the Qt app drives: one cudaPathTracerRender call per frame,
each a 1-spp launch followed by a blocking full-frame D2H copy into the library's host buffer
(CudaPathTracerKernel.cu:239-276; the app's loop, RayTracerFboItem.cpp:516-575), at 1920x1080,
maxDepth 10 (the app's default depth, RayTracerFboItem.h:109-113), for the reference's built-in
4-sphere scene and the Cornell-34 mesh; beside it hipptRenderFramesPresent (enqueue the frame +
a copy into one of two pinned hand-off frames, never wait) polled with hipptLatestFrame, as a
UI thread would.

Reports per variant: wall ms per frame (median and mean over --frames calls after --warmup), the
reference's own stats figure W*H*frames/wall (Mpixel-samples/s, RayTracerFboItem.cpp:554-569),
segments/s, and the device time per frame (kernel + combine from the library's HIP events), so
the host-side overhead per call is wall - device.  Prints one JSON object.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))

import hippt  # noqa: E402
from hippt import scenes  # noqa: E402


def run(lib, pt, scene, w, h, depth, frames, warmup, mode):
    if scene == "sphere4":
        pt.useBuiltinScene(hippt.SCENE_SPHERE4)
    else:
        pt.uploadMesh(scenes.get_scene(scene))
    if not pt.initialize(w, h):
        raise SystemExit(pt.lastError())
    err = ctypes.c_char_p()
    px = ctypes.POINTER(ctypes.c_uint)()
    times = []
    shown = 0
    pt.resetStats()
    for f in range(warmup + frames):
        if f == warmup:
            pt.resetStats()
            t_all = time.perf_counter()
        t0 = time.perf_counter()
        if mode == "legacy":
            ok = lib.cudaPathTracerRender(f, depth, ctypes.byref(px), ctypes.byref(err))
        else:
            ok = lib.hipptRenderFramesPresent(f, 1, depth, ctypes.byref(err))
            n = ctypes.c_int()
            if ok and lib.hipptLatestFrame(ctypes.byref(px), ctypes.byref(n), ctypes.byref(err)) and px:
                shown += 1 if f >= warmup else 0
        if not ok:
            raise SystemExit(err.value.decode() if err.value else "render failed")
        times.append(time.perf_counter() - t0)
    if mode == "present":
        if not lib.hipptSynchronize(ctypes.byref(err)):
            raise SystemExit(err.value.decode())
    wall = time.perf_counter() - t_all
    st = pt.stats()
    t = times[warmup:]
    d = {"scene": scene, "mode": mode, "width": w, "height": h, "max_depth": depth, "frames": frames,
         "wall_ms_per_frame_median": round(statistics.median(t) * 1e3, 4),
         "wall_ms_per_frame_mean": round(wall / frames * 1e3, 4),
         "reference_mpixel_samples_per_s": round(w * h * frames / wall / 1e6, 2),
         "msegments_per_s": round(st["segments"] / wall / 1e6, 2),
         "device_ms_per_frame": round((st["traceMs"] + st["combineMs"]) / frames, 4),
         "trace_launches": st["traceLaunches"], "combine_launches": st["combineLaunches"]}
    d["host_overhead_ms_per_frame"] = round(d["wall_ms_per_frame_mean"] - d["device_ms_per_frame"], 4)
    if mode == "present":
        d["frames_shown_without_waiting"] = shown
    return d


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--scenes", nargs="*", default=["sphere4", "cornell34"])
    ap.add_argument("--opt", action="append", default=[], help="KEY=VALUE hipptSetOption pair (numeric key)")
    a = ap.parse_args()
    lib = hippt.load_library()
    pt = hippt.PathTracer()
    pt.setDevices([0])
    for o in a.opt:
        k, v = o.split("=")
        assert lib.hipptSetOption(int(k), int(v)), o
    out = []
    for sc in a.scenes:
        for mode in ("legacy", "present"):
            out.append(run(lib, pt, sc, a.width, a.height, a.depth, a.frames, a.warmup, mode))
            print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    lib.cudaPathTracerShutdown()
    print(json.dumps({"tool": "tools/legacy_abi_bench.py", "results": out}))


if __name__ == "__main__":
    main()
