#!/usr/bin/env python3
"""Per-wave timeline of one mesh-kernel launch (debug build with -DHIPPT_DEBUG_TIMELINE, run with
HIPPT_LIB=qt-raytracer_amd/libv_tl.so): wave start / queue-drained / end times in µs from the
first wave start, summarised as quantiles.

usage: python tools/timeline.py [--scene cornell34] [--stride 8] [--spp 64]
"""
import argparse
import ctypes
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
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--chunk", type=int, default=None)
    a = ap.parse_args()
    pt = hippt.PathTracer()
    pt.setDevices([0])
    if a.chunk:
        pt.setOption(hippt.OPT_CHUNK, a.chunk)
    pt.setRowInterleave(0, a.stride)
    pt.uploadMesh(scenes.get_scene(a.scene))
    assert pt.initialize(1920, 1080)
    for _ in range(2):
        pt._lib.hipptRenderFramesAsync(0, a.spp, 8, None)
        pt.synchronize()
    pt.resetStats()
    pt._lib.hipptRenderFramesAsync(0, a.spp, 8, None)
    pt.synchronize()
    kernel_ms = pt.stats()["traceMs"]
    fn = pt._lib.hipptDebugTimeline
    fn.restype = ctypes.c_int
    buf = np.zeros((65536, 8), np.uint64)
    n = fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 65536)
    t = buf[:n]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = lambda v: (v.astype(np.float64) - float(t0)) / 100.0  # 100 MHz
    q = lambda v: [round(float(np.quantile(v, p)), 1) for p in (0, 0.1, 0.5, 0.9, 0.99, 1)]
    drained = t[:, 1][t[:, 1] > 0]
    print(json.dumps({"scene": a.scene, "chunk": a.chunk, "stride": a.stride, "spp": a.spp, "waves": int(len(t)), "kernel_ms": round(kernel_ms, 3),
                      "start_us_q": q(us(t[:, 0])), "drained_us_q": q(us(drained)), "end_us_q": q(us(t[:, 2])),
                      "end_minus_drained_us_q": q((t[:, 2].astype(np.float64) - t[:, 1]) / 100.0),
                      "items_q": q(t[:, 3].astype(np.float64)),
                      "rounds_after_drain_q": q(t[:, 6].astype(np.float64)),
                      "lane_samples_after_drain_q": q(t[:, 7].astype(np.float64)),
                      "round_us_after_drain_q": q((t[:, 2].astype(np.float64) - t[:, 1]) / 100.0 / np.maximum(1, t[:, 6]))}))
    hw = t[:, 4].astype(np.int64)
    xcc = t[:, 5].astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 3
    late = us(t[:, 0]) > 0.1 * kernel_ms * 1e3
    ids = xcc * 1000 + se * 100 + sh * 50 + cu
    blk = np.nonzero(t[:, 0] > 0)[0] // 4
    print(json.dumps({"distinct_cus": int(len(np.unique(ids))), "distinct_xcc": int(len(np.unique(xcc))),
                      "distinct_se": int(len(np.unique(xcc * 8 + se))), "late_waves": int(late.sum()),
                      "late_blocks_by_xcd(blockIdx%8)": np.bincount(blk[late] % 8, minlength=8).tolist(),
                      "late_by_xcc": np.bincount(xcc[late], minlength=8).tolist(),
                      "waves_per_cu_max": int(np.bincount(np.unique(ids, return_inverse=True)[1]).max()),
                      "waves_per_cu_min": int(np.bincount(np.unique(ids, return_inverse=True)[1]).min())}))


if __name__ == "__main__":
    main()
