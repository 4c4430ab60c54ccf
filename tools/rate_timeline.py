#!/usr/bin/env python3
"""Throughput over the time of one mesh-kernel launch (debug build with -DHIPPT_DEBUG_RATE, run with
HIPPT_LIB=qt-raytracer_amd/libv_rate.so): samples and segments finished per 10 us bucket, wave
rounds and lane occupancy, for a list of (stride, spp) jobs, so that a 1/N row share can be compared
with the whole image bucket by bucket.

usage: python tools/rate_timeline.py [--scene cornell34] [--jobs 1:64,8:64,1:8,8:64:8] [--bucket-us 50]
       (a job is stride:spp[:batches]; batches > 1 are submitted back to back before one sync)
       [KEY=VALUE option pairs]
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

NB = 1024


def run(scene, stride, spp, opts, agg, batches=1):
    pt = hippt.PathTracer()
    pt.setDevices([0])
    for k, v in opts:
        pt.setOption(k, v)
    pt.setRowInterleave(0, stride)
    pt.uploadMesh(scenes.get_scene(scene))
    assert pt.initialize(1920, 1080)
    fn = pt._lib.hipptDebugRate
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(2):
        pt._lib.hipptRenderFramesAsync(0, spp, 8, None)
        pt.synchronize()
    buf = np.zeros((NB, 5), np.uint64)
    fn(None, 1)
    pt.resetStats()
    for b in range(batches):  # back-to-back async batches (chained with HIPPT_OPT_CHAIN)
        pt._lib.hipptRenderFramesAsync(b * spp, spp, 8, None)
    pt.synchronize()
    st = pt.stats()
    fn(buf.ctypes.data, 1)
    del pt
    nz = np.nonzero(buf[:, 4])[0]
    last = int(nz.max()) + 1 if len(nz) else 0
    b = buf[:last].astype(np.float64)
    k = max(1, agg // 10)
    n = (last + k - 1) // k
    b = np.pad(b, ((0, n * k - last), (0, 0))).reshape(n, k, 5).sum(axis=1)
    tot_samples = b[:, 0].sum()
    tot_segs = b[:, 1].sum()
    rows = []
    for i in range(n):
        rows.append({"t_us": i * agg, "samples_frac": round(b[i, 0] / max(1, tot_samples), 4),
                     "segs_per_us": round(b[i, 1] / agg / 1e3, 2),  # G segments/s
                     "lane_util": round(b[i, 3] / max(1, 64 * b[i, 2]), 3),
                     "waves": round(b[i, 4] / k, 0)})
    return {"scene": scene, "stride": stride, "spp": spp, "batches": batches, "trace_ms": round(st["traceMs"], 4),
            "segments": int(st["segments"]), "samples": int(st["pixelSamples"]),
            "gseg_per_s": round(st["segments"] / st["traceMs"] / 1e6, 2), "buckets": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--jobs", default="1:64,8:64,1:8")
    ap.add_argument("--bucket-us", type=int, default=50)
    ap.add_argument("opts", nargs="*")
    a = ap.parse_args()
    opts = [tuple(int(x) for x in o.split("=")) for o in a.opts]
    for j in a.jobs.split(","):
        f = [int(x) for x in j.split(":")]
        print(json.dumps(run(a.scene, f[0], f[1], opts, a.bucket_us, f[2] if len(f) > 2 else 1)), flush=True)


if __name__ == "__main__":
    main()
