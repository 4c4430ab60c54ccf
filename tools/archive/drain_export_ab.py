#!/usr/bin/env python3
"""A/B of the drain export (HIPPT_OPT_DRAIN_EXPORT, HIPPT_OPT_TAIL_BLOCKS_PER_CU): kernel time per step
of a 1/N row share and of the whole image for each setting, alternating settings within each pass,
and the image's accumulation SHA-256 (must not depend on the setting).

usage: python tools/drain_export_ab.py [--scene cornell34] [--strides 1,8] [--spp 64] [--steps 5]
       [--passes 2] [--settings 0:0,16:2,32:2,64:2]   (threshold:tail blocks per CU)
"""
import argparse
import hashlib
import json
import os
import sys
import zlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell34")
    ap.add_argument("--strides", default="1,8")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--settings", default="0:0,16:2,32:2,64:2")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    settings = [tuple(int(x) for x in s.split(":")) for s in a.settings.split(",")]
    scene = scenes.get_scene(a.scene)
    for stride in [int(x) for x in a.strides.split(",")]:
        pt = hippt.PathTracer()
        pt.setDevices([0])
        pt.setRowInterleave(0, stride)
        pt.uploadMesh(scene)
        assert pt.initialize(a.width, a.height)
        res = {s: [] for s in settings}
        digest = {}
        for p in range(a.passes):
            for s in settings:
                pt.setOption(hippt.OPT_DRAIN_EXPORT, s[0])
                pt.setOption(hippt.OPT_TAIL_BLOCKS_PER_CU, s[1])
                if p == 0:  # the image of one step, from a reset accumulation
                    pt.resetAccumulation()
                    pt._lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
                    pix, acc = pt.readback()
                    rows = slice(0, None, stride)
                    digest[s] = (zlib.crc32(pix[rows].tobytes()), hashlib.sha256(acc[rows].tobytes()).hexdigest()[:16])
                pt._lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
                pt.synchronize()
                pt.resetStats()
                for _ in range(a.steps):
                    pt._lib.hipptRenderFramesAsync(0, a.spp, a.depth, None)
                pt.synchronize()
                st = pt.stats()
                res[s].append(st["traceMs"] / a.steps)
        base = digest[settings[0]]
        for s in settings:
            print(json.dumps({"scene": a.scene, "stride": stride, "spp": a.spp, "export_thr": s[0], "tail_bpc": s[1],
                              "trace_ms": [round(x, 4) for x in res[s]], "crc": digest[s][0], "sha": digest[s][1],
                              "same_image": digest[s] == base}), flush=True)
        del pt


if __name__ == "__main__":
    main()
