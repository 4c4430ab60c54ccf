#!/usr/bin/env python3
"""GPU vs oracle per-sample diff (debug aid): renders single frames and lists differing pixels."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "qt-raytracer_amd"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import hippt  # noqa: E402
import pyoracle as po  # noqa: E402
from hippt import scenes  # noqa: E402


def main():
    name, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    sc = scenes.get_scene(name)
    if "APERTURE" in os.environ:
        sc.aperture = float(os.environ["APERTURE"])
    pt = hippt.PathTracer()
    pt.uploadScene(sc)
    ora = po.MeshScene(sc, w, h)
    out = {}
    for mode in (0, 1):
        pt.setOption(hippt.OPT_PATH_MODE, mode)
        assert pt.initialize(w, h)
        diffs = []
        for f in range(frames):
            pt.resetStats()
            assert pt.renderFrames(1, 8)
            _, acc = pt.readback()
            # the accumulator after frame f; compare with the oracle's running average
            _, oacc, segs, _ = ora.frames(0, f + 1, 8)
            bad = np.argwhere(np.any(acc[..., :3] != oacc[..., :3], axis=-1))
            for yx in bad[:20]:
                y, x = map(int, yx)
                diffs.append({"frame": f, "x": x, "y": y, "gpu": acc[y, x, :3].tolist(), "ora": oacc[y, x, :3].tolist()})
            if len(bad):
                break
        out[mode] = diffs
        print(name, "aperture", sc.aperture, "mode", mode, "ndiff", len(diffs), json.dumps(diffs[:3]), flush=True)


if __name__ == "__main__":
    main()
