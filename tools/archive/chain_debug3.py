#!/usr/bin/env python3
"""test_chained_batches_match_oracle's sequence (progressive batches, 37 same-frame batches, mixed
sizes, a reset), repeated, reporting every scenario that differs from the oracle (NaN words too)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import hippt  # noqa: E402
import pyoracle as po  # noqa: E402
from hippt import scenes  # noqa: E402

sc = scenes.cornell34()
w, h = 45, 26
ora6 = po.MeshScene(sc, w, h).frames(0, 6, 8)
ora2 = po.MeshScene(sc, w, h).frames(0, 2, 8)
pt = hippt.PathTracer()
pt.setOption(hippt.OPT_ITEM_ORDER, int(sys.argv[1]) if len(sys.argv) > 1 else -1)
pt.uploadMesh(sc)
lib = hippt.load_library()


def check(tag, o):
    px, acc = pt.readback()
    bad = int((px != o[0]).sum())
    nan = int(np.isnan(acc).sum())
    print(f"{tag}: {bad} px differ, {nan} NaN words", flush=True)
    print(f"=== {tag} done", file=sys.stderr, flush=True)


for rep in range(3):
    for chain in (1, 2, 8, 0, -1):
        pt.setOption(hippt.OPT_CHAIN, chain)
        assert pt.initialize(w, h)
        pt.resetStats()
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8), pt.lastError()
        check(f"rep {rep} chain {chain} progressive", ora6)
        assert pt.initialize(w, h)
        for _ in range(37):
            assert lib.hipptRenderFramesAsync(0, 2, 8, None)
        check(f"rep {rep} chain {chain} same37", ora2)
        assert pt.initialize(w, h)
        assert pt.renderFramesAsync(1, 8) and pt.renderFramesAsync(2, 8) and pt.renderFramesAsync(2, 8)
        assert pt.renderFramesAsync(1, 8)
        check(f"rep {rep} chain {chain} mixed", ora6)
        assert pt.initialize(w, h)
        assert pt.renderFramesAsync(2, 8) and pt.renderFramesAsync(2, 8) and pt.resetAccumulation()
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8)
        check(f"rep {rep} chain {chain} reset", ora6)
