#!/usr/bin/env python3
"""Chained batches, many back-to-back batches of the same frames (step 0) and progressive ones,
against the oracle: per cap and batch count, the differing pixels and NaN words."""
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
ora2 = po.MeshScene(sc, w, h).frames(0, 2, 8)
pt = hippt.PathTracer()
pt.uploadMesh(sc)
lib = hippt.load_library()
pt.setOption(hippt.OPT_ITEM_ORDER, 1)
for chain in (2, 3, 8):
    pt.setOption(hippt.OPT_CHAIN, chain)
    for nb in (2, 3, 5, 9, 17, 37):
        assert pt.initialize(w, h)
        print(f"--- chain {chain} batches {nb}", file=sys.stderr, flush=True)
        for _ in range(nb):
            assert lib.hipptRenderFramesAsync(0, 2, 8, None)
        px, acc = pt.readback()
        bad = px != ora2[0]
        print(f"chain {chain} same-frame batches {nb}: {int(bad.sum())} px differ, {int(np.isnan(acc).sum())} NaN words",
              flush=True)
