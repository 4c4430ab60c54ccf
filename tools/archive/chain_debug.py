#!/usr/bin/env python3
"""Diagnose chained batches on the GPU: small sequences against the oracle, per row and per
hypothesis (which frames' contributions the GPU accumulation matches)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import hippt  # noqa: E402
import pyoracle as po  # noqa: E402
from hippt import scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cornell34"
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (45, 26)
sc = scenes.get_scene(name)
ms = po.MeshScene(sc, w, h)
ora = {n: ms.frames(0, n, 8) for n in (2, 4, 6)}
pt = hippt.PathTracer()
pt.uploadMesh(sc)
lib = hippt.load_library()
for item_order in (1, 0):
    pt.setOption(hippt.OPT_ITEM_ORDER, item_order)
    for chain in (0, 1, 2, 8):
        pt.setOption(hippt.OPT_CHAIN, chain)
        for nb in (1, 2, 3):
            assert pt.initialize(w, h)
            for _ in range(nb):
                assert pt.renderFramesAsync(2, 8), pt.lastError()
            px, acc = pt.readback()
            o = ora[2 * nb]
            bad = px != o[0]
            rows = np.nonzero(bad.any(axis=1))[0]
            line = f"item_order {item_order} chain {chain} batches {nb}: {int(bad.sum())} px differ"
            if bad.any():
                line += f", rows {rows[:6].tolist()}..{rows[-3:].tolist()}"
                y, x = np.argwhere(bad)[0]
                line += f"; first ({x},{y}) gpu acc {acc[y, x, :3].tolist()} ora {o[1][y, x, :3].tolist()}"
                for n2, o2 in ora.items():
                    if np.array_equal(acc[bad], o2[1][bad]):
                        line += f"; the differing pixels equal the oracle after {n2} frames"
            print(line, flush=True)
