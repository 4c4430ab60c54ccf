"""Statistical agreement of the FP32/hash-RNG restatement with the REFERENCE ray_color
(RayTracer.h:579-596, FP64, its own RNG), on converged images from
tests/golden/ref_converge_*.npy.

The reference CPU tracer is nondeterministic (thread-id-seeded RNG, RayTracer.h:32-38), so
per-pixel parity with it can only be statistical: per-pixel |z| <= 5 with z computed from the
reference's per-pixel variance, and image means within 0.5%.
"""
import os

import numpy as np
import pytest

import pyoracle as po
from hippt import scenes


@pytest.mark.parametrize("name,w,h,spp,n", [("cornell34", 64, 64, 4096, 256), ("blob70k", 32, 32, 1024, 256)])
def test_converged_radiance_matches_reference(golden_dir, name, w, h, spp, n):
    ref = np.load(os.path.join(golden_dir, f"ref_converge_{name}_{w}x{h}_{spp}.npy"))
    ms = po.MeshScene(scenes.get_scene(name), w, h, accel=1)
    _, acc, segs, samples = ms.frames(0, n, 8)
    m, rm, rv = acc[..., :3], ref[..., :3], ref[..., 3:]
    z = (m - rm) / (np.sqrt(rv / n + rv / spp) + 1e-6)
    assert np.abs(z).max() < 6.0
    assert (np.abs(z) > 4.0).mean() < 1e-3
    assert 0.6 < np.abs(z).mean() < 1.0  # ~0.80 for pure Monte-Carlo noise
    rel = m.mean(axis=(0, 1)) / rm.mean(axis=(0, 1)) - 1.0
    assert np.all(np.abs(rel) < 5e-3), rel
    assert samples == w * h * n and samples <= segs <= 8 * samples
