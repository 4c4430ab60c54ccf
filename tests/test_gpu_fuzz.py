"""Seeded random scenes (GPU): triangle soups with degenerate, tiny, huge, axis-aligned and
edge-sharing triangles, overlapping spheres, all three materials, pinhole and thin-lens cameras,
rendered through the C ABI in the LDS-resident, global-memory (float, 8-bit, hybrid and half-plane nodes),
2-wide and wavefront paths, and
compared bit for bit (ARGB words, accumulation floats, segment counts) with the oracle.

The named benchmark scenes exercise the hot path at scale; these exercise the geometry the
contract has to get right on its edges (grazing and coplanar hits, equal-t ties between
primitives, rays starting inside spheres, zero direction components)."""
import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes

pytestmark = pytest.mark.gpu

W, H, SPP, DEPTH = 48, 32, 3, 6


def fuzz_scene(seed: int) -> scenes.Scene:
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 420))
    centre = rng.uniform(-40.0, 40.0, size=(n, 1, 3))
    size = 10.0 ** rng.uniform(-2.0, 1.4, size=(n, 1, 1))
    verts = centre + size * rng.normal(size=(n, 3, 3))
    kind = rng.integers(0, 6, size=n)
    verts[kind == 0, 1] = verts[kind == 0, 0]                          # repeated vertex: degenerate
    verts[kind == 1, 2] = 2.0 * verts[kind == 1, 1] - verts[kind == 1, 0]  # collinear: degenerate
    ax = rng.integers(0, 3)
    verts[kind == 2, :, ax] = np.round(verts[kind == 2, :1, ax])       # axis-aligned, integer plane
    verts = verts.reshape(n, 9)
    share = np.flatnonzero(kind == 3)[1:]                               # shares an edge with its predecessor
    verts[share, 0:6] = verts[share - 1, 3:9]
    nm = int(rng.integers(1, 7))
    mat_kind = rng.integers(0, 3, size=nm).astype(np.int32)
    if seed % 4 == 0:
        mat_kind[:] = scenes.MAT_LAMBERTIAN
    albedo = rng.uniform(0.05, 0.95, size=(nm, 3)).astype(np.float32)
    fuzz = rng.uniform(0.0, 1.0, size=nm).astype(np.float32)
    ir = rng.uniform(1.0, 2.4, size=nm).astype(np.float32)
    ns = 0 if seed % 4 == 0 else int(rng.integers(0, 14))
    spheres = np.concatenate([rng.uniform(-35.0, 35.0, size=(ns, 3)), 10.0 ** rng.uniform(-1.0, 1.4, size=(ns, 1))],
                             axis=1)
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    lookfrom = tuple(float(x) for x in d * rng.uniform(60.0, 160.0))
    if seed % 5 == 1 and ns:                                            # camera inside a sphere
        spheres[0, :3] = lookfrom
        spheres[0, 3] = 3.0
    if seed % 7 == 2:                                                   # axis-parallel view: zero direction components
        lookfrom = (0.0, 0.0, 120.0)
    return scenes.Scene(
        name=f"fuzz{seed}", verts=np.ascontiguousarray(verts, np.float32),
        tri_mat=rng.integers(0, nm, size=n).astype(np.int32), albedo=albedo,
        lookfrom=lookfrom, lookat=tuple(float(x) for x in rng.uniform(-5.0, 5.0, size=3)), vup=(0.0, 1.0, 0.0),
        vfov=float(rng.uniform(20.0, 90.0)), aperture=float(rng.choice([0.0, rng.uniform(0.05, 2.0)])),
        focus=float(rng.uniform(20.0, 150.0)), spheres=np.ascontiguousarray(spheres, np.float32),
        sph_mat=rng.integers(0, nm, size=ns).astype(np.int32), mat_kind=mat_kind, fuzz=fuzz, ir=ir)


@pytest.fixture()
def pt():
    t = hippt.PathTracer()
    t.setDevices([])
    t.setRowRange(0, 0)
    t.useBuiltinScene(hippt.SCENE_SPHERE4)
    yield t
    for k, v in ((hippt.OPT_LDS_SCENE, 1), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_PATH_MODE, 0),
                 (hippt.OPT_WAVEFRONT_SLOTS, 1 << 24), (hippt.OPT_BVH_QUANT, -1)):
        t.setOption(k, v)
    hippt.load_library().cudaPathTracerShutdown()


MODES = {
    "default": ((hippt.OPT_LDS_SCENE, 1), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_PATH_MODE, 0)),
    "global": ((hippt.OPT_LDS_SCENE, 0), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_PATH_MODE, 0)),
    "wide2": ((hippt.OPT_LDS_SCENE, 0), (hippt.OPT_BVH_WIDTH, 2), (hippt.OPT_PATH_MODE, 0)),
    "quant8": ((hippt.OPT_LDS_SCENE, 0), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_BVH_QUANT, 1)),
    "hybrid": ((hippt.OPT_LDS_SCENE, 0), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_BVH_QUANT, 2)),
    "half": ((hippt.OPT_LDS_SCENE, 0), (hippt.OPT_BVH_WIDTH, 0), (hippt.OPT_BVH_QUANT, 3)),
    "wavefront": ((hippt.OPT_LDS_SCENE, 1), (hippt.OPT_BVH_QUANT, -1), (hippt.OPT_PATH_MODE, 1),
                  (hippt.OPT_WAVEFRONT_SLOTS, 500)),
}


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_scene_matches_oracle(pt, seed):
    sc = fuzz_scene(seed)
    ora_px, ora_acc, segs, samples = po.MeshScene(sc, W, H).frames(0, SPP, DEPTH)
    for mode, opts in MODES.items():
        for k, v in opts:
            pt.setOption(k, v)
        pt.uploadScene(sc) if not sc.lambertian_triangles else pt.uploadMesh(sc)
        assert pt.initialize(W, H), pt.lastError()
        pt.resetStats()
        assert pt.renderFrames(SPP, DEPTH), pt.lastError()
        px, acc = pt.readback()
        diff = np.count_nonzero(px != ora_px)
        assert diff == 0, f"{mode}: {diff} of {px.size} pixels differ"
        assert acc.tobytes() == ora_acc.tobytes(), mode
        st = pt.stats()
        assert st["segments"] == segs and st["pixelSamples"] == samples, mode
