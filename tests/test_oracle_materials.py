"""Spheres and the Metal/Dielectric materials in the oracle (the mesh path's general scenes),
pinned against the REFERENCE RayTracer.h (fixtures from tests/golden/make_golden.py):

* po_sphere_t (the contract's precision-robust FP32 roots) against the reference's FP64
  Sphere::hit golden vectors;
* po_reflect / po_refract against the reference's FP64 reflect / refract (:174-183);
* ref_random_scene.scene: a random_scene() (RayTracer.h:599-643) the reference itself built,
  and converged radiance of the reference ray_color on it and on cornell_mixed (triangles,
  spheres, all three materials), matched statistically.

Statistics: per-pixel z with the larger of the reference's and the oracle's own variance
(rare trapped-in-glass paths make the reference's 2048-sample variance unreliable on a few
silhouette pixels), |z| > 4 on at most 0.5% of values, mean |z| of Monte-Carlo noise, image
means within 0.5%.
"""
import json
import os

import numpy as np
import pytest

import pyoracle as po
from hippt import scenes


@pytest.fixture(scope="module")
def ref(golden_dir):
    with open(os.path.join(golden_dir, "ref_functions.json")) as f:
        return json.load(f)


def test_sphere_roots_match_reference_sphere_hit(ref):
    bad = 0
    for e in ref["sphere_hit"]:
        t = po.sphere_t(e["c"], e["r"], e["o"], e["d"])
        if (t is not None) != bool(e["hit"]):
            bad += 1
            continue
        if t is not None:
            assert t == pytest.approx(e["t"], rel=1e-5, abs=1e-6)
    assert bad <= 1, f"{bad} hit/miss disagreements"


def test_sphere_roots_far_origin_are_accurate():
    # a large, distant sphere: the literal hb^2 - a*c form loses ~1e-3 in t here in FP32
    c, r = (420.0, 60.0, 150.0), 60.0
    rng = np.random.default_rng(7)
    for _ in range(200):
        o = np.array([278.0, 278.0, -800.0]) + rng.uniform(-1, 1, 3)
        u = rng.normal(size=3)
        tgt = np.array(c) + u / np.linalg.norm(u) * rng.uniform(0.0, 0.95) * r  # inside the ball
        d = (tgt - o).astype(np.float32)
        o = o.astype(np.float32)
        t = po.sphere_t(c, r, o, d)
        od, dd, cd = o.astype(np.float64), d.astype(np.float64), np.asarray(c, np.float64)
        oc = od - cd
        a, hb, cc = dd @ dd, oc @ dd, oc @ oc - r * r
        t64 = (-hb - np.sqrt(hb * hb - a * cc)) / a
        assert t is not None and abs(t - t64) <= 2e-6 * t64


def test_reflect_refract_match_reference(ref):
    for e in ref["reflect"]:
        v, n = np.asarray(e["v"]), np.asarray(e["n"])
        assert np.allclose(po.reflect(v, n), e["reflect"], atol=2e-6 * (1 + np.abs(v).max()))
        uv = v / np.linalg.norm(v)
        assert np.allclose(po.refract(uv, n, e["eta"]), e["refract"], atol=2e-5)


def test_reference_random_scene_fixture(golden_dir):
    sc = scenes.load_scene_file(os.path.join(golden_dir, "ref_random_scene.scene"))
    kinds = sc.materials()["kind"][sc.sph_mat]
    assert sc.num_tris == 0 and 400 < sc.num_spheres <= 488  # 1 + <= 22*22 + 3
    assert tuple(sc.spheres[0]) == (0.0, -1000.0, 0.0, 1000.0)  # ground, RayTracer.h:603
    assert set(kinds.tolist()) == {scenes.MAT_LAMBERTIAN, scenes.MAT_METAL, scenes.MAT_DIELECTRIC}
    assert sc.lookfrom == (13.0, 2.0, 3.0) and sc.aperture == pytest.approx(0.1) and sc.vfov == 20.0


@pytest.mark.parametrize("name", ["random_scene", "cornell_mixed"])
def test_oracle_bvh_equals_brute_force(name):
    sc = scenes.get_scene(name)
    a = po.MeshScene(sc, 40, 24, accel=0).frames(0, 3, 8)
    b = po.MeshScene(sc, 40, 24, accel=1).frames(0, 3, 8)
    assert np.array_equal(a[0], b[0]) and a[1].tobytes() == b[1].tobytes() and a[2:] == b[2:]


def _batch_means(ms, n, batches):
    """Per-pixel means of `batches` independent frame ranges (running average rescaled)."""
    out = []
    m = n // batches
    for b in range(batches):
        _, acc, _, _ = ms.frames(b * m, m, 8)
        out.append(acc[..., :3].astype(np.float64) * ((b + 1) * m) / m)
    return np.stack(out)


@pytest.mark.parametrize("name,w,h,spp,n", [("ref_random_scene", 48, 27, 2048, 512),
                                            ("cornell_mixed", 48, 48, 2048, 512)])
def test_converged_radiance_matches_reference(golden_dir, name, w, h, spp, n):
    ref_img = np.load(os.path.join(golden_dir, f"ref_converge_{name}_{w}x{h}_{spp}.npy"))
    sc = (scenes.load_scene_file(os.path.join(golden_dir, "ref_random_scene.scene"), name)
          if name == "ref_random_scene" else scenes.get_scene(name))
    bm = _batch_means(po.MeshScene(sc, w, h, accel=1), n, 8)
    m = bm.mean(axis=0)
    own_var = bm.var(axis=0, ddof=1) * (n // 8)  # per-sample variance estimate
    rm, rv = ref_img[..., :3].astype(np.float64), ref_img[..., 3:].astype(np.float64)
    var = np.maximum(rv, own_var)
    z = (m - rm) / (np.sqrt(var / n + var / spp) + 1e-7)
    assert (np.abs(z) > 4.0).mean() < 5e-3
    assert np.abs(z).max() < 8.0
    assert 0.55 < np.abs(z).mean() < 1.0
    rel = m.mean(axis=(0, 1)) / rm.mean(axis=(0, 1)) - 1.0
    assert np.all(np.abs(rel) < 5e-3), rel
