"""Primary candidate lists (hipptPrimaryLists, qt-raytracer_amd/csrc/primary_lists.cpp) on the CPU.

The GPU path replaces a camera ray's BVH traversal by the triangles listed for its pixel; the
closest hit (argmin (t, primitive id) over every triangle the FP32 test reports hit, the oracle's
brute force) is unchanged as long as the list holds every triangle some camera ray through the
pixel can hit.  These tests check exactly that against the oracle's own ray generation and
triangle test (po_pixel_any_hits: a grid over the pixel's footprint, its edges included, plus
random points), on the headline scenes and on adversarial triangles (edge-on, near and behind the
camera plane, slivers, sub-pixel and screen-filling ones).  The GPU side is in test_gpu_parity.py.
"""
import ctypes

import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes


def _cams(scene, w, h):
    cam = hippt.build_camera(scene.lookfrom, scene.lookat, scene.vup, scene.vfov, w / h, scene.aperture, scene.focus)
    return cam, po.PoCamera.from_buffer_copy(bytes(cam))


def _check(verts, cam, pcam, w, h, n, extra=0, y0=0, rows=None, stride=1, seed=1):
    rows = h if rows is None else rows
    res = hippt.primary_lists(verts, cam, w, h, y0, rows, stride)
    assert res is not None
    off, ids = res
    assert off.shape == (rows * w + 1,) and off[0] == 0 and np.all(np.diff(off.astype(np.int64)) >= 0)
    assert off[-1] == ids.size
    tris = po.tri_array(verts)
    missing = []
    for k in range(rows):
        y = y0 + k * stride
        for x in range(w):
            lst = ids[off[k * w + x]:off[k * w + x + 1]]
            assert np.all(np.diff(lst.astype(np.int64)) > 0)  # ascending, no duplicates
            hit = po.pixel_any_hits(tris, pcam, w, h, x, y, n=n, extra=extra, seed=seed)
            lost = np.setdiff1d(hit, lst)
            if lost.size:
                missing.append((x, y, lost[:4].tolist()))
    assert not missing, f"hit triangles missing from their pixel's list: {missing[:8]}"
    return off, ids


def test_cornell34_lists_hold_every_hit():
    sc = scenes.get_scene("cornell34")
    w, h = 64, 36
    cam, pcam = _cams(sc, w, h)
    off, ids = _check(sc.verts, cam, pcam, w, h, n=4, extra=4)
    mean = ids.size / (w * h)
    assert 0.5 < mean < 3.0, mean  # tight: about one wall per pixel, not the whole scene


def test_blob70k_lists_hold_every_hit():
    sc = scenes.get_scene("blob70k")
    w, h = 32, 18
    cam, pcam = _cams(sc, w, h)
    off, ids = _check(sc.verts, cam, pcam, w, h, n=2)
    assert ids.size / (w * h) < 2000  # 32x18: a pixel covers hundreds of blob triangles (front and back)


def test_band_rows_equal_full_image_rows():
    sc = scenes.get_scene("cornell34")
    w, h = 40, 30
    cam, _ = _cams(sc, w, h)
    off, ids = hippt.primary_lists(sc.verts, cam, w, h)
    for y0, stride in ((0, 1), (1, 3), (5, 2), (29, 1)):
        rows = len(range(y0, h, stride))
        boff, bids = hippt.primary_lists(sc.verts, cam, w, h, y0, rows, stride)
        for k in range(rows):
            y = y0 + k * stride
            for x in range(w):
                full = ids[off[y * w + x]:off[y * w + x + 1]]
                band = bids[boff[k * w + x]:boff[k * w + x + 1]]
                assert np.array_equal(full, band), (y0, stride, x, y)


def test_lens_camera_has_no_lists():
    sc = scenes.get_scene("cornell34")
    cam = hippt.build_camera(sc.lookfrom, sc.lookat, sc.vup, sc.vfov, 16 / 9, 0.5, 10.0)
    assert hippt.primary_lists(sc.verts, cam, 16, 9) is None


def _adversarial(rng, n):
    """Triangles around a camera at the origin looking down -z (vfov 60, 4:3)."""
    out = []
    for i in range(n):
        kind = i % 8
        c = np.array([rng.uniform(-3, 3), rng.uniform(-2, 2), -rng.uniform(1, 20)])
        if kind == 0:  # ordinary
            v = c + rng.normal(scale=1.0, size=(3, 3))
        elif kind == 1:  # plane through the camera origin (edge-on)
            a, b = c + rng.normal(scale=1.0, size=3), c + rng.normal(scale=1.0, size=3)
            v = np.stack([a, b, rng.uniform(0.2, 1.5) * a + rng.uniform(0.2, 1.5) * b])
        elif kind == 2:  # plane a hair off the origin
            a, b = c + rng.normal(scale=1.0, size=3), c + rng.normal(scale=1.0, size=3)
            nrm = np.cross(a, b)
            v = np.stack([a, b, 0.7 * a + 0.6 * b]) + 1e-4 * nrm / np.linalg.norm(nrm)
        elif kind == 3:  # one vertex behind the camera plane
            v = np.stack([c + rng.normal(scale=1.0, size=3), c + rng.normal(scale=1.0, size=3),
                          np.array([rng.uniform(-2, 2), rng.uniform(-2, 2), rng.uniform(0.1, 3)])])
        elif kind == 4:  # sliver
            a, b = c + rng.normal(scale=2.0, size=3), c + rng.normal(scale=2.0, size=3)
            v = np.stack([a, b, 0.5 * (a + b) + rng.normal(scale=1e-3, size=3)])
        elif kind == 5:  # sub-pixel, far
            v = c * 5 + rng.normal(scale=1e-3, size=(3, 3))
        elif kind == 6:  # screen-filling, near
            v = np.array([[-50.0, -50.0, -0.5], [50.0, -50.0, -0.7], [0.0, 80.0, -0.6]]) + rng.normal(scale=0.1,
                                                                                                          size=(3, 3))
        else:  # grazing floor: a large triangle in a plane just below the camera
            y = -rng.uniform(1e-3, 0.5)
            v = np.array([[-30.0, y, -0.2], [30.0, y, -0.2], [0.0, y + rng.uniform(-1e-3, 1e-3), -60.0]])
        out.append(v.reshape(9))
    return np.array(out, np.float32)


@pytest.mark.parametrize("seed", [3, 11])
def test_adversarial_triangles(seed):
    rng = np.random.default_rng(seed)
    verts = _adversarial(rng, 96)
    w, h = 32, 24
    cam = hippt.build_camera((0.0, 0.0, 0.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 60.0, w / h, 0.0, 1.0)
    # origin (0,0,0): pinhole rays still start exactly at the origin (origin + 0 * offset)
    pcam = po.PoCamera.from_buffer_copy(bytes(cam))
    _check(verts, cam, pcam, w, h, n=6, extra=8, seed=seed)
    # and from a camera away from the origin (nonzero origin coordinates)
    cam2 = hippt.build_camera((0.3, 0.2, 0.5), (0.3, 0.1, -1.0), (0.0, 1.0, 0.0), 60.0, w / h, 0.0, 1.0)
    _check(verts, cam2, po.PoCamera.from_buffer_copy(bytes(cam2)), w, h, n=6, extra=8, seed=seed + 1)
