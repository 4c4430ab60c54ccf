"""The reference's own gtest known answers (tests/unit/*.cpp), restated against the FP32 oracle.

Each test cites the gtest it restates.  Tolerances: the reference checks FP64 at 1e-9; the
oracle is FP32, so values are compared at 1e-6 (exact where the FP32 result is exact).
"""
import math

import numpy as np
import pytest

import pyoracle as po

EPS = 1e-6


def test_sphere_hit_expected_t():  # SphereTests.cpp:9-27 RayHitsSphereAtExpectedT
    hit, t, n, front = po.sphere_hit((0, 0, -1), 0.5, (0, 0, 0), (0, 0, -1))
    assert hit and front
    assert t == pytest.approx(0.5, abs=EPS)
    assert n == pytest.approx((0.0, 0.0, 1.0), abs=EPS)


def test_sphere_miss():  # SphereTests.cpp:29-36 RayMissesSphere
    assert not po.sphere_hit((0, 0, -1), 0.5, (0, 0, 0), (0, 1, 0))[0]


def test_closest_hit_regardless_of_order():  # HitableListTests.cpp:9-25 ReturnsClosestHit (triangles)
    def quad_at(z):
        return [[-1, -1, z, 1, -1, z, 1, 1, z], [-1, -1, z, 1, 1, z, -1, 1, z]]

    class S:  # far quad listed first, like the gtest's far sphere
        verts = np.asarray(quad_at(-2.0) + quad_at(-0.5), np.float32)
        num_tris = 4

    idx, t = po.closest_hit(S, (0.2, 0.1, 0), (0, 0, -1))
    assert idx in (2, 3) and t == pytest.approx(0.5, abs=EPS)


def test_degrees_to_radians():  # MathUtilsTests.cpp:9-13; FP64 restated in the camera build
    cam = po.camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90.0, 1.0, 0.0, 1.0)
    # tan(45deg) = 1 -> vertical extent 2 -> vertical = (0, 2, 0)
    assert np.allclose(np.frombuffer(bytes(cam.vertical), np.float32), [0, 2, 0], atol=EPS)


def test_clamp_in_tonemap():  # MathUtilsTests.cpp:15-19 ClampLimitsToRange, via the ARGB pack
    acc = (np.zeros(4, np.float32))
    import ctypes
    a = np.array([-2.0, 0.25, 9.0, 0.0], np.float32)
    s = np.zeros(3, np.float32)
    w = po.lib().po_accumulate(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                               s.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 1)
    # frame 1: acc = (acc*1 + 0)/2 -> (-1, 0.125, 4.5) -> clamp -> (0, .125, 1) -> sqrt*255 trunc
    assert (w >> 16) & 255 == 0
    assert (w >> 8) & 255 == int(math.sqrt(np.float32(0.125)) * 255)
    assert w & 255 == 255 and w >> 24 == 255
    del acc


def test_random_in_unit_sphere_inside():  # MathUtilsTests.cpp:21-26
    import ctypes
    st = ctypes.c_uint32(12345)
    p = np.zeros(3, np.float32)
    for _ in range(256):
        po.lib().po_random_in_unit_sphere(ctypes.byref(st), p.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        assert float(p @ p) < 1.0


def test_random_in_unit_disk_plane():  # MathUtilsTests.cpp:28-34
    import ctypes
    st = ctypes.c_uint32(999)
    p = np.zeros(3, np.float32)
    for _ in range(256):
        po.lib().po_random_in_unit_disk(ctypes.byref(st), p.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        assert float(p @ p) < 1.0 and p[2] == 0.0


def test_aabb_hit_and_miss():  # AabbTests.cpp:11-23
    assert po.aabb_hit((-1, -1, -3), (1, 1, -1), (0, 0, 0), (0, 0, -1))
    assert not po.aabb_hit((-1, -1, -3), (1, 1, -1), (0, 2, 0), (0, 0, -1))


def test_camera_center_ray_zero_aperture():  # CameraTests.cpp:9-25
    import ctypes
    cam = po.camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90.0, 2.0, 0.0, 1.0)
    st = ctypes.c_uint32(7)
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    pf = ctypes.POINTER(ctypes.c_float)
    po.lib().po_camera_get_ray(ctypes.byref(cam), 0.5, 0.5, ctypes.byref(st), o.ctypes.data_as(pf), d.ctypes.data_as(pf))
    assert np.allclose(o, 0, atol=EPS) and np.allclose(d, [0, 0, -1], atol=EPS)


def test_lens_offset_within_aperture():  # CameraTests.cpp:27-39
    import ctypes
    aperture = 2.0
    cam = po.camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90.0, 2.0, aperture, 1.0)
    st = ctypes.c_uint32(3)
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    pf = ctypes.POINTER(ctypes.c_float)
    for _ in range(128):
        po.lib().po_camera_get_ray(ctypes.byref(cam), 0.5, 0.5, ctypes.byref(st), o.ctypes.data_as(pf), d.ctypes.data_as(pf))
        assert np.linalg.norm(o) <= aperture * 0.5 + EPS
        assert abs(o[2]) <= EPS


def test_triangle_hit_at_expected_t():  # SphereTests analogue for the new triangle primitive
    tri = po.tri_setup([-1, -1, -0.5, 1, -1, -0.5, 0, 1, -0.5])
    hit, t = po.tri_hit(tri, (0, 0, 0), (0, 0, -1))
    assert hit and t == 0.5
    assert not po.tri_hit(tri, (0, 0, 0), (0, 1, 0))[0]
    assert np.allclose(np.frombuffer(bytes(tri.n), np.float32), [0, 0, 1])


def test_degenerate_triangle_never_hit():
    tri = po.tri_setup([0, 0, -1, 1, 0, -1, 2, 0, -1])  # collinear
    assert not po.tri_hit(tri, (0.5, 0, 0), (0, 0, -1))[0]


def test_tmin_rejects_self_hit():  # ray_color uses t_min = 0.001 (RayTracer.h:585)
    tri = po.tri_setup([-1, -1, -0.0005, 1, -1, -0.0005, 0, 1, -0.0005])
    assert not po.tri_hit(tri, (0, 0, 0), (0, 0, -1))[0]


def test_rgba8_quantization_known_answers():
    """pyoracle.rgba8 (pt_oracle.c po_rgba8): the GL / Vulkan RGBA8 UNORM word of an accumulated
    colour — sqrt(clamp(c, 0, 1)) * 255 rounded to nearest, ties to even, bytes R, G, B, A —
    against a numpy float32 restatement, on hand-picked and random colours."""
    hand = np.array([[0.25, 0.5, 1.0, 1.0], [0.0, -1.0, 2.0, 1.0], [np.nan, 1e-30, 0.999, 1.0]], np.float32)
    rng = np.random.default_rng(7)
    acc = np.concatenate([rng.random((4096, 4), dtype=np.float32) * np.float32(1.2) - np.float32(0.1), hand[:2]])
    c = np.sqrt(np.clip(acc[:, :3], np.float32(0), np.float32(1))) * np.float32(255)
    q = np.rint(c).astype(np.uint32)
    want = np.uint32(255 << 24) | (q[:, 2] << 16) | (q[:, 1] << 8) | q[:, 0]
    assert np.array_equal(po.rgba8(acc), want)
    assert int(po.rgba8(hand[:1])[0]) == 0xFFFFB480  # 0.5*255 = 127.5 -> 128 (even), 180.3 -> 180
    assert int(po.rgba8(hand[1:2])[0]) == 0xFFFF0000  # clamped: R 0, G 0, B 255
    assert int(po.rgba8(hand[2:3])[0]) & 0xFF == 0  # NaN clamps to 0 (fminf/fmaxf)
