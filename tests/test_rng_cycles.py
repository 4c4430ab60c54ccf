"""The reference hash RNG (CudaPathTracerKernel.cu:23-35) has short cycles; rejection loops on
them would spin forever in the reference.  The contract escapes them (pt_oracle.c PO_ESCAPE);
these tests pin the cycle facts and the exact seeds that hit them."""
import ctypes

import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes

# pixel (x, y), frame of a 3840x2160 image whose seed lies on the 2-cycle {160893342, 357741884}
BAD_W, BAD_H, BAD_X, BAD_Y, BAD_F = 3840, 2160, 1750, 1610, 17


def h(x):
    return po.lib().po_hash32(x)


def test_hash32_short_cycles():
    assert h(0) == 0 and h(3496737362) == 3496737362  # fixed points rejected by every loop
    assert h(160893342) == 357741884 and h(357741884) == 160893342
    s = 2247562032
    seen = [s]
    for _ in range(4):
        seen.append(h(seen[-1]))
    assert h(seen[-1]) == s and len(set(seen)) == 5


def test_known_bad_seed():
    assert po.lib().po_pixel_seed(BAD_X, BAD_Y, BAD_W, BAD_F) == 357741884


def test_rejection_loops_terminate_on_cycles():
    p = np.zeros(3, np.float32)
    pf = p.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    for s0 in (0, 3496737362, 160893342, 2247562032):
        st = ctypes.c_uint32(s0)
        po.lib().po_random_in_unit_sphere(ctypes.byref(st), pf)
        assert float(p @ p) < 1.0
        st = ctypes.c_uint32(s0)
        po.lib().po_random_in_unit_disk(ctypes.byref(st), pf)
        assert float(p @ p) < 1.0 and p[2] == 0


def test_escape_does_not_touch_ordinary_sequences():
    # the first 64 attempts are the reference's loop: a state far from any short cycle gives
    # the same sample as a plain restatement of RayTracer.h:155-161 with the hash RNG
    st = ctypes.c_uint32(12345)
    p = np.zeros(3, np.float32)
    po.lib().po_random_in_unit_sphere(ctypes.byref(st), p.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    s = 12345
    while True:
        v = []
        for _ in range(3):
            s = h(s)
            v.append(np.float32(np.float32(s) / np.float32(4294967295.0)) * np.float32(2) - np.float32(1))
        v = np.array(v, np.float32)
        if float(np.float32(v[0] * v[0] + np.float32(v[1] * v[1] + v[2] * v[2]))) < 1.0:
            break
    assert np.array_equal(p, v) and st.value == s


def test_oracle_bad_pixel_terminates():
    ms = po.MeshScene(scenes.cornell34(), BAD_W, BAD_H)
    rgb, segs = ms.sample(BAD_X, BAD_Y, BAD_F, 8)
    assert 1 <= segs <= 8 and np.all(np.isfinite(rgb))
    out, acc = po.sphere4(BAD_W, BAD_H, BAD_F, 1, 8, y0=BAD_Y, y1=BAD_Y + 1)
    assert np.all(np.isfinite(acc))


@pytest.mark.gpu
@pytest.mark.parametrize("mesh", [True, False])
def test_gpu_bad_pixel_row_matches_oracle(mesh):
    pt = hippt.PathTracer()
    lib = hippt.load_library()
    try:
        pt.setDevices([])
        pt.setRowRange(BAD_Y, BAD_Y + 2)
        if mesh:
            pt.uploadMesh(scenes.cornell34())
        else:
            pt.useBuiltinScene(hippt.SCENE_SPHERE4)
        assert pt.initialize(BAD_W, BAD_H), pt.lastError()
        assert lib.hipptRenderFrames(BAD_F, 1, 8, None, None), lib.hipptLastError()
        px, acc = pt.readback(BAD_Y, BAD_Y + 2)
        if mesh:
            opx, oacc, _, _ = po.MeshScene(scenes.cornell34(), BAD_W, BAD_H).frames(
                BAD_F, 1, 8, y0=BAD_Y, y1=BAD_Y + 2, accum=np.zeros((2, BAD_W, 4), np.float32))
        else:
            opx, oacc = po.sphere4(BAD_W, BAD_H, BAD_F, 1, 8, y0=BAD_Y, y1=BAD_Y + 2)
        assert np.array_equal(px, opx) and acc.tobytes() == oacc.tobytes()
    finally:
        pt.setRowRange(0, 0)
        pt.useBuiltinScene(hippt.SCENE_SPHERE4)
        lib.cudaPathTracerShutdown()
