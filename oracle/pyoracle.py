"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  Never imported by the product package (qt-raytracer_amd/hippt).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")
REF_HARNESS_STRICT = os.path.join(HERE, "_ref", "ref_harness_strict")


class PoCamera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("llc", ctypes.c_float * 3), ("horizontal", ctypes.c_float * 3),
                ("vertical", ctypes.c_float * 3), ("u", ctypes.c_float * 3), ("v", ctypes.c_float * 3),
                ("lens_radius", ctypes.c_float), ("pad_", ctypes.c_float)]

    def as_array(self) -> np.ndarray:
        return np.frombuffer(bytes(self), dtype=np.float32).copy()


class PoTri(ctypes.Structure):
    _fields_ = [("v0", ctypes.c_float * 3), ("e1", ctypes.c_float * 3), ("e2", ctypes.c_float * 3),
                ("n", ctypes.c_float * 3)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    f, i, u32, d = ctypes.c_float, ctypes.c_int, ctypes.c_uint32, ctypes.c_double
    pf, pi, pu32, pd = (ctypes.POINTER(x) for x in (f, i, u32, d))
    pu64 = ctypes.POINTER(ctypes.c_uint64)

    def sig(name, res, *args):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = list(args)

    sig("po_hash32", u32, u32)
    sig("po_rand01", f, pu32)
    sig("po_pixel_seed", u32, i, i, i, i)
    sig("po_camera_build", None, pd, pd, pd, d, d, d, d, ctypes.POINTER(PoCamera))
    sig("po_tri_setup", None, pf, ctypes.POINTER(PoTri))
    sig("po_tri_hit", i, ctypes.POINTER(PoTri), pf, pf, f, pf)
    sig("po_sphere_hit", i, pf, f, pf, pf, f, f, pf, pf, pi)
    sig("po_aabb_hit", i, pf, pf, pf, pf, f, f)
    sig("po_random_in_unit_sphere", None, pu32, pf)
    sig("po_random_in_unit_disk", None, pu32, pf)
    sig("po_camera_get_ray", None, ctypes.POINTER(PoCamera), f, f, pu32, pf, pf)
    sig("po_closest_hit", i, ctypes.POINTER(PoTri), pi, i, pf, pf, f, pf)
    sig("po_sphere4_frames", None, i, i, i, i, i, i, i, pf, pu32, i)
    sig("po_scene_create", ctypes.c_void_p, pf, pi, i, pf, i, ctypes.POINTER(PoCamera), i)
    sig("po_scene_create2", ctypes.c_void_p, pf, pi, i, pf, pi, i, ctypes.c_void_p, i, ctypes.POINTER(PoCamera), i)
    sig("po_sphere_t", i, pf, f, pf, pf, f, pf)
    sig("po_reflect", None, pf, pf, pf)
    sig("po_refract", None, pf, pf, f, pf)
    sig("po_scene_destroy", None, ctypes.c_void_p)
    sig("po_mesh_frames", None, ctypes.c_void_p, i, i, i, i, i, i, i, pf, pu32, pu64, i)
    sig("po_mesh_sample", None, ctypes.c_void_p, i, i, i, i, i, i, pf, pi)
    sig("po_accumulate", u32, pf, pf, i)
    sig("po_rgba8", None, pf, ctypes.c_longlong, pu32)
    _lib = L
    return L


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def f3(v):
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def d3(v):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus) -> PoCamera:
    c = PoCamera()
    lib().po_camera_build(d3(lookfrom), d3(lookat), d3(vup), float(vfov), float(aspect), float(aperture),
                          float(focus), ctypes.byref(c))
    return c


def scene_camera(scene, width, height) -> PoCamera:
    return camera(scene.lookfrom, scene.lookat, scene.vup, scene.vfov, float(width) / float(height),
                  scene.aperture, scene.focus)


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def sphere4(width, height, first_frame, count, max_depth, y0=0, y1=None, accum=None, nthreads=None):
    """Legacy 4-sphere kernel restated (CudaPathTracerKernel.cu:136-179). Returns (out, accum)."""
    y1 = height if y1 is None else y1
    rows = y1 - y0
    acc = np.zeros((rows, width, 4), np.float32) if accum is None else np.array(accum, np.float32, copy=True)
    out = np.zeros((rows, width), np.uint32)
    lib().po_sphere4_frames(width, height, y0, y1, first_frame, count, max_depth, _p(acc, ctypes.c_float),
                            _p(out, ctypes.c_uint32), nthreads or default_threads())
    return out, acc


class MeshScene:
    """Oracle-side scene: triangles, spheres, materials (brute-force closest hit when accel=0,
    private BVH when 1)."""

    def __init__(self, scene, width, height, accel=1, cam: PoCamera = None):
        self.scene = scene
        self.width, self.height = width, height
        self.cam = cam if cam is not None else scene_camera(scene, width, height)
        self._v = np.ascontiguousarray(scene.verts, np.float32).reshape(-1, 9)
        self._m = np.ascontiguousarray(scene.tri_mat, np.int32)
        self._s = np.ascontiguousarray(getattr(scene, "spheres", np.zeros((0, 4))), np.float32).reshape(-1, 4)
        self._sm = np.ascontiguousarray(getattr(scene, "sph_mat", np.zeros(0)), np.int32)
        self._mats = np.ascontiguousarray(scene.materials())  # == po_material layout
        self.handle = lib().po_scene_create2(_p(self._v, ctypes.c_float), _p(self._m, ctypes.c_int),
                                             int(self._v.shape[0]), _p(self._s, ctypes.c_float),
                                             _p(self._sm, ctypes.c_int), int(self._s.shape[0]),
                                             self._mats.ctypes.data_as(ctypes.c_void_p), int(self._mats.shape[0]),
                                             ctypes.byref(self.cam), int(accel))

    def __del__(self):
        if getattr(self, "handle", None):
            lib().po_scene_destroy(self.handle)
            self.handle = None

    def frames(self, first_frame, count, max_depth, y0=0, y1=None, accum=None, nthreads=None):
        """Returns (out (rows,W) uint32, accum (rows,W,4) float32, segments, pixel_samples)."""
        y1 = self.height if y1 is None else y1
        rows = y1 - y0
        acc = np.zeros((rows, self.width, 4), np.float32) if accum is None else np.array(accum, np.float32, copy=True)
        out = np.zeros((rows, self.width), np.uint32)
        stats = np.zeros(2, np.uint64)
        lib().po_mesh_frames(self.handle, self.width, self.height, y0, y1, first_frame, count, max_depth,
                             _p(acc, ctypes.c_float), _p(out, ctypes.c_uint32), _p(stats, ctypes.c_uint64),
                             nthreads or default_threads())
        return out, acc, int(stats[0]), int(stats[1])

    def sample(self, x, y, frame, max_depth):
        rgb = np.zeros(3, np.float32)
        segs = ctypes.c_int()
        lib().po_mesh_sample(self.handle, self.width, self.height, x, y, frame, max_depth,
                             _p(rgb, ctypes.c_float), ctypes.byref(segs))
        return rgb, segs.value


def _f3(v):
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def sphere_t(c, r, o, d, tmin=0.001):
    """Contract sphere root (po_sphere_t): t or None."""
    t = ctypes.c_float()
    ok = lib().po_sphere_t(_f3(c), float(np.float32(r) * np.float32(r)), _f3(o), _f3(d), tmin, ctypes.byref(t))
    return t.value if ok else None


def reflect(v, n):
    out = (ctypes.c_float * 3)()
    lib().po_reflect(_f3(v), _f3(n), out)
    return np.array(out[:], np.float32)


def refract(uv, n, ratio):
    out = (ctypes.c_float * 3)()
    lib().po_refract(_f3(uv), _f3(n), float(ratio), out)
    return np.array(out[:], np.float32)


def tri_setup(v9) -> PoTri:
    t = PoTri()
    lib().po_tri_setup((ctypes.c_float * 9)(*[float(x) for x in v9]), ctypes.byref(t))
    return t


def tri_hit(tri: PoTri, o, d, tmin=0.001):
    t = ctypes.c_float()
    h = lib().po_tri_hit(ctypes.byref(tri), f3(o), f3(d), float(tmin), ctypes.byref(t))
    return bool(h), t.value


def sphere_hit(c, r, o, d, tmin=0.001, tmax=float("inf")):
    t = ctypes.c_float()
    n = (ctypes.c_float * 3)()
    front = ctypes.c_int()
    h = lib().po_sphere_hit(f3(c), float(r), f3(o), f3(d), float(tmin), float(tmax), ctypes.byref(t), n,
                            ctypes.byref(front))
    return bool(h), t.value, tuple(n), bool(front.value)


def aabb_hit(lo, hi, o, d, tmin=0.001, tmax=float("inf")):
    return bool(lib().po_aabb_hit(f3(lo), f3(hi), f3(o), f3(d), float(tmin), float(tmax)))


def closest_hit(scene, o, d, tmin=0.001):
    """Brute-force closest hit over the scene's triangles: (index or -1, t)."""
    tris = (PoTri * scene.num_tris)()
    for i in range(scene.num_tris):
        lib().po_tri_setup((ctypes.c_float * 9)(*scene.verts[i].tolist()), ctypes.byref(tris[i]))
    t = ctypes.c_float()
    idx = lib().po_closest_hit(tris, None, scene.num_tris, f3(o), f3(d), float(tmin), ctypes.byref(t))
    return idx, t.value


def argb_to_rgb(img: np.ndarray) -> np.ndarray:
    img = np.asarray(img, np.uint32)
    return np.stack([(img >> 16) & 255, (img >> 8) & 255, img & 255], axis=-1).astype(np.uint8)


def rgba8(acc: np.ndarray) -> np.ndarray:
    """The GL / Vulkan backends' RGBA8 UNORM words (include/hippt.h HIPPT_PIXEL_RGBA8) of an
    accumulation image (float32 [..., 4]), as the kernels write them with HIPPT_OPT_PIXEL_FORMAT 1."""
    a = np.ascontiguousarray(acc, dtype=np.float32)
    out = np.zeros(a.shape[:-1], np.uint32)
    lib().po_rgba8(_p(a, ctypes.c_float), a.size // 4, _p(out, ctypes.c_uint32))
    return out
