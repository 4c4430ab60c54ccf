"""Python host mirror of the reference backend interface, over libhippt.so (C ABI).

``PathTracer`` mirrors ``CudaPathTracer`` (CudaPathTracer.h:6-23 / .cpp:14-94): the same
methods (initialize, renderFrame, hostPixels, frameIndex, lastError), the same frame-index
bookkeeping (renderFrame passes the current index and increments it after success,
CudaPathTracer.cpp:41-57) and the same error behaviour (False + lastError()).  Extensions
(scene upload, batched frames, devices, row bands, counters) wrap the hippt* entry points
of include/hippt.h.

The product path is libhippt.so only: if it is missing the import fails loudly — there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

from . import scenes  # noqa: F401  (re-export)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libhippt.so")

SCENE_SPHERE4 = 0
SCENE_MESH = 1

OPT_COUNT_TRAVERSAL = 1
OPT_WAVE_THRESHOLD = 2
OPT_SCRATCH_MB = 3
OPT_CHUNK = 4
OPT_BLOCKS_PER_CU = 5
OPT_LDS_SCENE = 6
OPT_PATH_MODE = 8
OPT_WAVEFRONT_SLOTS = 9
OPT_BVH_LEAF = 10
OPT_BVH_TRAVERSAL_COST = 11
OPT_BVH_MAX_DEPTH = 12
OPT_DEVICE_ROWS = 13
OPT_LEAF_EXIT = 14
OPT_NODE_EXIT = 15
OPT_BVH_SAH = 16
OPT_BVH_WIDTH = 17
OPT_STACK_CAP = 18
OPT_BVH_QUANT = 19
OPT_LDS_TOP_NODES = 20
OPT_BVH_COLLAPSE = 21
OPT_BVH_NODE_COST = 22
OPT_BVH_LEAF4 = 23
OPT_RNG_TABLE = 24
OPT_CAMERA_POOL = 26
OPT_FUSE_COMBINE = 27
OPT_ITEM_ORDER = 28
OPT_WAVEFRONT_SORT = 29
OPT_CHAIN = 30
OPT_CHAIN_AUDIT = 31
OPT_PIXEL_TILE = 32
OPT_PIXEL_FORMAT = 25
PIXEL_ARGB = 0
PIXEL_RGBA8 = 1
INFO_LDS_TOP_BYTES = 100
INFO_BLOCKS_PER_CU = 101
INFO_CHUNK = 102
INFO_CHAIN_CAP = 103

# Every symbol include/hippt.h declares (checked by tests/test_abi_cpu.py).
EXPORTS = (
    "cudaPathTracerInit", "cudaPathTracerRender", "cudaPathTracerShutdown",
    "hipPathTracerInit", "hipPathTracerRender", "hipPathTracerShutdown",
    "hipptBuildCamera", "hipptUseBuiltinScene", "hipptUploadMesh", "hipptUploadScene", "hipptReadMesh",
    "hipptFreeMesh", "hipptSetCamera",
    "hipptDeviceCount", "hipptSetDevices", "hipptSetRowRange", "hipptSetRowInterleave",
    "hipptRenderFrames", "hipptRenderFramesAsync", "hipptSynchronize", "hipptRenderFramesPresent",
    "hipptLatestFrame", "hipptReadback",
    "hipptResetAccumulation", "hipptGetStats", "hipptResetStats", "hipptGetCounters", "hipptSetOption",
    "hipptGetOption",
    "hipptLastError", "hipptBvhBuild", "hipptBvhNodeCount", "hipptBvhDepth", "hipptBvhCopy", "hipptBvhFree",
    "hipptBvh4NodeCount", "hipptBvh4Depth", "hipptBvh4StackBound", "hipptBvh4Copy", "hipptBvh4QCopy", "hipptBvh4QNodeCount",
    "hipptActiveBvhWidth", "hipptChainAudit",
)


class HipptError(RuntimeError):
    pass


class Camera(ctypes.Structure):
    """hipptCamera (include/hippt.h), 80 bytes."""
    _fields_ = [("origin", ctypes.c_float * 3), ("llc", ctypes.c_float * 3), ("horizontal", ctypes.c_float * 3),
                ("vertical", ctypes.c_float * 3), ("u", ctypes.c_float * 3), ("v", ctypes.c_float * 3),
                ("lens_radius", ctypes.c_float), ("reserved", ctypes.c_float)]

    def as_array(self) -> np.ndarray:
        return np.frombuffer(bytes(self), dtype=np.float32).copy()


class Mesh(ctypes.Structure):
    """hipptMesh (include/hippt.h)."""
    _fields_ = [("verts", ctypes.POINTER(ctypes.c_float)), ("triGroup", ctypes.POINTER(ctypes.c_int)),
                ("numTris", ctypes.c_int), ("numGroups", ctypes.c_int),
                ("groupNames", ctypes.POINTER(ctypes.c_char_p)), ("owner_", ctypes.c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_ulonglong), ("pixelSamples", ctypes.c_ulonglong),
                ("nodeVisits", ctypes.c_ulonglong), ("triTests", ctypes.c_ulonglong),
                ("traceMs", ctypes.c_double), ("combineMs", ctypes.c_double),
                ("traceLaunches", ctypes.c_int), ("combineLaunches", ctypes.c_int),
                ("bvhNodes", ctypes.c_int), ("bvhDepth", ctypes.c_int), ("numTris", ctypes.c_int),
                ("numDevices", ctypes.c_int)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib: Optional[ctypes.CDLL] = None


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Loads libhippt.so (or $HIPPT_LIB, for build-variant experiments) and declares the C
    signatures.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("HIPPT_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise HipptError(f"{path} is missing: build it with `make -C qt-raytracer_amd` "
                         "(or __graft_entry__.build()); there is no fallback path")
    lib = ctypes.CDLL(path)
    c_int, c_bool, c_char_p, c_double, c_float = ctypes.c_int, ctypes.c_bool, ctypes.c_char_p, ctypes.c_double, ctypes.c_float
    pp_char = ctypes.POINTER(ctypes.c_char_p)
    p_uint = ctypes.POINTER(ctypes.c_uint)
    pp_uint = ctypes.POINTER(p_uint)
    p_float = ctypes.POINTER(ctypes.c_float)
    p_int = ctypes.POINTER(ctypes.c_int)
    p_double = ctypes.POINTER(ctypes.c_double)

    variant = bool(os.environ.get("HIPPT_LIB"))  # an older build under test may lack newer entry points

    def sig(name, res, *args):
        if variant and not hasattr(lib, name):
            return
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = list(args)

    for pre in ("cuda", "hip"):
        sig(f"{pre}PathTracerInit", c_bool, c_int, c_int, pp_char)
        sig(f"{pre}PathTracerRender", c_bool, c_int, c_int, pp_uint, pp_char)
        sig(f"{pre}PathTracerShutdown", None)
    sig("hipptBuildCamera", None, p_double, p_double, p_double, c_double, c_double, c_double, c_double,
        ctypes.POINTER(Camera))
    sig("hipptUseBuiltinScene", c_bool, c_int, pp_char)
    sig("hipptUploadMesh", c_bool, p_float, p_int, c_int, p_float, c_int, p_double, p_double, p_double,
        c_double, c_double, c_double, pp_char)
    sig("hipptUploadScene", c_bool, p_float, p_int, c_int, p_float, p_int, c_int, ctypes.c_void_p, c_int, p_double,
        p_double, p_double, c_double, c_double, c_double, pp_char)
    sig("hipptReadMesh", c_bool, c_char_p, ctypes.POINTER(Mesh), pp_char)
    sig("hipptFreeMesh", None, ctypes.POINTER(Mesh))
    sig("hipptSetCamera", c_bool, ctypes.POINTER(Camera), pp_char)
    sig("hipptDeviceCount", c_int)
    sig("hipptSetDevices", c_bool, p_int, c_int, pp_char)
    sig("hipptSetRowRange", c_bool, c_int, c_int, pp_char)
    sig("hipptSetRowInterleave", c_bool, c_int, c_int, pp_char)
    sig("hipptRenderFrames", c_bool, c_int, c_int, c_int, pp_uint, pp_char)
    sig("hipptRenderFramesAsync", c_bool, c_int, c_int, c_int, pp_char)
    sig("hipptSynchronize", c_bool, pp_char)
    sig("hipptRenderFramesPresent", c_bool, c_int, c_int, c_int, pp_char)
    sig("hipptLatestFrame", c_bool, pp_uint, ctypes.POINTER(c_int), pp_char)
    sig("hipptReadback", c_bool, p_uint, p_float, pp_char)
    sig("hipptResetAccumulation", c_bool, pp_char)
    sig("hipptGetStats", c_bool, ctypes.POINTER(Stats))
    sig("hipptResetStats", None)
    sig("hipptGetCounters", c_int, ctypes.POINTER(ctypes.c_ulonglong), c_int)
    sig("hipptSetOption", c_bool, c_int, ctypes.c_longlong)
    sig("hipptGetOption", ctypes.c_longlong, c_int)
    sig("hipptLastError", c_char_p)
    sig("hipptBvhBuild", ctypes.c_void_p, p_float, c_int, c_float, pp_char)
    sig("hipptBvhNodeCount", c_int, ctypes.c_void_p)
    sig("hipptBvhDepth", c_int, ctypes.c_void_p)
    sig("hipptBvhCopy", None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), p_int)
    sig("hipptBvhFree", None, ctypes.c_void_p)
    sig("hipptActiveBvhWidth", c_int)
    sig("hipptBvh4NodeCount", c_int, ctypes.c_void_p)
    sig("hipptBvh4Depth", c_int, ctypes.c_void_p)
    sig("hipptBvh4StackBound", c_int, ctypes.c_void_p)
    sig("hipptBvh4Copy", None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32))
    sig("hipptBvh4QCopy", None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32))
    sig("hipptBvh4QNodeCount", c_int, ctypes.c_void_p)
    sig("hipptChainAudit", c_int, p_uint, c_int)
    _lib = lib
    return lib


def _err(e: ctypes.c_char_p, default: str) -> str:
    return e.value.decode() if e.value else default


def _ptr(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _d3(v) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def read_mesh(path: str):
    """hipptReadMesh: (verts (n, 9) float32, tri_group (n,) int32, group names) of an OBJ/PLY file."""
    lib = load_library()
    m = Mesh()
    e = ctypes.c_char_p()
    if not lib.hipptReadMesh(os.fsencode(path), ctypes.byref(m), ctypes.byref(e)):
        raise HipptError(_err(e, f"cannot read {path}"))
    try:
        n = m.numTris
        verts = np.ctypeslib.as_array(m.verts, shape=(n * 9,)).reshape(n, 9).copy()
        groups = np.ctypeslib.as_array(m.triGroup, shape=(n,)).copy()
        names = [m.groupNames[g].decode() for g in range(m.numGroups)]
    finally:
        lib.hipptFreeMesh(ctypes.byref(m))
    return verts, groups, names


def build_camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus) -> Camera:
    lib = load_library()
    cam = Camera()
    lib.hipptBuildCamera(_d3(lookfrom), _d3(lookat), _d3(vup), float(vfov), float(aspect), float(aperture),
                         float(focus), ctypes.byref(cam))
    return cam


class Bvh:
    """Host BVH built by libhippt (hipptBvhBuild): nodes (N,16) uint32 and triangle order; the
    4-wide tree collapsed from it: nodes4 (M,32) uint32, depth4, stack_bound4."""

    def __init__(self, verts: np.ndarray, extent_hint: float = 0.0):
        lib = load_library()
        v = np.ascontiguousarray(verts, dtype=np.float32).reshape(-1, 9)
        e = ctypes.c_char_p()
        h = lib.hipptBvhBuild(_ptr(v, ctypes.c_float), int(v.shape[0]), float(extent_hint), ctypes.byref(e))
        if not h:
            raise HipptError(_err(e, "BVH build failed"))
        try:
            n = lib.hipptBvhNodeCount(h)
            self.depth = lib.hipptBvhDepth(h)
            self.nodes = np.zeros((n, 16), dtype=np.uint32)
            self.order = np.zeros(v.shape[0], dtype=np.int32)
            lib.hipptBvhCopy(h, _ptr(self.nodes, ctypes.c_uint32), _ptr(self.order, ctypes.c_int))
            self.depth4 = lib.hipptBvh4Depth(h)
            self.stack_bound4 = lib.hipptBvh4StackBound(h)
            self.nodes4 = np.zeros((lib.hipptBvh4NodeCount(h), 32), dtype=np.uint32)
            lib.hipptBvh4Copy(h, _ptr(self.nodes4, ctypes.c_uint32))
            self.nodes4q = np.zeros((lib.hipptBvh4QNodeCount(h), 16), dtype=np.uint32)
            lib.hipptBvh4QCopy(h, _ptr(self.nodes4q, ctypes.c_uint32))
        finally:
            lib.hipptBvhFree(h)


class PathTracer:
    """Mirror of CudaPathTracer (CudaPathTracer.h:6-23) over the HIP backend."""

    def __init__(self):
        self._lib = load_library()
        self._width = 0
        self._height = 0
        self._frame_index = 0
        self._pixels: Optional[ctypes.POINTER] = None
        self._last_error = ""

    def __del__(self):  # ~CudaPathTracer -> cudaPathTracerShutdown (CudaPathTracer.cpp:14-18)
        try:
            self._lib.cudaPathTracerShutdown()
        except Exception:
            pass

    # --- CudaPathTracer interface -------------------------------------------------------------
    def initialize(self, width: int, height: int) -> bool:
        self._width, self._height = int(width), int(height)
        self._frame_index = 0
        self._pixels = None
        e = ctypes.c_char_p()
        if not self._lib.cudaPathTracerInit(self._width, self._height, ctypes.byref(e)):
            self._last_error = _err(e, "HIP initialization failed")
            return False
        return True

    def renderFrame(self, maxDepth: int) -> bool:  # noqa: N802 (reference name)
        e = ctypes.c_char_p()
        px = ctypes.POINTER(ctypes.c_uint)()
        if not self._lib.cudaPathTracerRender(self._frame_index, int(maxDepth), ctypes.byref(px), ctypes.byref(e)):
            self._last_error = _err(e, "HIP render failed")
            return False
        self._pixels = px
        self._frame_index += 1
        return True

    def hostPixels(self) -> Optional[np.ndarray]:  # noqa: N802
        """Copy of the library-owned W*H ARGB frame (row 0 = v = 0), or None before a render."""
        if not self._pixels:
            return None
        n = self._width * self._height
        return np.ctypeslib.as_array(self._pixels, shape=(n,)).reshape(self._height, self._width).copy()

    def frameIndex(self) -> int:  # noqa: N802
        return self._frame_index

    def lastError(self) -> str:  # noqa: N802
        return self._last_error

    # --- GpuPathTracer-shaped extensions (GpuPathTracer.h:9-38) -------------------------------
    def renderFrames(self, samplesPerFrame: int, maxDepth: int, copy: bool = True) -> bool:  # noqa: N802
        """Renders samplesPerFrame frames at once, continuing the frame index."""
        e = ctypes.c_char_p()
        px = ctypes.POINTER(ctypes.c_uint)()
        ok = self._lib.hipptRenderFrames(self._frame_index, int(samplesPerFrame), int(maxDepth),
                                         ctypes.byref(px) if copy else None, ctypes.byref(e))
        if not ok:
            self._last_error = _err(e, "HIP render failed")
            return False
        if copy:
            self._pixels = px
        self._frame_index += int(samplesPerFrame)
        return True

    def renderFramesAsync(self, samplesPerFrame: int, maxDepth: int) -> bool:  # noqa: N802
        e = ctypes.c_char_p()
        if not self._lib.hipptRenderFramesAsync(self._frame_index, int(samplesPerFrame), int(maxDepth), ctypes.byref(e)):
            self._last_error = _err(e, "HIP render failed")
            return False
        self._frame_index += int(samplesPerFrame)
        return True

    def renderFramesPresent(self, samplesPerFrame: int, maxDepth: int) -> bool:  # noqa: N802
        """Enqueues frames plus a copy into the next pinned hand-off frame; does not wait."""
        e = ctypes.c_char_p()
        if not self._lib.hipptRenderFramesPresent(self._frame_index, int(samplesPerFrame), int(maxDepth),
                                                  ctypes.byref(e)):
            self._last_error = _err(e, "HIP render failed")
            return False
        self._frame_index += int(samplesPerFrame)
        return True

    def latestFrame(self):  # noqa: N802
        """Non-blocking: (ARGB (H, W) copy or None, frames accumulated in it)."""
        e = ctypes.c_char_p()
        px = ctypes.POINTER(ctypes.c_uint)()
        n = ctypes.c_int()
        if not self._lib.hipptLatestFrame(ctypes.byref(px), ctypes.byref(n), ctypes.byref(e)):
            raise HipptError(_err(e, "latest frame failed"))
        if not px:
            return None, 0
        h, w = self._height, self._width
        return np.ctypeslib.as_array(px, shape=(h * w,)).reshape(h, w).copy(), n.value

    def synchronize(self) -> bool:
        e = ctypes.c_char_p()
        if not self._lib.hipptSynchronize(ctypes.byref(e)):
            self._last_error = _err(e, "HIP synchronize failed")
            return False
        return True

    def resetAccumulation(self) -> bool:  # noqa: N802
        e = ctypes.c_char_p()
        if not self._lib.hipptResetAccumulation(ctypes.byref(e)):
            self._last_error = _err(e, "reset failed")
            return False
        self._frame_index = 0
        return True

    def readback(self, y0: int = 0, y1: Optional[int] = None):
        """(pixels (H,W) uint32, accum (H,W,4) float32) of the current image; rows outside this
        process's row range are zero."""
        pixels = np.zeros((self._height, self._width), dtype=np.uint32)
        accum = np.zeros((self._height, self._width, 4), dtype=np.float32)
        e = ctypes.c_char_p()
        if not self._lib.hipptReadback(_ptr(pixels, ctypes.c_uint), _ptr(accum, ctypes.c_float), ctypes.byref(e)):
            raise HipptError(_err(e, "readback failed"))
        y1 = self._height if y1 is None else y1
        return pixels[y0:y1], accum[y0:y1]

    # --- scene / devices / counters -------------------------------------------------------------
    def useBuiltinScene(self, scene_id: int = SCENE_SPHERE4) -> None:  # noqa: N802
        e = ctypes.c_char_p()
        if not self._lib.hipptUseBuiltinScene(int(scene_id), ctypes.byref(e)):
            raise HipptError(_err(e, "bad scene"))

    def uploadScene(self, scene) -> None:  # noqa: N802
        """hipptUploadScene: triangles + spheres + materials (hippt.scenes.Scene)."""
        v = np.ascontiguousarray(scene.verts, dtype=np.float32).reshape(-1, 9)
        m = np.ascontiguousarray(scene.tri_mat, dtype=np.int32)
        sp = np.ascontiguousarray(scene.spheres, dtype=np.float32).reshape(-1, 4)
        sm = np.ascontiguousarray(scene.sph_mat, dtype=np.int32)
        mats = np.ascontiguousarray(scene.materials())
        e = ctypes.c_char_p()
        ok = self._lib.hipptUploadScene(_ptr(v, ctypes.c_float), _ptr(m, ctypes.c_int), int(v.shape[0]),
                                        _ptr(sp, ctypes.c_float), _ptr(sm, ctypes.c_int), int(sp.shape[0]),
                                        mats.ctypes.data_as(ctypes.c_void_p), int(mats.shape[0]),
                                        _d3(scene.lookfrom), _d3(scene.lookat), _d3(scene.vup), float(scene.vfov),
                                        float(scene.aperture), float(scene.focus), ctypes.byref(e))
        if not ok:
            raise HipptError(_err(e, "scene upload failed"))

    def uploadMesh(self, scene) -> None:  # noqa: N802
        """hipptUploadMesh for Lambertian triangle scenes; other scenes go through uploadScene."""
        if not getattr(scene, "lambertian_triangles", True):
            return self.uploadScene(scene)
        v = np.ascontiguousarray(scene.verts, dtype=np.float32).reshape(-1, 9)
        m = np.ascontiguousarray(scene.tri_mat, dtype=np.int32)
        a = np.ascontiguousarray(scene.albedo, dtype=np.float32).reshape(-1, 3)
        e = ctypes.c_char_p()
        ok = self._lib.hipptUploadMesh(_ptr(v, ctypes.c_float), _ptr(m, ctypes.c_int), int(v.shape[0]),
                                       _ptr(a, ctypes.c_float), int(a.shape[0]), _d3(scene.lookfrom),
                                       _d3(scene.lookat), _d3(scene.vup), float(scene.vfov),
                                       float(scene.aperture), float(scene.focus), ctypes.byref(e))
        if not ok:
            raise HipptError(_err(e, "mesh upload failed"))

    def setDevices(self, device_ids: Sequence[int]) -> None:  # noqa: N802
        arr = (ctypes.c_int * max(1, len(device_ids)))(*device_ids)
        e = ctypes.c_char_p()
        if not self._lib.hipptSetDevices(arr, len(device_ids), ctypes.byref(e)):
            raise HipptError(_err(e, "bad devices"))

    def setRowRange(self, y0: int, y1: int) -> None:  # noqa: N802
        e = ctypes.c_char_p()
        if not self._lib.hipptSetRowRange(int(y0), int(y1), ctypes.byref(e)):
            raise HipptError(_err(e, "bad row range"))

    def setRowInterleave(self, phase: int, stride: int) -> None:  # noqa: N802
        """Render rows phase, phase+stride, ... (one process per GPU: phase=rank, stride=world)."""
        e = ctypes.c_char_p()
        if not self._lib.hipptSetRowInterleave(int(phase), int(stride), ctypes.byref(e)):
            raise HipptError(_err(e, "bad row interleave"))

    def setOption(self, key: int, value: int) -> None:  # noqa: N802
        if not self._lib.hipptSetOption(int(key), int(value)):
            raise HipptError(f"invalid option {key}={value}")

    def stats(self) -> dict:
        s = Stats()
        if not self._lib.hipptGetStats(ctypes.byref(s)):
            raise HipptError("hipptGetStats failed")
        return s.as_dict()

    PHASES = ("outer", "camera", "traversal_round", "node", "leaf", "triangle", "shade", "sphere_reject")

    def counters(self) -> dict:
        """Raw device counters incl. per-phase SIMD efficiency (counting builds)."""
        buf = (ctypes.c_ulonglong * 32)()
        n = self._lib.hipptGetCounters(buf, 32)
        v = list(buf)[:n]
        out = {"segments": v[0], "pixelSamples": v[1], "nodeVisits": v[2], "triTests": v[3]}
        for k, name in enumerate(self.PHASES):
            w, l = v[4 + 2 * k], v[5 + 2 * k]
            out[name] = {"wave": w, "lane": l, "simd_eff": round(l / (64 * w), 4) if w else None}
        # 4-wide node visits by number of hit children (0..4)
        out["hit_children"] = v[20:25]
        # of the visits with none hit: those with a child box hit before the closest-hit cut
        out["culled_by_best_t"] = v[25]
        # node visits served by the LDS copy of the top of a global-memory tree
        out["lds_top_visits"] = v[26] if len(v) > 26 else 0
        return out

    def resetStats(self) -> None:  # noqa: N802
        self._lib.hipptResetStats()


AUDIT_MAGIC = 0xC4A1D17
AUDIT_BATCHES = 256


def chain_audit() -> list:
    """The chained runs closed since the last call (HIPPT_OPT_CHAIN_AUDIT, include/hippt.h
    hipptChainAudit): a list of (header dict, records uint32 array [batches + 1, 16]).  Synchronises."""
    lib = load_library()
    runs = []
    while True:
        buf = np.zeros(1 << 22, np.uint32)
        n = lib.hipptChainAudit(_ptr(buf, ctypes.c_uint), buf.size)
        if n < 0:
            raise HipptError("hipptChainAudit failed")
        if n == 0:
            return runs
        k = 0
        while k < n:
            h = buf[k:k + 16]
            assert h[0] == AUDIT_MAGIC, "audit stream out of step"
            hdr = dict(run=int(h[1]), device=int(h[2]), firstFrame=int(h[3].astype(np.int32)),
                       step=int(h[4].astype(np.int32)), frames=int(h[5]), bandPixels=int(h[6]), totalItems=int(h[7]),
                       batches=int(h[8]), launches=int(h[9]), slots=int(h[10]), overflow=int(h[11]))
            recs = min(hdr["batches"], AUDIT_BATCHES) + 1
            runs.append((hdr, buf[k + 16:k + 16 + recs * 16].reshape(recs, 16).copy()))
            k += 16 + recs * 16


def device_count() -> int:
    return int(load_library().hipptDeviceCount())


def row_band(rank: int, world: int, height: int):
    """Contiguous row band of rank in [0, world): rows [floor(r*H/N), floor((r+1)*H/N))."""
    return (rank * height) // world, ((rank + 1) * height) // world
