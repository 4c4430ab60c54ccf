"""Host-only checks of libhippt.so (no GPU compute): exports, camera, BVH builder, errors."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    header = open(os.path.join(REPO, "include", "hippt.h")).read()
    declared = set(re.findall(r"\b((?:cuda|hip)PathTracer\w+|hippt[A-Z]\w*)\s*\(", header))
    out = subprocess.run(["nm", "-D", "--defined-only", hippt.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert declared, "parsed no declarations"
    assert declared <= exported, declared - exported
    assert declared == set(hippt.EXPORTS)
    lib = hippt.load_library()
    for name in declared:
        assert getattr(lib, name)


def test_reference_abi_signatures_are_exact():
    # CudaPathTracer.cpp:4-8 — the caller's extern "C" declarations
    header = open(os.path.join(REPO, "include", "hippt.h")).read()
    assert "bool cudaPathTracerInit(int width, int height, const char **errorMessage);" in header
    assert ("bool cudaPathTracerRender(int frameIndex, int maxDepth, const unsigned int **hostPixels,\n"
            "                          const char **errorMessage);") in header
    assert "void cudaPathTracerShutdown(void);" in header


def test_render_before_init_fails_with_reference_message():
    # CudaPathTracerKernel.cu:240-244 — "not initialized" error, no device work
    lib = hippt.load_library()
    lib.cudaPathTracerShutdown()
    e = ctypes.c_char_p()
    px = ctypes.POINTER(ctypes.c_uint)()
    assert not lib.cudaPathTracerRender(0, 8, ctypes.byref(px), ctypes.byref(e))
    assert b"not initialized" in e.value
    assert not lib.cudaPathTracerRender(0, 8, None, None)  # null out-pointers allowed
    lib.cudaPathTracerShutdown()
    lib.cudaPathTracerShutdown()  # idempotent


def test_python_mirror_reports_errors_like_cudapathtracer():
    pt = hippt.PathTracer()
    assert pt.frameIndex() == 0
    assert not pt.renderFrame(8)
    assert "not initialized" in pt.lastError()
    assert pt.frameIndex() == 0  # not incremented on failure (CudaPathTracer.cpp:45-50)
    assert pt.hostPixels() is None


@pytest.mark.parametrize("aspect", [16 / 9, 1.0, 0.5])
def test_camera_bitwise_equals_oracle(aspect):
    for sc in (scenes.cornell34(), scenes.blob70k()):
        a = hippt.build_camera(sc.lookfrom, sc.lookat, sc.vup, sc.vfov, aspect, sc.aperture, sc.focus).as_array()
        b = po.camera(sc.lookfrom, sc.lookat, sc.vup, sc.vfov, aspect, sc.aperture, sc.focus).as_array()
        assert a.tobytes() == b.tobytes()
    a = hippt.build_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 1.5, 0.1, 10).as_array()
    b = po.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 1.5, 0.1, 10).as_array()
    assert a.tobytes() == b.tobytes()


def test_options_validate():
    lib = hippt.load_library()
    assert lib.hipptSetOption(hippt.OPT_WAVE_THRESHOLD, 8)
    assert lib.hipptGetOption(hippt.OPT_WAVE_THRESHOLD) == 8
    assert not lib.hipptSetOption(hippt.OPT_WAVE_THRESHOLD, 65)
    assert not lib.hipptSetOption(hippt.OPT_CHUNK, 100)
    assert lib.hipptGetOption(hippt.OPT_CHUNK) == 0  # automatic (enqueue_locked)
    assert lib.hipptSetOption(hippt.OPT_CHUNK, 512) and lib.hipptGetOption(hippt.OPT_CHUNK) == 512
    assert lib.hipptSetOption(hippt.OPT_CHUNK, 0) and lib.hipptGetOption(hippt.OPT_CHUNK) == 0
    assert not lib.hipptSetOption(999, 1)
    assert lib.hipptSetOption(hippt.OPT_WAVE_THRESHOLD, -1)
    assert not lib.hipptSetOption(hippt.OPT_WAVE_THRESHOLD, -2)


@pytest.mark.parametrize("key,good,bad,default", [
    (hippt.OPT_LDS_TOP_NODES, (0, 1, 85, 1365), (-2, 1366), -1),
    (hippt.OPT_BVH_COLLAPSE, (-1, 0, 1), (-2, 2), -1),
    (hippt.OPT_BVH_NODE_COST, (1, 250, 100000), (0, 100001), 200),
    (hippt.OPT_BVH_LEAF4, (1, 8, 15), (0, 16), 4),
    (hippt.OPT_RNG_TABLE, (0, 1), (-1, 2), 0),
    (hippt.OPT_CAMERA_POOL, (-1, 0, 1), (-2, 2), -1),
    (hippt.OPT_FUSE_COMBINE, (-1, 0, 1), (-2, 2), -1),
    (hippt.OPT_ITEM_ORDER, (-1, 0, 1), (-2, 2), -1),
    (hippt.OPT_STACK_CAP, (0, 4, 30), (3, 31), 0),
    (hippt.OPT_BVH_QUANT, (-1, 0, 1, 2, 3), (-2, 4), -1),
    (hippt.OPT_WAVEFRONT_SORT, (-1, 0, 3, 6), (-2, 1, 2, 4, 7), -1),
    (hippt.OPT_CHAIN, (-1, 0, 1, 2, 8, 16), (-2, 17), -1),
    (hippt.OPT_CHAIN_AUDIT, (0, 1), (-1, 2), 0),
    (hippt.OPT_PIXEL_TILE, (-1, 0, 8, 16, 32), (-2, 4, 12, 64), -1),
])
def test_round2_options_round_trip(key, good, bad, default):
    """Each option accepts its documented range (include/hippt.h), reads back what was set,
    rejects values outside it without changing the setting, and starts at its default."""
    lib = hippt.load_library()
    assert lib.hipptGetOption(key) == default
    try:
        for v in good:
            assert lib.hipptSetOption(key, v), v
            assert lib.hipptGetOption(key) == v
        for v in bad:
            assert not lib.hipptSetOption(key, v), v
            assert lib.hipptGetOption(key) == good[-1]
    finally:
        assert lib.hipptSetOption(key, default)


def test_info_keys_before_any_render():
    """The read-only facts of the last megakernel render are 0 before one ran."""
    lib = hippt.load_library()
    assert lib.hipptGetOption(hippt.INFO_LDS_TOP_BYTES) >= 0
    assert lib.hipptGetOption(hippt.INFO_BLOCKS_PER_CU) >= 0
    assert not lib.hipptSetOption(hippt.INFO_LDS_TOP_BYTES, 1)


def test_mesh_upload_validates_inputs():
    pt = hippt.PathTracer()
    sc = scenes.cornell34()
    bad = scenes.Scene("bad", sc.verts, sc.tri_mat.copy(), sc.albedo)
    bad.tri_mat[3] = 7
    with pytest.raises(hippt.HipptError, match="material"):
        pt.uploadMesh(bad)
    empty = scenes.Scene("empty", np.zeros((0, 9), np.float32), np.zeros(0, np.int32), sc.albedo)
    with pytest.raises(hippt.HipptError, match="at least one triangle"):  # RayTracer.h:398-400
        pt.uploadMesh(empty)


def test_device_count_without_gpu_is_safe():
    assert hippt.device_count() >= 0


_OOM_CHILD = r"""
import ctypes, resource, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import hippt
from hippt import scenes
lib = hippt.load_library()
sc = scenes.blob70k()
v = np.ascontiguousarray(sc.verts, np.float32).reshape(-1, 9)
m = np.ascontiguousarray(sc.tri_mat, np.int32)
a = np.ascontiguousarray(sc.albedo, np.float32).reshape(-1, 3)
d3 = lambda t: (ctypes.c_double * 3)(*t)
def upload():
    e = ctypes.c_char_p()
    ok = lib.hipptUploadMesh(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                             m.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), v.shape[0],
                             a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), a.shape[0], d3(sc.lookfrom),
                             d3(sc.lookat), d3(sc.vup), float(sc.vfov), float(sc.aperture), float(sc.focus),
                             ctypes.byref(e))
    return ok, e.value
assert upload()[0]  # the same upload succeeds without the limit
vm = int(open("/proc/self/status").read().split("VmSize:")[1].split()[0]) * 1024
resource.setrlimit(resource.RLIMIT_AS, (vm + (4 << 20), resource.RLIM_INFINITY))
ok, msg = upload()
resource.setrlimit(resource.RLIMIT_AS, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))
print("RESULT", ok, msg)
assert not ok and msg and msg.startswith(b"HIP path tracer:"), (ok, msg)
"""


def test_allocation_failure_returns_false_not_terminate(tmp_path):
    """an exception inside an extern "C" entry point (here std::bad_alloc from the host
    BVH build of a valid blob70k upload under a lowered RLIMIT_AS) must come back as the reference's
    false + message convention (CudaPathTracerKernel.cu:181-184), not std::terminate the caller."""
    script = tmp_path / "oom_child.py"
    script.write_text(_OOM_CHILD)
    r = subprocess.run([sys.executable, str(script), os.path.join(REPO, "qt-raytracer_amd")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "RESULT False" in r.stdout
