"""Process lifecycle of libhippt.so on the GPU: a process that leaves while a host-side
run-cost job (HIPPT_OPT_ITEM_ORDER automatic, item_order.h) is still computing, without calling
cudaPathTracerShutdown, exits normally.  The library's State is a function-local static destroyed
at exit; before round 5 its Ctx held a joinable std::thread, whose destructor called std::terminate
(SIGABRT).  The job threads are now detached and own their job (hippt_api.cpp CostJob)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import ctypes, sys
sys.path.insert(0, {pkg!r})
import hippt
from hippt import scenes
sc = scenes.cornell34()
pt = hippt.PathTracer()
pt.setOption(hippt.OPT_ITEM_ORDER, -1)
pt.uploadMesh(sc)
assert pt.initialize(1920, 1080), pt.lastError()
lib = hippt.load_library()
# each camera starts a cost job on a host thread; the renders go on in image order meanwhile
err = ctypes.c_char_p()
for k in range(3):
    cam = hippt.build_camera(lookfrom=(sc.lookfrom[0] + 10.0 * k, sc.lookfrom[1], sc.lookfrom[2]), lookat=sc.lookat,
                             vup=sc.vup, vfov=sc.vfov, aspect=1920 / 1080, aperture=sc.aperture, focus=sc.focus)
    assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
    assert lib.hipptRenderFramesAsync(0, 1, 8, None)
assert pt.synchronize()
print("leaving without shutdown", flush=True)
pt._lib = None  # no shutdown from __del__ either (its call then fails and is ignored)
"""


def test_exit_with_cost_job_in_flight_is_clean():
    code = SCRIPT.format(pkg=os.path.join(REPO, "qt-raytracer_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "leaving without shutdown" in r.stdout
