"""round 6: the sweep's slow settings (r6ad: 2 of 24 blob70k settings timed at 2-3% of the rate while
their trace time per step was normal) — the same call sequence with every host call timed, to find
the call that stalls.  Prints one JSON line per setting, plus every call over 50 ms."""
import itertools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
import hippt  # noqa: E402
from hippt import scenes  # noqa: E402

pt = hippt.PathTracer()
pt.setDevices([0])
sc = scenes.get_scene(sys.argv[1] if len(sys.argv) > 1 else "blob70k")
pt.uploadMesh(sc)
lib = pt._lib
assert pt.initialize(1920, 1080)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    pt.renderFrames(64, 8, copy=False)


def timed(name, fn, slow, log):
    t = time.perf_counter()
    r = fn()
    dt = time.perf_counter() - t
    if dt > 0.05:
        slow.append({"call": name, "s": round(dt, 3)})
    log.append(round(dt * 1e3, 2))
    return r


for rep in range(int(os.environ.get("REPS", "3"))):
    for le, ne in itertools.product([12, 17, 24, 32], [32, 48, 64]):
        slow, log = [], []
        pt.setOption(hippt.OPT_LEAF_EXIT, le)
        pt.setOption(hippt.OPT_NODE_EXIT, ne)
        timed("initialize", lambda: pt.initialize(1920, 1080), slow, log)
        timed("renderFrames", lambda: pt.renderFrames(64, 8, copy=False), slow, log)
        pt.resetStats()
        t = time.perf_counter()
        for k in range(5):
            timed(f"async{k}", lambda: lib.hipptRenderFramesAsync(0, 64, 8, None), slow, log)
        timed("synchronize", pt.synchronize, slow, log)
        dt = time.perf_counter() - t
        st = pt.stats()
        print(json.dumps({"rep": rep, "leafexit": le, "nodeexit": ne, "msamples_s": round(st["segments"] / dt / 1e6, 1),
                          "trace_ms_step": round(st["traceMs"] / 5, 3), "launches": st["traceLaunches"],
                          "call_ms": log, "slow": slow}), flush=True)
