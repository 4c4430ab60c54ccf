"""Seeded random host-call sequences through the chained path (HIPPT_OPT_CHAIN, the device side of
tests/native/chain_model.cpp's host model): asynchronous batches of random frame counts continuing
the run, repeating its frames or breaking its pattern, resets, camera moves, scene uploads,
pixel-format switches, readbacks in the middle, at random caps and item orders.  Every readback's
image and accumulation equal the same sequence with one launch per batch (HIPPT_OPT_CHAIN 0, itself
checked against the oracle by test_gpu_parity.py), and the device audit of every chained run is
clean (each batch traced once with its own frames, combined once, in order)."""
import ctypes
import os

import numpy as np
import pytest

import chain_audit
import hippt
from hippt import scenes

pytestmark = pytest.mark.gpu


def _apply(pt, lib, ops, chain, order, scs, w, h):
    """Runs one op list with HIPPT_OPT_CHAIN `chain`; returns every readback's (pixels, accum)."""
    pt.setOption(hippt.OPT_CHAIN, chain)
    pt.setOption(hippt.OPT_ITEM_ORDER, order)
    pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB)
    pt.uploadMesh(scs[0])
    assert pt.initialize(w, h), pt.lastError()
    err = ctypes.c_char_p()
    frame = 0
    out = []
    for op, arg in ops:
        if op == "next":  # the run's next frames
            assert lib.hipptRenderFramesAsync(frame, arg, 8, None), pt.lastError()
            frame += arg
        elif op == "again":  # frames from 0 again (each batch restarts the average)
            assert lib.hipptRenderFramesAsync(0, arg, 8, None), pt.lastError()
            frame = arg
        elif op == "jump":  # frames out of the run's pattern
            frame += arg
            assert lib.hipptRenderFramesAsync(frame, 2, 8, None), pt.lastError()
            frame += 2
        elif op == "reset":
            assert pt.resetAccumulation()
            frame = 0
        elif op == "camera":
            sc = scs[0]
            cam = hippt.build_camera(lookfrom=(sc.lookfrom[0] + arg, sc.lookfrom[1] + 0.5 * arg, sc.lookfrom[2]),
                                     lookat=sc.lookat, vup=sc.vup, vfov=sc.vfov, aspect=w / h,
                                     aperture=sc.aperture, focus=sc.focus)
            assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
        elif op == "scene":
            pt.uploadMesh(scs[arg])
        elif op == "format":
            pt.setOption(hippt.OPT_PIXEL_FORMAT, arg)
        elif op == "read":
            out.append(pt.readback())
    out.append(pt.readback())
    return out


def _ops(rng):
    # a sequence's usual batch size (a run needs the same frames per batch), sometimes another
    size = int(rng.choice([1, 8, 64, 256]))
    pick = lambda: size if rng.random() < 0.85 else int(rng.choice([1, 2, 8, 64]))  # noqa: E731
    ops = []
    for _ in range(int(rng.integers(10, 30))):
        r = rng.random()
        if r < 0.5:
            ops.append(("next", pick()))
        elif r < 0.60:
            ops.append(("again", pick()))
        elif r < 0.66:
            ops.append(("jump", int(rng.integers(1, 5))))
        elif r < 0.72:
            ops.append(("reset", 0))
        elif r < 0.79:
            ops.append(("camera", float(rng.uniform(-30, 30))))
        elif r < 0.83:
            ops.append(("scene", int(rng.integers(0, 2))))
        elif r < 0.87:
            ops.append(("format", int(rng.choice([hippt.PIXEL_ARGB, hippt.PIXEL_RGBA8]))))
        else:
            ops.append(("read", 0))
    return ops


# HIPPT_FUZZ_SEEDS widens the run (the suite's default is 16 sequences; profiles/round6 logs a longer one)
@pytest.mark.parametrize("seed", range(int(os.environ.get("HIPPT_FUZZ_SEEDS", "16"))))
def test_random_chained_sequences_equal_one_launch_per_batch(seed):
    rng = np.random.default_rng(1000 + seed)
    pt = hippt.PathTracer()
    pt.setDevices([])
    pt.setRowRange(0, 0)
    lib = hippt.load_library()
    try:
        first = ("cornell34", "blob70k", "cornell_mixed")[seed % 3]
        scs = [scenes.get_scene(first), scenes.get_scene("blob70k" if first != "blob70k" else "cornell34")]
        # (every 8th sequence at 320x180: launches long enough that later batches are posted while
        # they run, so the device moves into them inside the launch)
        w, h = (320, 180) if seed % 8 == 7 else [(45, 26), (128, 72), (96, 54)][seed % 3]
        if seed % 4 == 3:
            pt.setRowInterleave(seed % 2, 2)  # a rank's interleaved share
        ops = _ops(rng)
        chain = int(rng.choice([-1, 2, 3, 8, 16]))
        order = int(rng.choice([-1, 0, 1]))
        pt.setOption(hippt.OPT_CHAIN_AUDIT, 1)
        hippt.chain_audit()
        got = _apply(pt, lib, ops, chain, order, scs, w, h)
        runs = hippt.chain_audit()
        pt.setOption(hippt.OPT_CHAIN_AUDIT, 0)
        ref = _apply(pt, lib, ops, 0, order, scs, w, h)
        assert len(got) == len(ref)
        for k, (a, b) in enumerate(zip(got, ref)):
            diff = np.count_nonzero(a[0] != b[0])
            assert diff == 0 and a[1].tobytes() == b[1].tobytes(), \
                f"readback {k}: {diff} pixels differ (chain {chain}, order {order}, ops {ops})"
        problems = chain_audit.check(runs)
        assert not problems, f"{problems[:4]} (chain {chain}, order {order}, ops {ops})"
        # (how much chaining the sequence produced: runs, batches, and launches that took more than
        # their own batch or group)
        print(f"seed {seed}: chain {chain} order {order}: {len(runs)} runs, "
              f"{sum(r[0]['batches'] for r in runs)} batches in {sum(r[0]['launches'] for r in runs)} launches")
    finally:
        pt.setOption(hippt.OPT_CHAIN_AUDIT, 0)
        pt.setOption(hippt.OPT_CHAIN, -1)
        pt.setOption(hippt.OPT_ITEM_ORDER, -1)
        pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB)
        pt.setRowRange(0, 0)
        lib.cudaPathTracerShutdown()
