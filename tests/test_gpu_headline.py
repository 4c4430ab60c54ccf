"""The BASELINE.json workloads at their real sizes (GPU), through the C ABI.

* configs[1] (Cornell-34) and configs[2] (blob70k), 1920x1080, 64 spp, 8 bounces: the WHOLE image
  the bench times equals the oracle's whole image (golden CRC32 of the ARGB words, SHA-256 of the
  accumulation floats, exact segment and sample counts; tests/golden/make_golden.py headline,
  oracle/pt_oracle.c over frames 0..63 with the running average of CudaPathTracerKernel.cu:157-178).
* configs[3] (blob70k, 3840x2160, 8 GPUs row-tiled) rehearsed on one GPU: 8 contexts on device 0
  (hipptSetDevices([0]*8), interleaved rows) and 8 one-process-per-GPU shares
  (hipptSetRowInterleave(r, 8), gathered on the host) each give the one-context image bit for bit,
  and sampled rows equal the oracle.  2 spp keeps the oracle's rows to seconds.
* configs[3] at its real sample count (3840x2160, 256 spp, 8 bounces): 16 rows of the image (top,
  through the mesh, bottom, and row 1610, whose pixel (1750, 1610) starts a short RNG cycle in
  frame 17) equal the oracle's rows after all 256 frames (tests/golden/make_golden.py headline4k),
  rendered as one context and as 8 hipptSetRowInterleave(r, 8) shares.
"""
import json
import os
import zlib

import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture()
def pt():
    t = hippt.PathTracer()
    t.setDevices([])
    t.setRowRange(0, 0)
    t.setOption(hippt.OPT_DEVICE_ROWS, 1)
    t.resetStats()
    yield t
    t.setDevices([])
    t.setRowRange(0, 0)
    hippt.load_library().cudaPathTracerShutdown()


@pytest.mark.parametrize("name", ["cornell34", "blob70k"])
def test_headline_image_equals_oracle_golden(pt, name):
    import hashlib
    with open(os.path.join(GOLDEN, f"oracle_headline_{name}_1920x1080_64.json")) as f:
        g = json.load(f)
    pt.uploadMesh(scenes.get_scene(name))
    assert pt.initialize(g["width"], g["height"]), pt.lastError()
    pt.resetStats()
    # the bench's call: one batch of all 64 frames, async, then the readback's sync
    assert pt.renderFramesAsync(g["spp"], g["max_depth"]), pt.lastError()
    px, acc = pt.readback()
    st = pt.stats()
    rows = [y for y in range(g["height"]) if zlib.crc32(px[y].tobytes()) & 0xFFFFFFFF != g["row_crc32"][y]]
    assert not rows, f"{len(rows)} rows differ from the oracle, first {rows[:8]}"
    assert zlib.crc32(px.tobytes()) & 0xFFFFFFFF == g["image_crc32"]
    assert hashlib.sha256(acc.tobytes()).hexdigest() == g["accum_sha256"]
    assert st["segments"] == g["segments"] and st["pixelSamples"] == g["pixel_samples"]


def test_config4_row_split_on_one_gpu(pt):
    w, h, spp, depth, n = 3840, 2160, 2, 8, 8
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFrames(spp, depth), pt.lastError()
    one = pt.readback()
    one_segs = pt.stats()["segments"]
    # 8 contexts on one device, interleaved rows (the in-process multi-GPU split)
    pt.setDevices([0] * n)
    pt.setOption(hippt.OPT_DEVICE_ROWS, 1)
    assert pt.initialize(w, h), pt.lastError()
    pt.resetStats()
    assert pt.renderFrames(spp, depth), pt.lastError()
    st = pt.stats()
    assert st["numDevices"] == n and st["segments"] == one_segs
    eight = pt.readback()
    assert np.array_equal(eight[0], one[0]) and eight[1].tobytes() == one[1].tobytes()
    assert np.array_equal(pt.hostPixels(), one[0])
    # 8 one-process-per-GPU shares (bench.py --gpus 8: rank r renders rows r, r+8, ...), gathered
    pt.setDevices([])
    px = np.zeros((h, w), np.uint32)
    acc = np.zeros((h, w, 4), np.float32)
    segs = 0
    for r in range(n):
        pt.setRowInterleave(r, n)
        assert pt.initialize(w, h), pt.lastError()
        pt.resetStats()
        assert pt.renderFrames(spp, depth), pt.lastError()
        segs += pt.stats()["segments"]
        got = pt.readback()
        px[r::n], acc[r::n] = got[0][r::n], got[1][r::n]
    assert segs == one_segs
    assert np.array_equal(px, one[0]) and acc.tobytes() == one[1].tobytes()
    # and the image is the oracle's on sampled rows (top, middle through the mesh, bottom)
    ms = po.MeshScene(sc, w, h, accel=1)
    for y0 in (0, h // 2 - 1, h - 2):
        ora = ms.frames(0, spp, depth, y0=y0, y1=y0 + 2)
        assert np.array_equal(one[0][y0:y0 + 2], ora[0])
        assert one[1][y0:y0 + 2].tobytes() == ora[1].tobytes()


def test_config4_full_spp_rows_equal_oracle_golden(pt):
    """configs[3]'s job at 256 spp: the frames 2..255 that the 2-spp split test above leaves out,
    including the short-cycle escape pixel, against the oracle's running average
    (CudaPathTracerKernel.cu:157-178) of all 256 frames, as one image and as the 8-way row split."""
    import hashlib
    with open(os.path.join(GOLDEN, "oracle_headline4k_blob70k_3840x2160_256.json")) as f:
        g = json.load(f)
    w, h, spp, depth = g["width"], g["height"], g["spp"], g["max_depth"]
    pt.uploadMesh(scenes.get_scene(g["scene"]))

    def check(px, acc, rows, what):
        for r in rows:
            y = r["y"]
            assert zlib.crc32(px[y].tobytes()) & 0xFFFFFFFF == r["crc32"], f"{what}: row {y} differs"
            assert hashlib.sha256(acc[y].tobytes()).hexdigest() == r["accum_sha256"], f"{what}: row {y}"

    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFramesAsync(spp, depth), pt.lastError()
    px, acc = pt.readback()
    check(px, acc, g["rows"], "one context")
    n = 8
    for k in range(n):
        rows = [r for r in g["rows"] if r["y"] % n == k]
        if not rows:
            continue
        pt.setRowInterleave(k, n)
        assert pt.initialize(w, h), pt.lastError()
        pt.resetStats()
        assert pt.renderFramesAsync(spp, depth), pt.lastError()
        px, acc = pt.readback()
        check(px, acc, rows, f"share {k}/{n}")


@pytest.mark.parametrize("name,share", [("cornell34", None), ("blob70k", None), ("cornell34", 8), ("blob70k", 8)])
def test_bench_steps_chained_equal_oracle_golden(pt, name, share):
    """bench.py's timed loop with chained batches (HIPPT_OPT_CHAIN 3 and 8): back-to-back async
    steps of frames 0..63 (each step's frame 0 restarts the average), as the whole image and as a
    1/8 interleaved row share (a SCALE rank).  The launches chain the steps, combine them beside
    their own paths and the readback flushes the last ones; the image is still the oracle's golden
    image (row CRCs, accumulation of the rows), and the segment and sample counts are exactly the
    steps' sum."""
    import hashlib
    with open(os.path.join(GOLDEN, f"oracle_headline_{name}_1920x1080_64.json")) as f:
        g = json.load(f)
    pt.uploadMesh(scenes.get_scene(name))
    if share:
        pt.setRowInterleave(share - 1, share)
    assert pt.initialize(g["width"], g["height"]), pt.lastError()
    lib = hippt.load_library()
    steps = 6 if share is None else 11
    pt.setOption(hippt.OPT_CHAIN, 3 if share is None else 8)
    pt.resetStats()
    for _ in range(steps):
        assert lib.hipptRenderFramesAsync(0, g["spp"], g["max_depth"], None)
    px, acc = pt.readback()
    st = pt.stats()
    ys = range(g["height"]) if share is None else range(share - 1, g["height"], share)
    rows = [y for y in ys if zlib.crc32(px[y].tobytes()) & 0xFFFFFFFF != g["row_crc32"][y]]
    assert not rows, f"{len(rows)} rows differ from the oracle, first {rows[:8]}"
    if share is None:
        assert hashlib.sha256(acc.tobytes()).hexdigest() == g["accum_sha256"]
        assert st["segments"] == steps * g["segments"] and st["pixelSamples"] == steps * g["pixel_samples"]
    else:
        assert st["pixelSamples"] == steps * len(ys) * g["width"] * g["spp"]
    pt.setRowRange(0, 0)
    pt.setOption(hippt.OPT_CHAIN, -1)

