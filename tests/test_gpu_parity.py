"""GPU parity: libhippt.so on an MI355X vs the CPU oracle (oracle/pt_oracle.c), bit-exact.

Bar: integer/byte outputs (ARGB words, segment counts) identical; accumulation floats
bit-identical (the arithmetic contract makes every float op the same on both sides).
All calls go through the C ABI (legacy cudaPathTracer* and hippt* extensions).
"""
import os

import numpy as np
import pytest

import chain_audit
import hippt
import pyoracle as po
from hippt import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture()
def pt():
    """The library's defaults, except that the item order is computed on the render path
    (HIPPT_OPT_ITEM_ORDER 1) rather than by the detached cost job of the automatic mode, so that
    host timing does not choose the code path a test runs (a green run then proves only
    one interleaving); the automatic mode has tests of its own.  Every chained run of every test is
    audited (HIPPT_OPT_CHAIN_AUDIT, tests/chain_audit.py): each batch traced once with its own frames,
    combined once, in order."""
    t = hippt.PathTracer()
    t.setDevices([])
    t.setRowRange(0, 0)
    t.setOption(hippt.OPT_DEVICE_ROWS, 1)
    t.useBuiltinScene(hippt.SCENE_SPHERE4)
    for k, v in ((hippt.OPT_WAVE_THRESHOLD, -1), (hippt.OPT_SCRATCH_MB, 32768), (hippt.OPT_CHUNK, 0),
                 (hippt.OPT_COUNT_TRAVERSAL, 0), (hippt.OPT_BLOCKS_PER_CU, 0), (hippt.OPT_LDS_SCENE, 1),
                 (hippt.OPT_PATH_MODE, 0), (hippt.OPT_WAVEFRONT_SLOTS, 1 << 24), (hippt.OPT_LEAF_EXIT, -1),
                 (hippt.OPT_NODE_EXIT, -1), (hippt.OPT_BVH_SAH, 1), (hippt.OPT_BVH_WIDTH, 0),
                 (hippt.OPT_STACK_CAP, 0), (hippt.OPT_BVH_QUANT, -1), (hippt.OPT_LDS_TOP_NODES, -1),
                 (hippt.OPT_RNG_TABLE, 0), (hippt.OPT_BVH_COLLAPSE, -1), (hippt.OPT_BVH_NODE_COST, 200),
                 (hippt.OPT_BVH_LEAF4, 4), (hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB),
                 (hippt.OPT_CAMERA_POOL, -1), (hippt.OPT_FUSE_COMBINE, -1), (hippt.OPT_ITEM_ORDER, 1),
                 (hippt.OPT_WAVEFRONT_SORT, -1), (hippt.OPT_CHAIN, -1), (hippt.OPT_CHAIN_AUDIT, 1)):
        t.setOption(k, v)
    t.resetStats()
    hippt.chain_audit()  # (drops records of earlier tests)
    yield t
    runs = hippt.chain_audit()
    t.setOption(hippt.OPT_CHAIN_AUDIT, 0)
    hippt.load_library().cudaPathTracerShutdown()
    t.audited = runs
    problems = chain_audit.check(runs)
    assert not problems, f"{len(problems)} chain audit problems in {len(runs)} runs: {problems[:6]}"


def _assert_same(gpu_px, gpu_acc, ora_px, ora_acc):
    diff = np.count_nonzero(gpu_px != ora_px)
    assert diff == 0, f"{diff} of {ora_px.size} pixels differ"
    assert gpu_acc.tobytes() == ora_acc.tobytes()


# ---- legacy 4-sphere scene (CudaPathTracerKernel.cu semantics) ----------------------------------
@pytest.mark.parametrize("w,h", [(160, 90), (7, 5), (1, 1), (64, 1)])
def test_legacy_abi_frames_match_oracle(pt, w, h):
    assert pt.initialize(w, h), pt.lastError()
    for _ in range(3):
        assert pt.renderFrame(8), pt.lastError()
    assert pt.frameIndex() == 3
    px = pt.hostPixels()
    _, acc = pt.readback()
    ora_px, ora_acc = po.sphere4(w, h, 0, 3, 8)
    _assert_same(px, acc, ora_px, ora_acc)


@pytest.mark.parametrize("w,h,share", [(320, 240, None), (512, 256, (1, 2)), (1920, 1080, None)])
def test_legacy_large_frames_match_oracle(pt, w, h, share):
    """Blocking frames at the app's size (1920x1080) and at an interleaved row share: the host
    pixels the call hands out and the accumulation are the oracle's, frame after frame."""
    if share:
        pt.setRowInterleave(*share)
    assert pt.initialize(w, h), pt.lastError()
    frames = 2 if w == 1920 else 3
    for _ in range(frames):
        assert pt.renderFrame(8), pt.lastError()
    px = pt.hostPixels()
    _, acc = pt.readback()
    ora_px, ora_acc = po.sphere4(w, h, 0, frames, 8)
    if share:
        r, n = share
        _assert_same(px[r::n], acc[r::n], ora_px[r::n], ora_acc[r::n])
    else:
        _assert_same(px, acc, ora_px, ora_acc)


def test_legacy_reinit_resets_accumulation(pt):
    # RayTracerFboItem.cpp:520-521 calls initialize again on frame 0
    assert pt.initialize(32, 16)
    assert pt.renderFrame(4)
    assert pt.initialize(32, 16)
    assert pt.renderFrame(4)
    ora_px, _ = po.sphere4(32, 16, 0, 1, 4)
    assert np.array_equal(pt.hostPixels(), ora_px)


def test_legacy_batched_frames_equal_single_frames(pt):
    assert pt.initialize(96, 64)
    assert pt.renderFrames(5, 6)
    a = pt.readback()
    assert pt.initialize(96, 64)
    for _ in range(5):
        assert pt.renderFrame(6)
    b = pt.readback()
    _assert_same(a[0], a[1], b[0], b[1])


@pytest.mark.parametrize("depth", [0, 1, 50])
def test_legacy_depth_edge_cases(pt, depth):
    assert pt.initialize(40, 30)
    assert pt.renderFrames(2, depth)
    px, acc = pt.readback()
    ora_px, ora_acc = po.sphere4(40, 30, 0, 2, depth)
    _assert_same(px, acc, ora_px, ora_acc)


# ---- triangle meshes -------------------------------------------------------------------------------
@pytest.mark.parametrize("name,w,h,spp,depth", [
    ("cornell34", 256, 256, 4, 4),  # BASELINE configs[0] (the CPU plumbing/parity case), whole image
    ("cornell34", 96, 64, 8, 8),
    ("cornell34", 33, 17, 3, 4),
    ("blob70k", 64, 48, 4, 8),
    ("blob70k", 17, 9, 2, 2),
])
def test_mesh_matches_oracle(pt, name, w, h, spp, depth):
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFrames(spp, depth), pt.lastError()
    px, acc = pt.readback()
    ora_px, ora_acc, segs, samples = po.MeshScene(sc, w, h).frames(0, spp, depth)
    _assert_same(px, acc, ora_px, ora_acc)
    st = pt.stats()
    assert st["segments"] == segs and st["pixelSamples"] == samples


def test_reinitialize_reuses_work_buffers(pt):
    """A re-initialization keeps the destroyed contexts' big work buffers (sample scratch, chain ring,
    spill area) for the new contexts of the device (a fresh 13 GB ring took up to 5.9 s to allocate,
    DESIGN_LOG.md §A.R6 r6af): sizes that grow and shrink, blocking and chained batches, blob70k's
    spilling traversal and Cornell — every image the oracle's, whichever kept buffer it landed in."""
    lib = hippt.load_library()
    seq = [("blob70k", 64, 48, 3), ("blob70k", 20, 11, 2), ("cornell34", 96, 64, 2), ("blob70k", 80, 40, 3),
           ("cornell34", 33, 17, 4), ("blob70k", 64, 48, 3)]
    for name, w, h, frames in seq:
        sc = scenes.get_scene(name)
        pt.uploadMesh(sc)
        assert pt.initialize(w, h), pt.lastError()
        assert pt.renderFrames(1, 8), pt.lastError()  # blocking
        for f in range(1, frames):  # then asynchronous one-frame batches (the chained path)
            assert lib.hipptRenderFramesAsync(f, 1, 8, None), pt.lastError()
        px, acc = pt.readback()
        ora_px, ora_acc, _, _ = po.MeshScene(sc, w, h).frames(0, frames, 8)
        _assert_same(px, acc, ora_px, ora_acc)


@pytest.mark.parametrize("name,w,h,spp,depth,slots,width,cap", [
    ("cornell34", 96, 64, 8, 8, 1 << 21, 0, 0),
    ("cornell34", 33, 17, 3, 4, 64, 2, 0),
    ("blob70k", 64, 48, 4, 8, 1000, 0, 0),
    ("blob70k", 64, 48, 4, 8, 5000, 0, 6),
    ("blob70k", 20, 11, 2, 1, 100, 2, 0),
    ("cornell34", 40, 30, 4, 50, 1 << 20, 0, 0),
    ("blob70k", 32, 24, 3, 1, 1 << 20, 0, 0),
])
def test_wavefront_matches_oracle(pt, name, w, h, spp, depth, slots, width, cap):
    """The wavefront variant (BASELINE config 5) is bit-identical to the oracle/megakernel,
    including with a path pool much smaller than the work (many regenerate rounds), over the
    2-wide and the 4-wide trees (a small LDS stack cap forces spills to the global area), and
    with a pool that holds the whole batch (at most maxDepth iterations, the queue poll ending a
    deep maxDepth early)."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, 1)
    pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, slots)
    pt.setOption(hippt.OPT_BVH_WIDTH, width)
    pt.setOption(hippt.OPT_STACK_CAP, cap)
    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFrames(spp, depth), pt.lastError()
    px, acc = pt.readback()
    ora_px, ora_acc, segs, samples = po.MeshScene(sc, w, h).frames(0, spp, depth)
    _assert_same(px, acc, ora_px, ora_acc)
    st = pt.stats()
    assert st["segments"] == segs and st["pixelSamples"] == samples


@pytest.mark.parametrize("name,w,h", [("cornell34", 96, 54), ("blob70k", 80, 45), ("cornell_mixed", 64, 40),
                                      ("random_scene", 77, 41)])
def test_wavefront_sort_does_not_change_results(pt, name, w, h):
    """HIPPT_OPT_WAVEFRONT_SORT: the shade kernel's appends ordered by direction octant (3) or octant
    and scene-box cell (6) per block; the image and the counts are the oracle's for every key, with
    a pool small enough that paths regenerate (slots shared between generations)."""
    sc = scenes.get_scene(name)
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, 1)
    for slots in (1 << 24, 4096):
        pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, slots)
        for key in (3, 6, 0):
            pt.setOption(hippt.OPT_WAVEFRONT_SORT, key)
            assert pt.initialize(w, h), pt.lastError()
            pt.resetStats()
            assert pt.renderFrames(3, 8), pt.lastError()
            got = pt.readback()
            _assert_same(got[0], got[1], ora[0], ora[1])
            st = pt.stats()
            assert st["segments"] == ora[2] and st["pixelSamples"] == ora[3]


@pytest.mark.parametrize("name", ["blob70k", "random_scene"])
@pytest.mark.parametrize("quant", [0, 1, 3])
def test_wavefront_node_formats_match_oracle(pt, name, quant):
    """The wavefront's extend kernel over a tree in global memory with float, 8-bit and
    half-precision nodes (HIPPT_OPT_BVH_QUANT 0 / 1 / 3), the top of each in LDS: the oracle's image,
    segment and sample counts."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    pt.setOption(hippt.OPT_PATH_MODE, 1)
    pt.setOption(hippt.OPT_BVH_QUANT, quant)
    w, h = (40, 24) if name == "random_scene" else (56, 40)
    assert pt.initialize(w, h), pt.lastError()
    pt.resetStats()
    assert pt.renderFrames(3, 8), pt.lastError()
    px, acc = pt.readback()
    ora_px, ora_acc, segs, samples = po.MeshScene(sc, w, h).frames(0, 3, 8)
    _assert_same(px, acc, ora_px, ora_acc)
    st = pt.stats()
    assert st["segments"] == segs and st["pixelSamples"] == samples


@pytest.mark.parametrize("slots", [1 << 21, 1 << 24])
def test_wavefront_equals_megakernel_1080p(pt, slots):
    """Full-width frames; 2^21 slots regenerate (shards refill unevenly), 2^24 hold every path."""
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, slots)
    got = []
    for mode in (0, 1):
        pt.setOption(hippt.OPT_PATH_MODE, mode)
        assert pt.initialize(1920, 1080)
        assert pt.renderFrames(2, 8)
        got.append(pt.readback())
    _assert_same(got[0][0], got[0][1], got[1][0], got[1][1])


@pytest.mark.parametrize("slots,w,h,spp", [(None, 1920, 1080, 64), (1 << 28, 3840, 2160, 32)])
def test_wavefront_large_pools_equal_megakernel(pt, slots, w, h, spp):
    """The default pool (2^27 slots: the whole 1080p/64 spp bench step in flight, one
    generation) and the largest one (2^28 entries, 28 GB of queues: a 4K/32 spp call) give the
    megakernel's image bit for bit (the megakernel is oracle-checked above)."""
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    lib = hippt.load_library()
    pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, slots if slots else 1 << 27)
    got = []
    for mode in (0, 1):
        pt.setOption(hippt.OPT_PATH_MODE, mode)
        assert pt.initialize(w, h)
        pt.resetStats()
        assert pt.renderFrames(spp, 8, copy=False), pt.lastError()
        got.append((pt.readback(), pt.stats()["segments"]))
    assert lib.hipptGetOption(hippt.OPT_WAVEFRONT_SLOTS) == (slots if slots else 1 << 27)
    (a, sa), (b, sb) = got
    assert sa == sb
    _assert_same(a[0], a[1], b[0], b[1])
    if (w, h, spp) == (1920, 1080, 64):
        # configs[4]'s wavefront image against configs[2]'s oracle golden directly, not only
        # through the megakernel
        import hashlib
        import json
        import zlib
        with open(os.path.join(os.path.dirname(__file__), "golden",
                               "oracle_headline_blob70k_1920x1080_64.json")) as f:
            g = json.load(f)
        assert zlib.crc32(b[0].tobytes()) & 0xFFFFFFFF == g["image_crc32"]
        assert hashlib.sha256(b[1].tobytes()).hexdigest() == g["accum_sha256"]
        assert sb == g["segments"]


def test_wavefront_pools_on_a_shared_device(pt):
    """Three contexts on one device (hipptSetDevices([0, 0, 0])), wavefront mode with the
    default 2^27-slot request: each context's pool is sized to its share of the device's free
    memory (or retried smaller), and the image equals the one-context render."""
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, 1)
    pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, 1 << 27)
    w, h = 960, 540
    assert pt.initialize(w, h)
    assert pt.renderFrames(16, 8)
    one = pt.readback()
    pt.setDevices([0, 0, 0])
    assert pt.initialize(w, h)
    assert pt.renderFrames(16, 8), pt.lastError()
    three = pt.readback()
    _assert_same(one[0], one[1], three[0], three[1])


def _general_scene(name, golden_dir):
    if name == "ref_random_scene":
        return scenes.load_scene_file(os.path.join(golden_dir, "ref_random_scene.scene"), name)
    return scenes.get_scene(name)


@pytest.mark.parametrize("name,w,h,spp,mode", [
    ("random_scene", 64, 36, 4, 0),
    ("random_scene", 48, 27, 3, 1),
    ("ref_random_scene", 64, 36, 4, 0),
    ("cornell_mixed", 64, 64, 4, 0),   # 36 primitives: LDS-resident scene
    ("cornell_mixed", 40, 40, 3, 1),
])
def test_general_scene_matches_oracle(pt, golden_dir, name, w, h, spp, mode):
    """Spheres + Metal/Dielectric (RayTracer.h:289-314, :490-540) through hipptUploadScene, in the
    megakernel (mode 0) and the wavefront kernels (mode 1): bit-identical to the oracle."""
    sc = _general_scene(name, golden_dir)
    pt.uploadScene(sc)
    pt.setOption(hippt.OPT_PATH_MODE, mode)
    pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, 1000)
    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFrames(spp, 8), pt.lastError()
    px, acc = pt.readback()
    ora_px, ora_acc, segs, samples = po.MeshScene(sc, w, h).frames(0, spp, 8)
    _assert_same(px, acc, ora_px, ora_acc)
    st = pt.stats()
    assert st["segments"] == segs and st["pixelSamples"] == samples


def test_general_kernel_equals_lambertian_kernel(pt):
    """cornell34 plus a sphere no ray reaches selects the general kernel; the image is unchanged."""
    base = scenes.cornell34()
    pt.uploadMesh(base)
    assert pt.initialize(72, 40)
    assert pt.renderFrames(4, 8)
    want = pt.readback()
    sc = scenes.cornell34()
    sc.spheres = np.asarray([[5.0e4, 5.0e4, -5.0e4, 1.0]], np.float32)
    sc.sph_mat = np.asarray([0], np.int32)
    pt.uploadScene(sc)
    assert pt.initialize(72, 40)
    assert pt.renderFrames(4, 8)
    got = pt.readback()
    _assert_same(got[0], got[1], want[0], want[1])


def test_present_hand_off_double_buffers(pt):
    """hipptRenderFramesPresent / hipptLatestFrame: non-blocking hand-off of the newest image;
    after a sync the latest frame is the last one presented and equals the accumulation."""
    sc = scenes.cornell34()
    pt.uploadMesh(sc)
    w, h = 64, 48
    assert pt.initialize(w, h)
    assert pt.latestFrame() == (None, 0)
    for _ in range(5):
        assert pt.renderFramesPresent(2, 8), pt.lastError()
        img, n = pt.latestFrame()  # whatever has finished; never waits
        assert img is None or n in (2, 4, 6, 8, 10)
    assert pt.synchronize()
    img, n = pt.latestFrame()
    assert n == 10
    ora_px, _, _, _ = po.MeshScene(sc, w, h).frames(0, 10, 8)
    assert np.array_equal(img, ora_px)
    assert np.array_equal(pt.readback()[0], ora_px)
    st = pt.stats()  # launches harvested without a sync are still accounted
    assert st["traceLaunches"] == 5 and st["combineLaunches"] == 5


def test_mesh_wave_threshold_and_chunk_do_not_change_results(pt):
    sc = scenes.cornell34()
    pt.uploadMesh(sc)
    ref = None
    for thr, chunk in ((0, 64), (16, 256), (63, 4096), (32, 1024)):
        pt.setOption(hippt.OPT_WAVE_THRESHOLD, thr)
        pt.setOption(hippt.OPT_CHUNK, chunk)
        assert pt.initialize(80, 40)
        assert pt.renderFrames(4, 8)
        got = pt.readback()
        if ref is None:
            ref = got
        else:
            _assert_same(got[0], got[1], ref[0], ref[1])


@pytest.mark.parametrize("name,mode", [("blob70k", 0), ("cornell34", 0), ("blob70k", 1)])
def test_loop_exits_do_not_change_results(pt, name, mode):
    """The node and leaf loops' early exits (HIPPT_OPT_LEAF_EXIT / NODE_EXIT) only reorder work:
    identical images, megakernel and wavefront."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, mode)
    ref = None
    for k, n in ((0, 0), (3, 0), (16, 0), (64, 0), (-1, 0), (0, 8), (-1, 16), (16, 64), (-1, -1)):
        pt.setOption(hippt.OPT_LEAF_EXIT, k)
        pt.setOption(hippt.OPT_NODE_EXIT, n)
        assert pt.initialize(56, 40)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        if ref is None:
            ora = po.MeshScene(sc, 56, 40).frames(0, 3, 8)
            _assert_same(got[0], got[1], ora[0], ora[1])
            ref = got
        else:
            _assert_same(got[0], got[1], ref[0], ref[1])


@pytest.mark.parametrize("name", ["blob70k", "cornell34", "random_scene", "cornell_mixed"])
def test_bvh_width_and_stack_spill_do_not_change_results(pt, name):
    """The 4-wide tree (HIPPT_OPT_BVH_WIDTH 4, with the LDS stack capped at 4 entries so deep
    traversals spill to the global spill area and refill; float and 8-bit child boxes) and the
    2-wide tree give the oracle's image bit for bit; the LDS-resident and global-memory scene
    paths alike."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    w, h = (40, 24) if name == "random_scene" else (56, 40)
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    for lds in (1, 0):
        pt.setOption(hippt.OPT_LDS_SCENE, lds)
        for width, cap, quant in ((2, 0, -1), (0, 0, -1), (4, 0, 0), (4, 0, 1), (4, 4, 1), (4, 7, 0), (4, 0, 3),
                                  (4, 4, 3)):
            pt.setOption(hippt.OPT_BVH_WIDTH, width)
            pt.setOption(hippt.OPT_STACK_CAP, cap)
            pt.setOption(hippt.OPT_BVH_QUANT, quant)
            assert pt.initialize(w, h)
            assert pt.renderFrames(3, 8)
            got = pt.readback()
            _assert_same(got[0], got[1], ora[0], ora[1])


@pytest.mark.parametrize("name", ["blob70k", "random_scene", "cornell34"])
def test_lds_top_of_tree_does_not_change_results(pt, name):
    """Trees read from global memory with the top of the tree copied into LDS
    (HIPPT_OPT_LDS_TOP_NODES: none, the root alone, 5 and 85 nodes, the automatic size, which
    covers all of cornell34's 16 nodes), float, 8-bit and hybrid nodes (float top, 8-bit below;
    with no top it falls back to 8-bit nodes), the spilling LDS stack (cap 4) and the default:
    the oracle's image bit for bit.  Counting builds report LDS-served visits exactly when a top
    is in LDS."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    w, h = (40, 24) if name == "random_scene" else (56, 40)
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    # 0 float nodes, 1 8-bit nodes (top too), 2 hybrid: float top in LDS, 8-bit nodes below,
    # 3 half-precision planes (top too)
    quants = (0, 2, 3) if name == "random_scene" else (0, 1, 2, 3)
    for quant in quants:
        for cap in (0, 4):
            for top in (0, 1, 5, 85, -1):
                pt.setOption(hippt.OPT_BVH_QUANT, quant)
                pt.setOption(hippt.OPT_STACK_CAP, cap)
                pt.setOption(hippt.OPT_LDS_TOP_NODES, top)
                assert pt.initialize(w, h)
                pt.setOption(hippt.OPT_COUNT_TRAVERSAL, top in (0, -1))
                pt.resetStats()
                assert pt.renderFrames(3, 8)
                got = pt.readback()
                _assert_same(got[0], got[1], ora[0], ora[1])
                if top in (0, -1):
                    c = pt.counters()
                    top_bytes = pt._lib.hipptGetOption(hippt.INFO_LDS_TOP_BYTES)
                    assert (c["lds_top_visits"] > 0) == (top_bytes > 0), (quant, cap, top, top_bytes)
                    assert c["lds_top_visits"] <= c["nodeVisits"]
                    if top == 0:
                        assert top_bytes == 0
                pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 0)


@pytest.mark.parametrize("name", ["cornell34", "cornell_mixed", "random_scene", "blob70k"])
def test_rng_table_and_sah_collapse_do_not_change_results(pt, name):
    """The memoized random_in_unit_sphere (HIPPT_OPT_RNG_TABLE 1: one lookup per Lambertian or
    Metal scatter instead of the rejection loop) and the loop (the default) give the oracle's
    image bit for bit, megakernel and wavefront; so does the SAH-optimal 4-wide collapse
    (HIPPT_OPT_BVH_COLLAPSE 1, leaves merged up to 8 primitives)."""
    sc = scenes.get_scene(name)
    w, h = (40, 24) if name == "random_scene" else (48, 32)
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    for collapse in (0, 1):
        pt.setOption(hippt.OPT_BVH_COLLAPSE, collapse)
        pt.setOption(hippt.OPT_BVH_LEAF4, 8)
        pt.uploadMesh(sc)
        for mode in (0, 1):
            pt.setOption(hippt.OPT_PATH_MODE, mode)
            for tab in (1, 0):
                pt.setOption(hippt.OPT_RNG_TABLE, tab)
                assert pt.initialize(w, h)
                assert pt.renderFrames(3, 8)
                got = pt.readback()
                _assert_same(got[0], got[1], ora[0], ora[1])


@pytest.mark.parametrize("name,variant", [
    ("cornell34", "pinhole"),       # pool entries without the origin (every ray starts at cam.origin)
    ("cornell34", "zero_origin"),   # a pinhole at an origin with a zero component: origin stored
    ("cornell34", "lens"),          # aperture > 0: origin stored
    ("cornell_mixed", "pinhole"),   # general kernel, LDS scene
    ("random_scene", "lens"),       # general kernel, tree in global memory
    ("blob70k", "pinhole"),         # Lambertian kernel, tree in global memory (+ LDS top)
])
def test_camera_pool_does_not_change_results(pt, name, variant):
    """The megakernel's camera-ray pool (HIPPT_OPT_CAMERA_POOL: each wave generates the camera rays
    of its next 64 samples at once into LDS) gives the oracle's image bit for bit, on and off, at
    sizes whose item count is not a multiple of 64 (a partly filled last pool)."""
    sc = scenes.get_scene(name)
    if variant == "zero_origin":
        sc.lookfrom = (0.0, 278.0, -800.0)
    elif variant == "lens" and name == "cornell34":
        sc.aperture = 25.0
        sc.focus = 800.0
    w, h = (37, 23) if name != "cornell34" else (53, 29)
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    pt.uploadMesh(sc)
    for pool in (1, 0, -1):
        pt.setOption(hippt.OPT_CAMERA_POOL, pool)
        assert pt.initialize(w, h), pt.lastError()
        assert pt.renderFrames(3, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        st = pt.stats()
        assert st["segments"] == ora[2] and st["pixelSamples"] == ora[3]
        pt.resetStats()


@pytest.mark.parametrize("tile", [0, 8, 16, 32])
@pytest.mark.parametrize("name,w,h,frames", [("cornell34", 192, 77, 3), ("blob70k", 131, 64, 2),
                                               ("blob70k", 160, 45, 2), ("cornell_mixed", 96, 53, 2)])
def test_item_order_tiles(pt, name, w, h, frames, tile):
    """HIPPT_OPT_PIXEL_TILE: the item order's runs as tiles of `tile` columns x 64 / tile band rows
    over the band's whole strips, then row runs (item_order.h RunLayout; a width that is not a
    multiple of the tile keeps row runs).  Blocking and chained async batches, the whole image and an
    interleaved row share: the oracle's images and counts."""
    sc = scenes.get_scene(name)
    ora = po.MeshScene(sc, w, h).frames(0, frames, 8)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PIXEL_TILE, tile)
    try:
        assert pt.initialize(w, h), pt.lastError()
        assert pt.renderFrames(frames, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        st = pt.stats()
        assert st["segments"] == ora[2] and st["pixelSamples"] == ora[3]
        assert pt.initialize(w, h)
        for _ in range(frames):
            assert pt.renderFramesAsync(1, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        pt.setRowInterleave(1, 3)
        assert pt.initialize(w, h)
        assert pt.renderFrames(frames, 8)
        got = pt.readback()
        rows = np.arange(1, h, 3)
        _assert_same(got[0][rows], got[1][rows], ora[0][rows], ora[1][rows])
    finally:
        pt.setRowRange(0, 0)
        pt.setOption(hippt.OPT_PIXEL_TILE, -1)


@pytest.mark.parametrize("name,w,h,frames", [("cornell34", 200, 77, 3), ("blob70k", 131, 64, 2),
                                               ("cornell_mixed", 96, 53, 2)])
def test_item_order_does_not_change_results(pt, name, w, h, frames):
    """HIPPT_OPT_ITEM_ORDER: the queues hand out each XCD queue's scene-hitting 64-pixel runs first
    and the sky's last (item_order.cpp); the image and the counts are the oracle's either way, for
    bands whose pixel count is not a multiple of 64 and for interleaved rows."""
    sc = scenes.get_scene(name)
    ora = po.MeshScene(sc, w, h).frames(0, frames, 8)
    pt.uploadMesh(sc)
    for order in (1, 0, -1):
        pt.setOption(hippt.OPT_ITEM_ORDER, order)
        assert pt.initialize(w, h), pt.lastError()
        assert pt.renderFrames(frames, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        st = pt.stats()
        assert st["segments"] == ora[2] and st["pixelSamples"] == ora[3]
        pt.resetStats()
    pt.setOption(hippt.OPT_ITEM_ORDER, 1)
    pt.setRowInterleave(1, 3)
    assert pt.initialize(w, h)
    assert pt.renderFrames(frames, 8)
    got = pt.readback()
    rows = np.arange(1, h, 3)
    _assert_same(got[0][rows], got[1][rows], ora[0][rows], ora[1][rows])
    pt.setRowRange(0, 0)


def test_item_order_camera_change_does_not_stall(pt):
    """in automatic mode (HIPPT_OPT_ITEM_ORDER -1) a camera change does not stall the next
    call on the host's run-cost estimate (0.34 s single-threaded at 1080p): the estimate runs on a
    host thread of its own and the batches queued meanwhile run in image order.  Every call's image
    is the oracle's, before, during and after the switch to the new order; calls with batches of
    different sizes reuse their tables."""
    import ctypes
    import time
    sc = scenes.cornell34()
    w, h = 1920, 1080
    pt.setOption(hippt.OPT_ITEM_ORDER, -1)  # the automatic mode under test (the fixture forces 1)
    pt.uploadMesh(sc)
    assert pt.initialize(w, h), pt.lastError()
    assert pt.renderFrames(1, 8, copy=False), pt.lastError()
    moved = dict(lookfrom=(sc.lookfrom[0] + 40.0, sc.lookfrom[1] + 25.0, sc.lookfrom[2]), lookat=sc.lookat,
                 vup=sc.vup, vfov=sc.vfov, aspect=w / h, aperture=sc.aperture, focus=sc.focus)
    cam = hippt.build_camera(**moved)
    lib = hippt.load_library()
    err = ctypes.c_char_p()
    assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
    t0 = time.perf_counter()
    assert pt.renderFramesAsync(1, 8), pt.lastError()
    assert pt.synchronize()
    first = time.perf_counter() - t0
    assert first < 0.15, f"first call after the camera change took {first:.3f} s"
    # small image: the oracle's frames for the moved camera, through the switch to the new order
    pt.resetAccumulation()
    ws, hs = 160, 90
    sc2 = scenes.cornell34()
    sc2.lookfrom = moved["lookfrom"]
    ora = po.MeshScene(sc2, ws, hs).frames(0, 3, 8)
    pt.uploadMesh(sc2)
    assert pt.initialize(ws, hs), pt.lastError()
    for _ in range(20):  # the first calls in image order, later ones (the estimate done) in cost order
        assert pt.resetAccumulation()
        assert pt.renderFrames(3, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        time.sleep(0.005)


@pytest.mark.parametrize("name", ["cornell34", "blob70k", "random_scene"])
def test_rgba8_pixel_format(pt, name):
    """HIPPT_OPT_PIXEL_FORMAT = RGBA8 (the GL / Vulkan backends' image words): the accumulation is
    unchanged and every word is the oracle's RGBA8 UNORM quantization of it; the reference ABI
    (cudaPathTracerRender) still hands out ARGB words with the option set."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    w, h = (40, 24) if name == "random_scene" else (48, 32)
    ora_px, ora_acc = po.MeshScene(sc, w, h).frames(0, 3, 8)[:2]
    pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_RGBA8)
    try:
        for mode in (0, 1):
            pt.setOption(hippt.OPT_PATH_MODE, mode)
            assert pt.initialize(w, h)
            assert pt.renderFrames(3, 8)
            px, acc = pt.readback()
            assert acc.tobytes() == ora_acc.tobytes()
            assert np.array_equal(px, po.rgba8(ora_acc))
        lib = hippt.load_library()
        assert lib.cudaPathTracerInit(w, h, None)
        for f in range(3):
            assert lib.cudaPathTracerRender(f, 8, None, None)
        px, acc = pt.readback()
        assert np.array_equal(px, ora_px) and acc.tobytes() == ora_acc.tobytes()
    finally:
        pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB)


@pytest.mark.parametrize("mode", [0, 1])
def test_small_stack_cap_on_deep_lds_scene(pt, mode):
    """LDS-resident scene with a deep 4-wide tree (cloud180: stack bound 16) traversed with the
    smallest LDS stack caps (4 and 5: half the cap is below the 3 pushes of a 4-hit visit, so
    the spill must move more than half) and the default: the spill never writes past the lane's
    LDS stack (which would corrupt the block's LDS scene copy); bit-exact against the oracle,
    megakernel and wavefront."""
    sc = scenes.cloud_scene(180)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, mode)
    w, h = 64, 48
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    for cap in (4, 5, 6, 0):
        pt.setOption(hippt.OPT_STACK_CAP, cap)
        assert pt.initialize(w, h)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])


def test_quantized_tree_grid_aligned_geometry(pt):
    """Integer-coordinate cubes (every child-box plane on its node's power-of-two grid) read
    from global memory with 8-bit child boxes (whole tree, and below a float LDS top): bit-exact
    against the oracle, as the float 4-wide and the 2-wide trees."""
    sc = scenes.voxel_scene(6)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    w, h = 64, 48
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    for width, quant in ((4, 1), (4, 2), (4, 0), (2, -1)):
        pt.setOption(hippt.OPT_BVH_WIDTH, width)
        pt.setOption(hippt.OPT_BVH_QUANT, quant)
        assert pt.initialize(w, h)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])


def test_mesh_batches_and_frame_splits_are_bit_identical(pt):
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    assert pt.initialize(48, 40)
    assert pt.renderFrames(6, 8)
    one = pt.readback()
    pt.setOption(hippt.OPT_SCRATCH_MB, 1)  # forces several scratch batches per call
    assert pt.initialize(48, 40)
    for n in (1, 2, 3):
        assert pt.renderFrames(n, 8)
    split = pt.readback()
    _assert_same(one[0], one[1], split[0], split[1])


@pytest.mark.parametrize("order", [0, 1, -1])
@pytest.mark.parametrize("name", ["cornell34", "blob70k", "random_scene", "cornell_mixed"])
def test_chained_batches_match_oracle(pt, name, order):
    """HIPPT_OPT_CHAIN (Ctx::chain, hippt_trace.h chained batches): a launch whose batch is drained
    goes on with the asynchronous batches posted behind it, the next launch combines them beside its
    own paths, and the image's readers flush the rest.  At caps 1, 2 and 8, off and automatic, the
    images are the oracle's: progressive batches (frames 0-1, 2-3, 4-5), batches that render the
    same frames again (bench.py's steps: each batch's frame 0 restarts the average) more often than
    the ring has slots, batches of different sizes (each size change a new run), a reset inside a
    run; the pixel-sample count is exact (the chained kernels do not count samples, the host does).
    random_scene is the general kernel over a tree in global memory, which has no camera pool and
    never chains: its sequences run unchained under every setting."""
    sc = scenes.get_scene(name)
    w, h = 45, 26
    ora6 = po.MeshScene(sc, w, h).frames(0, 6, 8)
    ora2 = po.MeshScene(sc, w, h).frames(0, 2, 8)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_ITEM_ORDER, order)
    lib = hippt.load_library()
    for chain in (1, 2, 8, 0, -1):
        pt.setOption(hippt.OPT_CHAIN, chain)
        assert pt.initialize(w, h)
        pt.resetStats()
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora6[0], ora6[1])
        assert pt.stats()["pixelSamples"] == w * h * 6
        assert pt.initialize(w, h)
        for _ in range(37):  # more batches than the ring's slots, and the launches' caps
            assert lib.hipptRenderFramesAsync(0, 2, 8, None)
        got = pt.readback()
        _assert_same(got[0], got[1], ora2[0], ora2[1])
        assert pt.initialize(w, h)
        assert pt.renderFramesAsync(1, 8) and pt.renderFramesAsync(2, 8) and pt.renderFramesAsync(2, 8)
        assert pt.renderFramesAsync(1, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora6[0], ora6[1])
        assert pt.initialize(w, h)
        assert pt.renderFramesAsync(2, 8) and pt.renderFramesAsync(2, 8) and pt.resetAccumulation()
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8)
        got = pt.readback()  # (the reset restarts the frame index: frames 0..5 again)
        _assert_same(got[0], got[1], ora6[0], ora6[1])


def test_chained_batches_camera_change_and_row_shares(pt):
    """A camera change between queued batches starts a new run (the old run's launches must not take
    the new camera's batches; its combines are flushed first): the image equals one launch per batch.
    Every 1/4 row share (hipptSetRowInterleave, bench.py's split) with chained steps renders its rows
    of the unchained image."""
    import ctypes
    sc = scenes.cornell34()
    w, h = 96, 54
    lib = hippt.load_library()
    moved = dict(lookfrom=(sc.lookfrom[0] + 40.0, sc.lookfrom[1] + 25.0, sc.lookfrom[2]), lookat=sc.lookat,
                 vup=sc.vup, vfov=sc.vfov, aspect=w / h, aperture=sc.aperture, focus=sc.focus)
    err = ctypes.c_char_p()
    images = {}
    for chain in (0, 8):
        pt.setOption(hippt.OPT_CHAIN, chain)
        pt.uploadMesh(sc)
        assert pt.initialize(w, h)
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8)
        cam = hippt.build_camera(**moved)
        assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
        for _ in range(3):
            assert pt.renderFramesAsync(2, 8)
        images[chain] = pt.readback()
    _assert_same(images[8][0], images[8][1], images[0][0], images[0][1])
    pt.setOption(hippt.OPT_CHAIN, 0)
    pt.uploadMesh(sc)
    assert pt.initialize(w, h)
    for _ in range(4):
        assert lib.hipptRenderFramesAsync(0, 4, 8, None)
    full = pt.readback()
    pt.setOption(hippt.OPT_CHAIN, 8)
    for r in range(4):
        pt.setRowInterleave(r, 4)
        assert pt.initialize(w, h)
        for _ in range(11):
            assert lib.hipptRenderFramesAsync(0, 4, 8, None)
        share = pt.readback()
        rows = np.arange(r, h, 4)
        _assert_same(share[0][rows], share[1][rows], full[0][rows], full[1][rows])
    pt.setRowRange(0, 0)


def test_automatic_chain_and_claim_size(pt):
    """HIPPT_OPT_CHAIN -1 and HIPPT_OPT_CHUNK 0 (the defaults) as applied (HIPPT_INFO_CHAIN_CAP,
    HIPPT_INFO_CHUNK): a whole 1080p/64 spp image chains 8 batches (round 6; Cornell ran unchained and
    blob70k / cornell_mixed chained 3 before), Cornell and blob70k with 512-item claims, cornell_mixed
    (the general kernel) with 256; Cornell's 1/8 row share chains 8, blob70k's 16 (the automatic cap's
    ceiling for trees in global memory)."""
    lib = hippt.load_library()
    pt.setOption(hippt.OPT_CHAIN, -1)
    pt.setOption(hippt.OPT_CHUNK, 0)
    for name, stride, cap, chunk in (("cornell34", 1, 8, 512), ("cornell34", 8, 8, 512), ("blob70k", 1, 8, 512),
                                     ("blob70k", 8, 16, 512),
                                     ("cornell_mixed", 1, 8, 256)):
        pt.uploadMesh(scenes.get_scene(name))
        pt.setRowInterleave(0, stride)
        assert pt.initialize(1920, 1080)
        assert lib.hipptRenderFramesAsync(0, 64, 8, None)
        assert pt.synchronize()
        assert lib.hipptGetOption(hippt.INFO_CHAIN_CAP) == cap, name
        assert lib.hipptGetOption(hippt.INFO_CHUNK) == chunk, name
    pt.setRowRange(0, 0)


def test_chained_batches_with_skipped_launches(pt):
    """chain_batch holds the batches that arrive while the run's last launch has not started and
    launches them together as one group (MeshParams::chainGroup: one set of queues over the group's
    items, 64-item runs of its batches interleaved); a run that closes with held batches (a camera
    change, a readback) launches them first.  Batches long enough (256 frames of 96x54) that each
    launch is still queued behind the running one when the next batches arrive: the images equal one
    launch per batch, before and after a camera change, at caps 8 and 3, and the sample count is
    exact."""
    import ctypes
    sc = scenes.cornell34()
    w, h = 96, 54
    lib = hippt.load_library()
    moved = dict(lookfrom=(sc.lookfrom[0] - 30.0, sc.lookfrom[1] + 20.0, sc.lookfrom[2]), lookat=sc.lookat,
                 vup=sc.vup, vfov=sc.vfov, aspect=w / h, aperture=sc.aperture, focus=sc.focus)
    err = ctypes.c_char_p()
    images = {}
    for chain in (0, 8, 3):
        pt.setOption(hippt.OPT_CHAIN, chain)
        pt.uploadMesh(sc)
        assert pt.initialize(w, h)
        pt.resetStats()
        for _ in range(11):  # progressive batches: frames 0..2815
            assert pt.renderFramesAsync(256, 8), pt.lastError()
        cam = hippt.build_camera(**moved)
        assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
        for _ in range(5):  # the same frames again: every batch restarts the average
            assert lib.hipptRenderFramesAsync(0, 256, 8, None)
        images[chain] = pt.readback()
        assert pt.stats()["pixelSamples"] == w * h * 256 * 16
    for chain in (8, 3):
        _assert_same(images[chain][0], images[chain][1], images[0][0], images[0][1])


def _moved_camera(sc, w, h, dx=40.0, dy=25.0):
    return hippt.build_camera(lookfrom=(sc.lookfrom[0] + dx, sc.lookfrom[1] + dy, sc.lookfrom[2]), lookat=sc.lookat,
                              vup=sc.vup, vfov=sc.vfov, aspect=w / h, aperture=sc.aperture, focus=sc.focus)


def _audited_runs(min_batches=2):
    runs = hippt.chain_audit()
    problems = chain_audit.check(runs)
    assert not problems, problems[:6]
    return [r for r in runs if r[0]["batches"] >= min_batches]


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("name", ["blob70k", "cornell34"])
def test_run_closes_while_a_launch_runs(pt, name, order):
    """a run that closes while its launch still runs.  Four long progressive
    batches (256x144 x 512 frames: the first launch runs for milliseconds and takes the posted batches
    behind it, the later ones are held), then a camera change (a new run: the host's mailbox moves on
    while the old run's waves are still inside their batches, some holding claimed items), a burst of
    small batches of the new camera, and the readback's flush.  The image and accumulation equal one
    launch per batch (HIPPT_OPT_CHAIN 0) bit for bit, two rows equal the oracle's continuation across
    the camera change, and the audit finds every batch of both runs traced once with its own frames
    and combined once, in order."""
    import ctypes
    sc = scenes.get_scene(name)
    w, h = 256, 144
    lib = hippt.load_library()
    err = ctypes.c_char_p()
    pt.setOption(hippt.OPT_ITEM_ORDER, order)
    cam = _moved_camera(sc, w, h)
    images = {}
    for chain in (-1, 0):
        pt.setOption(hippt.OPT_CHAIN, chain)
        pt.uploadMesh(sc)
        assert pt.initialize(w, h), pt.lastError()
        pt.resetStats()
        for _ in range(4):
            assert pt.renderFramesAsync(512, 8), pt.lastError()
        assert lib.hipptSetCamera(ctypes.byref(cam), ctypes.byref(err)), err.value
        for _ in range(6):
            assert pt.renderFramesAsync(4, 8), pt.lastError()
        images[chain] = pt.readback()
        assert pt.stats()["pixelSamples"] == w * h * (4 * 512 + 6 * 4)
        if chain == -1:
            runs = _audited_runs()
            assert any(r[0]["batches"] == 4 and r[0]["totalItems"] == w * h * 512 for r in runs), \
                [r[0] for r in runs]
    _assert_same(images[-1][0], images[-1][1], images[0][0], images[0][1])
    ms = po.MeshScene(sc, w, h)
    ys = (57, 58)
    a = ms.frames(0, 4 * 512, 8, y0=ys[0], y1=ys[1] + 1)
    moved = po.MeshScene(sc, w, h, cam=po.PoCamera.from_buffer_copy(bytes(cam)))
    b = moved.frames(4 * 512, 6 * 4, 8, y0=ys[0], y1=ys[1] + 1, accum=a[1])
    _assert_same(images[-1][0][ys[0]:ys[1] + 1], images[-1][1][ys[0]:ys[1] + 1], b[0], b[1])


@pytest.mark.parametrize("event", ["upload", "pixel_format", "blocks_per_cu", "readback"])
def test_held_group_closed_by_event(pt, event):
    """a run whose batches are held (arrived while the run's last launch had not started)
    and is then closed by a scene upload (its buffers freed and replaced: the held group launches
    first, ensure_scene), a pixel-format change, a grid change or a readback.  The image equals one
    launch per batch and the audit is clean."""
    sc, other = scenes.blob70k(), scenes.cornell34()
    w, h = 192, 108
    images = {}
    for chain in (-1, 0):
        pt.setOption(hippt.OPT_CHAIN, chain)
        pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB)
        pt.setOption(hippt.OPT_BLOCKS_PER_CU, 0)
        pt.uploadMesh(sc)
        assert pt.initialize(w, h), pt.lastError()
        for _ in range(5):  # the first launch runs while the next batches arrive: held
            assert pt.renderFramesAsync(256, 8), pt.lastError()
        if event == "upload":
            pt.uploadMesh(other)
        elif event == "pixel_format":
            pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_RGBA8)
        elif event == "blocks_per_cu":
            pt.setOption(hippt.OPT_BLOCKS_PER_CU, 2)
        else:
            images[(chain, "mid")] = pt.readback()
        for _ in range(3):
            assert pt.renderFramesAsync(256, 8), pt.lastError()
        images[chain] = pt.readback()
        if chain == -1:
            assert _audited_runs(), "no chained run"
    pt.setOption(hippt.OPT_PIXEL_FORMAT, hippt.PIXEL_ARGB)
    pt.setOption(hippt.OPT_BLOCKS_PER_CU, 0)
    _assert_same(images[-1][0], images[-1][1], images[0][0], images[0][1])
    if event == "readback":
        _assert_same(images[(-1, "mid")][0], images[(-1, "mid")][1], images[(0, "mid")][0], images[(0, "mid")][1])


def test_chain_ring_within_scratch_budget(pt):
    """the chain ring (slots x 2^shift samples x 12 B) stays within HIPPT_OPT_SCRATCH_MB: a
    budget under two slots runs the batches unchained (HIPPT_INFO_CHAIN_CAP 0), a budget of two slots
    chains with cap 1, a larger one with the automatic cap; the images are the oracle's."""
    sc = scenes.cornell34()
    w, h = 640, 360  # one frame per batch: 230400 items, 2^18-sample slots of 3 MiB
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    pt.uploadMesh(sc)
    lib = hippt.load_library()
    for mb, cap in ((4, 0), (8, 1), (64, 8)):
        pt.setOption(hippt.OPT_SCRATCH_MB, mb)
        assert pt.initialize(w, h), pt.lastError()
        for _ in range(3):
            assert pt.renderFramesAsync(1, 8), pt.lastError()
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        assert lib.hipptGetOption(hippt.INFO_CHAIN_CAP) == cap, mb
    pt.setOption(hippt.OPT_SCRATCH_MB, 32768)


@pytest.mark.parametrize("order", [0, 1, -1])
@pytest.mark.parametrize("name", ["cornell34", "blob70k", "random_scene"])
def test_deferred_combine_across_async_calls(pt, name, order):
    """Back-to-back hipptRenderFramesAsync calls: each megakernel batch's combine (running average
    + tonemap) runs inside the next batch's launch (Ctx::deferred), from the other scratch buffer;
    anything that reads or resets the image runs the pending one first.  Every sequence below
    gives the oracle's progressive image bit for bit.  Item order 0 and 1 fix the code path; -1
    (the library's default) lets the detached cost job finish at any point of a sequence, closing
    the chained run it lands in (GPUTEST_r05's trigger) — exact and audited all the same."""
    sc = scenes.get_scene(name)
    w, h = 45, 26
    ora6 = po.MeshScene(sc, w, h).frames(0, 6, 8)
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_ITEM_ORDER, order)
    # fused off: every batch's combine its own launch
    pt.setOption(hippt.OPT_FUSE_COMBINE, 0)
    assert pt.initialize(w, h)
    for _ in range(6):
        assert pt.renderFramesAsync(1, 8), pt.lastError()
    got = pt.readback()
    _assert_same(got[0], got[1], ora6[0], ora6[1])
    pt.setOption(hippt.OPT_FUSE_COMBINE, -1)
    # one frame per call: a chain of five deferred combines, the last one run by readback's sync
    assert pt.initialize(w, h)
    for _ in range(6):
        assert pt.renderFramesAsync(1, 8), pt.lastError()
    got = pt.readback()
    _assert_same(got[0], got[1], ora6[0], ora6[1])
    # several batches per call (tiny scratch cap): deferred within the call as well
    pt.setOption(hippt.OPT_SCRATCH_MB, 1)
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(4, 8) and pt.renderFramesAsync(2, 8)
    got = pt.readback()
    _assert_same(got[0], got[1], ora6[0], ora6[1])
    pt.setOption(hippt.OPT_SCRATCH_MB, 32768)
    # a reset between async calls runs the pending combine first, then clears the accumulation
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(3, 8)
    assert pt.resetAccumulation()
    for _ in range(6):
        assert pt.renderFramesAsync(1, 8)
    got = pt.readback()
    _assert_same(got[0], got[1], ora6[0], ora6[1])
    # a wavefront batch after megakernel batches flushes their combine before its own
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(2, 8)
    pt.setOption(hippt.OPT_PATH_MODE, 1)
    assert pt.renderFramesAsync(2, 8)
    pt.setOption(hippt.OPT_PATH_MODE, 0)
    assert pt.renderFramesAsync(2, 8)
    got = pt.readback()
    _assert_same(got[0], got[1], ora6[0], ora6[1])
    # the present hand-off and a blocking render see finished images
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(3, 8)
    assert pt.renderFramesPresent(3, 8)
    assert pt.synchronize()
    img, frames = pt.latestFrame()
    assert frames == 6 and np.array_equal(img, ora6[0])
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(5, 8) and pt.renderFrames(1, 8)
    assert np.array_equal(pt.hostPixels(), ora6[0])


@pytest.mark.parametrize("call", ["async", "legacy_abi"])
def test_mesh_to_sphere_switch_flushes_deferred_combine(pt, call):
    """An async mesh batch leaves its combine pending (Ctx::deferred); a switch to the built-in
    4-sphere scene followed by a render from frame 0 must run that combine before the legacy
    kernel overwrites the accumulation, so the image equals a fresh sphere render (the
    sphere branch did not flush and blended mesh radiance into the sphere image)."""
    w, h = 40, 23
    ora = po.sphere4(w, h, 0, 2, 8)
    pt.uploadMesh(scenes.cornell34())
    assert pt.initialize(w, h)
    assert pt.renderFramesAsync(3, 8), pt.lastError()
    pt.useBuiltinScene(hippt.SCENE_SPHERE4)
    lib = hippt.load_library()
    for f in range(2):
        if call == "async":
            assert lib.hipptRenderFramesAsync(f, 1, 8, None)
        else:
            assert lib.cudaPathTracerRender(f, 8, None, None)
    got = pt.readback()
    _assert_same(got[0], got[1], ora[0], ora[1])


def test_mesh_row_range_and_two_contexts(pt):
    sc = scenes.cornell34()
    pt.uploadMesh(sc)
    w, h = 64, 40
    assert pt.initialize(w, h)
    assert pt.renderFrames(3, 8)
    full = pt.readback()
    # one process owning rows [13, 29) of the image
    pt.setRowRange(13, 29)
    assert pt.initialize(w, h)
    assert pt.renderFrames(3, 8)
    band = pt.readback(13, 29)
    _assert_same(band[0], band[1], full[0][13:29], full[1][13:29])
    # two contexts (row bands) on the same device: the multi-GPU host gather path
    pt.setRowRange(0, 0)
    pt.setDevices([0, 0])
    assert pt.initialize(w, h)
    assert pt.renderFrames(3, 8)
    assert pt.stats()["numDevices"] == 2
    two = pt.readback()
    _assert_same(two[0], two[1], full[0], full[1])
    assert np.array_equal(pt.hostPixels(), full[0])


@pytest.mark.parametrize("device_rows", [0, 1])
def test_row_interleave_and_device_split(pt, device_rows):
    """Interleaved rows (one process per GPU: rank r renders rows r, r+N, ...) and both in-process
    device splits give the single-context image bit for bit."""
    sc = scenes.cornell34()
    pt.uploadMesh(sc)
    w, h = 48, 37
    assert pt.initialize(w, h)
    assert pt.renderFrames(3, 8)
    full = pt.readback()
    for phase, stride in ((0, 3), (2, 3), (1, 8)):
        pt.setRowInterleave(phase, stride)
        assert pt.initialize(w, h)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        rows = np.arange(phase, h, stride)
        _assert_same(got[0][rows], got[1][rows], full[0][rows], full[1][rows])
        other = np.setdiff1d(np.arange(h), rows)
        assert not got[0][other].any()
    pt.setRowRange(0, 0)
    pt.setOption(hippt.OPT_DEVICE_ROWS, device_rows)
    pt.setDevices([0, 0, 0])
    assert pt.initialize(w, h)
    assert pt.renderFrames(3, 8)
    three = pt.readback()
    _assert_same(three[0], three[1], full[0], full[1])
    assert np.array_equal(pt.hostPixels(), full[0])
    pt.setOption(hippt.OPT_DEVICE_ROWS, 1)


def test_legacy_scene_row_interleave(pt):
    assert pt.initialize(40, 23)
    assert pt.renderFrames(2, 6)
    full = pt.readback()
    pt.setRowInterleave(1, 4)
    assert pt.initialize(40, 23)
    assert pt.renderFrames(2, 6)
    got = pt.readback()
    _assert_same(got[0][1::4], got[1][1::4], full[0][1::4], full[1][1::4])


def test_single_triangle_and_degenerate_sizes(pt):
    v = np.array([[200, 100, 300, 400, 100, 300, 300, 400, 300]], np.float32)
    sc = scenes.Scene("one", v, np.zeros(1, np.int32), np.array([[0.5, 0.6, 0.7]], np.float32))
    pt.uploadMesh(sc)
    for w, h in ((1, 1), (5, 1), (1, 7), (31, 29)):
        assert pt.initialize(w, h)
        assert pt.renderFrames(2, 3)
        px, acc = pt.readback()
        ora = po.MeshScene(sc, w, h).frames(0, 2, 3)
        _assert_same(px, acc, ora[0], ora[1])


def test_mesh_depth_zero_is_black(pt):
    pt.uploadMesh(scenes.cornell34())
    assert pt.initialize(16, 8)
    assert pt.renderFrames(2, 0)
    px, acc = pt.readback()
    assert np.all(px == 0xFF000000) and np.all(acc[..., :3] == 0) and pt.stats()["segments"] == 0


@pytest.mark.parametrize("name,w,h,spp", [("cornell34", 1920, 1080, 8), ("blob70k", 1920, 1080, 4),
                                           ("blob70k", 3840, 2160, 2)])
def test_full_size_1080p_rows_and_determinism(pt, name, w, h, spp):
    """BASELINE config 2/3/4 sizes (LDS 4-wide tree; global 8-bit 4-wide tree): bit-exact on
    sampled rows, deterministic, counts consistent."""
    sc = scenes.get_scene(name)
    pt.uploadMesh(sc)
    assert pt.initialize(w, h)
    assert pt.renderFrames(spp, 8)
    a = pt.readback()
    st = pt.stats()
    assert st["pixelSamples"] == w * h * spp
    assert st["pixelSamples"] < st["segments"] < 8 * st["pixelSamples"]
    assert pt.initialize(w, h)
    assert pt.renderFrames(spp, 8)
    b = pt.readback()
    _assert_same(a[0], a[1], b[0], b[1])
    ms = po.MeshScene(sc, w, h, accel=1)
    for y0 in (0, h // 2 - 3, h - 2):
        ora = ms.frames(0, spp, 8, y0=y0, y1=y0 + 2)
        _assert_same(a[0][y0:y0 + 2], a[1][y0:y0 + 2], ora[0], ora[1])


@pytest.mark.parametrize("mode", [0, 1], ids=["megakernel", "wavefront"])
def test_counting_mode_reports_traversal(pt, mode):
    sc = scenes.blob70k()
    pt.uploadMesh(sc)
    pt.setOption(hippt.OPT_PATH_MODE, mode)
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 1)
    assert pt.initialize(64, 32)
    assert pt.renderFrames(2, 8)
    st = pt.stats()
    counted = pt.readback()
    assert st["nodeVisits"] > st["segments"] > 0 and st["triTests"] > 0
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 0)
    assert pt.initialize(64, 32)
    assert pt.renderFrames(2, 8)
    plain = pt.readback()
    _assert_same(counted[0], counted[1], plain[0], plain[1])


@pytest.mark.parametrize("offset", [(0.0, 0.0, 0.0), (2.5e4, -1.0e4, 3.0e4)])
def test_quantized_tree_far_from_origin(pt, offset):
    """The 8-bit 4-wide tree read from global memory (LDS scene copy off) stays conservative
    when the scene and camera sit far from the origin (large |o| in t = q*s*inv + o*inv - o_ray*inv,
    boxes padded relative to the largest coordinate): bit-exact against the oracle, float
    nodes and 2-wide tree alike."""
    import dataclasses
    base = scenes.blob_scene(64, 34, "blob_small")
    off = np.asarray(offset, np.float32)
    sc = dataclasses.replace(base, verts=(base.verts.reshape(-1, 3, 3) + off).reshape(-1, 9).astype(np.float32),
                             lookfrom=tuple(np.asarray(base.lookfrom, np.float32) + off),
                             lookat=tuple(np.asarray(base.lookat, np.float32) + off))
    pt.uploadMesh(sc)
    w, h = 48, 32
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    for width, quant in ((4, 1), (4, 2), (4, 3), (4, 0), (2, -1)):
        pt.setOption(hippt.OPT_BVH_WIDTH, width)
        pt.setOption(hippt.OPT_BVH_QUANT, quant)
        assert pt.initialize(w, h)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])


def test_half_tree_beyond_half_range_keeps_float_nodes(pt):
    """a scene whose planes leave the half range (|x| > 65504) has no half-precision tree:
    HIPPT_OPT_BVH_QUANT 3 then renders with float nodes (not with boxes widened to infinity, which
    every ray enters), bit-exact against the oracle and as fast as the float tree."""
    import dataclasses
    base = scenes.blob_scene(64, 34, "blob_small")
    off = np.asarray((9.0e4, 0.0, -7.0e4), np.float32)
    sc = dataclasses.replace(base, verts=(base.verts.reshape(-1, 3, 3) + off).reshape(-1, 9).astype(np.float32),
                             lookfrom=tuple(np.asarray(base.lookfrom, np.float32) + off),
                             lookat=tuple(np.asarray(base.lookat, np.float32) + off))
    pt.uploadMesh(sc)
    w, h = 48, 32
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    pt.setOption(hippt.OPT_BVH_WIDTH, 4)
    visits = {}
    for quant in (3, 0):
        pt.setOption(hippt.OPT_BVH_QUANT, quant)
        pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 1)
        assert pt.initialize(w, h)
        pt.resetStats()
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])
        visits[quant] = pt.stats()["nodeVisits"]
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 0)
    assert visits[3] == visits[0]  # the same (float) tree traversed


def test_quantized_tree_tiny_far_nodes(pt):
    """tiny nodes far from the ray origin on the 8-bit path.  A cluster of 400
    triangles of size ~1e-3 (nodes whose extent is ~1e-6 of their distance from the camera) in
    front of a large backdrop, so that the scene's largest coordinate (and with it the global box
    pad M * 2^-16) is set by the backdrop: the decoded 8-bit planes stay outside the float planes
    and no grazing hit is culled (bit-exact against the oracle, 8-bit, float and 2-wide trees)."""
    rng = np.random.default_rng(11)
    n = 400
    centre = np.array([1.0, 2.0, -1500.0]) + rng.normal(scale=0.02, size=(n, 1, 3))
    tiny = (centre + 1e-3 * rng.normal(size=(n, 3, 3))).reshape(n, 9)
    back = np.array([[-3000, -3000, -3000, 3000, -3000, -3000, 0, 3000, -3000]], np.float64)
    verts = np.concatenate([tiny, back]).astype(np.float32)
    sc = scenes.Scene("tiny_far", verts, (np.arange(n + 1) % 2).astype(np.int32),
                      np.array([[0.8, 0.7, 0.6], [0.3, 0.5, 0.9]], np.float32),
                      lookfrom=(1.0, 2.0, 0.0), lookat=(1.0, 2.0, -1500.0), vfov=0.003)
    pt.uploadMesh(sc)
    w, h = 48, 32
    ora = po.MeshScene(sc, w, h).frames(0, 3, 8)
    assert 0 < np.count_nonzero(ora[0] != ora[0][0, 0])  # the cluster is in the picture
    pt.setOption(hippt.OPT_LDS_SCENE, 0)
    for width, quant in ((4, 1), (4, 2), (4, 3), (4, 0), (2, -1)):
        pt.setOption(hippt.OPT_BVH_WIDTH, width)
        pt.setOption(hippt.OPT_BVH_QUANT, quant)
        assert pt.initialize(w, h)
        assert pt.renderFrames(3, 8)
        got = pt.readback()
        _assert_same(got[0], got[1], ora[0], ora[1])


def test_bench_json_contract():
    """bench.py prints one JSON line with the driver's keys, the roofline and the CPU baseline
    objects (a short run: 1 step, sampled CPU baseline)."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "1", "--warmup", "0",
                          "--width", "320", "--height", "180", "--cpu-seconds", "1", "--cpu-baseline", "port"],
                         capture_output=True, text=True, timeout=300, cwd=repo)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["value"] > 0 and d["n_gpus"] == 1 and d["steps"] == 1
    r = d["roofline"]
    assert r["bound"] == "valu" and r["unit"] == "TFLOP/s" and r["achieved"] > 0 and r["peak"] == 157.3
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # per step (a chained launch may trace several steps, another none): kernel time, FLOP and bytes
    assert r["algorithmic_bytes"]["per_step"] > 0 and r["kernel_ms_per_step"] > 0 and r["launches_per_step"] > 0
    assert d["config"]["chunk"]["applied"] in (256, 512) and "applied_cap" in d["config"]["chain"]
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["unit"] == "Msamples/s"
