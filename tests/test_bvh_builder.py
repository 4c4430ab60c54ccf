"""Invariants of the host SAH BVH builder (replaces BVHNode, RayTracer.h:393-429) and
result-equivalence of BVH traversal with brute force (the oracle's private BVH)."""
import os
import numpy as np
import pytest

import hippt
import pyoracle as po
from hippt import scenes


def _decode(nodes):
    boxes = nodes[:, :12].view(np.float32).reshape(-1, 2, 2, 3)  # node, child, lo/hi, xyz
    kids = nodes[:, 12:14].view(np.int32)
    return boxes, kids


def _walk(nodes):
    boxes, kids = _decode(nodes)
    leaves, depth = [], 0
    stack = [(0, 1)]
    while stack:
        n, d = stack.pop()
        depth = max(depth, d)
        for c in range(2):
            k = int(kids[n, c])
            if k >= 0:
                stack.append((k, d + 1))
            else:
                code = ~k
                leaves.append((code >> 4, code & 15, n, c))
    return leaves, depth


@pytest.fixture(params=[1, 0], ids=["sweep-sah", "binned-sah"])
def sah_mode(request):
    lib = hippt.load_library()
    assert lib.hipptSetOption(hippt.OPT_BVH_SAH, request.param)
    yield request.param
    lib.hipptSetOption(hippt.OPT_BVH_SAH, 1)


@pytest.mark.parametrize("name", ["cornell34", "blob70k"])
def test_bvh_covers_every_triangle_once_and_bounds_children(name, sah_mode):
    sc = scenes.get_scene(name)
    bvh = hippt.Bvh(sc.verts, extent_hint=800.0)
    assert sorted(bvh.order.tolist()) == list(range(sc.num_tris))
    leaves, depth = _walk(bvh.nodes)
    assert depth == bvh.depth <= 32  # kernel LDS stack depth
    covered = np.zeros(sc.num_tris, np.int32)
    boxes, kids = _decode(bvh.nodes)
    for first, count, n, c in leaves:
        assert count <= 4
        covered[first:first + count] += 1
        lo, hi = boxes[n, c]
        v = sc.verts[bvh.order[first:first + count]].reshape(-1, 3)
        if count:
            assert np.all(v >= lo) and np.all(v <= hi)  # padded box contains its triangles
    assert np.all(covered == 1)
    # interior child boxes contain their children's boxes (surrounding_box, RayTracer.h:251-265)
    for n in range(len(bvh.nodes)):
        for c in range(2):
            k = int(kids[n, c])
            if k >= 0:
                lo, hi = boxes[n, c]
                assert np.all(boxes[k, :, 0] >= lo - 1e-3) and np.all(boxes[k, :, 1] <= hi + 1e-3)


def test_single_triangle_scene_root_leaf():
    v = np.array([[0, 0, -1, 1, 0, -1, 0, 1, -1]], np.float32)
    bvh = hippt.Bvh(v)
    leaves, depth = _walk(bvh.nodes)
    assert len(bvh.nodes) == 1 and depth == 1
    assert sorted((f, c) for f, c, _, _ in leaves) == [(0, 0), (0, 1)]


def test_deep_degenerate_input_respects_stack_bound():
    # 20k coincident-centroid slivers plus a geometric progression that defeats SAH balance
    rng = np.random.default_rng(1)
    n = 20000
    x = np.cumsum(rng.exponential(size=n) ** 4).astype(np.float32)
    v = np.zeros((n, 9), np.float32)
    v[:, 0] = x
    v[:, 3] = x + 1e-3
    v[:, 7] = 1.0
    bvh = hippt.Bvh(v)
    assert bvh.depth <= 32
    assert sorted(bvh.order.tolist()) == list(range(n))


def test_empty_scene_rejected():
    with pytest.raises(hippt.HipptError):
        hippt.Bvh(np.zeros((0, 9), np.float32))


@pytest.mark.parametrize("name,w,h", [("cornell34", 48, 32), ("blob70k", 24, 16)])
def test_bvh_traversal_equals_brute_force(name, w, h):
    sc = scenes.get_scene(name)
    brute = po.MeshScene(sc, w, h, accel=0)
    bvh = po.MeshScene(sc, w, h, accel=1)
    a = brute.frames(0, 2, 8)
    b = bvh.frames(0, 2, 8)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]


def _decode4(nodes4):
    f = nodes4[:, :24].view(np.float32).reshape(-1, 3, 2, 4)  # node, axis, lo/hi, slot
    kids = nodes4[:, 24:28].view(np.int32)
    return f, kids


@pytest.mark.parametrize("name", ["cornell34", "blob70k", "random_scene"])
def test_bvh4_collapse_keeps_leaves_and_bounds_subtrees(name):
    """The 4-wide tree (hipptBvh4*) holds exactly the 2-wide tree's leaves, every child box
    contains its subtree's primitives, and the stack bound is the max over nodes of the
    (children - 1) pushes along the path."""
    sc = scenes.get_scene(name)
    if sc.num_tris == 0:
        pytest.skip("sphere-only scene: triangles are the collapse's test subject")
    bvh = hippt.Bvh(sc.verts, extent_hint=800.0)
    leaves2 = sorted(tuple(x[:2]) for x in _walk(bvh.nodes)[0])
    f, kids = _decode4(bvh.nodes4)
    assert kids.shape[0] >= 1 and bvh.depth4 <= bvh.depth
    leaves4, bound, depth = [], 0, 0
    stack = [(0, 0, 1)]
    seen = np.zeros(len(kids), bool)
    while stack:
        n, pushes, d = stack.pop()
        assert not seen[n]
        seen[n] = True
        depth = max(depth, d)
        used = [c for c in range(4) if not (kids[n, c] == -1 and f[n, 0, 0, c] > 1e37)]
        assert 2 <= len(used) <= 4
        bound = max(bound, pushes + len(used) - 1)
        for c in range(4):
            k = int(kids[n, c])
            lo, hi = f[n, :, 0, c], f[n, :, 1, c]
            if c not in used:  # unused slot: empty leaf under a point far outside the scene
                assert k == -1 and np.all(lo == hi) and abs(lo[0]) > 1e37
                continue
            if k >= 0:
                # a child node's boxes lie inside this box (the 2-wide boxes it was made of)
                cu = [cc for cc in range(4) if not (kids[k, cc] == -1 and f[k, 0, 0, cc] > 1e37)]
                assert np.all(f[k, :, 0, cu].T >= lo[:, None] - 1e-3) and np.all(f[k, :, 1, cu].T <= hi[:, None] + 1e-3)
                stack.append((k, pushes + len(used) - 1, d + 1))
            else:
                code = ~k
                first, count = code >> 4, code & 15
                leaves4.append((first, count))
                v = sc.verts[bvh.order[first:first + count]].reshape(-1, 3)
                assert np.all(v >= lo) and np.all(v <= hi)
    assert seen.all()
    assert sorted(leaves4) == leaves2
    assert bound == bvh.stack_bound4 and depth == bvh.depth4


@pytest.mark.parametrize("name", ["cornell34", "blob70k", "cloud"])
@pytest.mark.parametrize("leaf4", [4, 8, 15])
def test_bvh4_sah_collapse_partitions_primitives(name, leaf4):
    """The SAH-optimal collapse (HIPPT_OPT_BVH_COLLAPSE 1): every primitive lies in exactly one
    4-wide leaf of at most `leaf4` primitives (2-wide subtrees merged into one leaf are
    contiguous ranges), every child box contains its leaf's primitives and its child node's
    boxes, nodes have 2-4 children, and the reported stack bound and depth are the tree's."""
    sc = {"cloud": scenes.cloud_scene}.get(name, lambda: scenes.get_scene(name))()
    lib = hippt.load_library()
    try:
        assert lib.hipptSetOption(hippt.OPT_BVH_COLLAPSE, 1) and lib.hipptSetOption(hippt.OPT_BVH_LEAF4, leaf4)
        bvh = hippt.Bvh(sc.verts, extent_hint=800.0)
    finally:
        lib.hipptSetOption(hippt.OPT_BVH_COLLAPSE, -1)
        lib.hipptSetOption(hippt.OPT_BVH_LEAF4, 4)
    f, kids = _decode4(bvh.nodes4)
    covered = np.zeros(sc.num_tris, np.int32)
    bound, depth = 0, 0
    stack = [(0, 0, 1)]
    while stack:
        n, pushes, d = stack.pop()
        depth = max(depth, d)
        used = [c for c in range(4) if not (kids[n, c] == -1 and f[n, 0, 0, c] > 1e37)]
        assert 2 <= len(used) <= 4
        bound = max(bound, pushes + len(used) - 1)
        for c in used:
            k = int(kids[n, c])
            lo, hi = f[n, :, 0, c], f[n, :, 1, c]
            if k >= 0:
                cu = [cc for cc in range(4) if not (kids[k, cc] == -1 and f[k, 0, 0, cc] > 1e37)]
                assert np.all(f[k, :, 0, cu].T >= lo[:, None] - 1e-3) and np.all(f[k, :, 1, cu].T <= hi[:, None] + 1e-3)
                stack.append((k, pushes + len(used) - 1, d + 1))
            else:
                first, count = (~k) >> 4, (~k) & 15
                assert count <= max(leaf4, 4)
                covered[first:first + count] += 1
                v = sc.verts[bvh.order[first:first + count]].reshape(-1, 3)
                assert np.all(v >= lo) and np.all(v <= hi)
    assert np.all(covered == 1)
    assert bound == bvh.stack_bound4 and depth == bvh.depth4


@pytest.mark.parametrize("name", ["cornell34", "blob70k", "random_scene", "cornell_mixed", "voxel", "cloud"])
def test_bvh4_quantized_boxes_contain_float_boxes(name):
    """quantize_bvh4 (hipptBvh4QCopy): every child box decoded exactly (origin + byte * scale, a
    power-of-two scale) contains the float 4-wide box strictly (a plane on the grid moves one
    step outward, so the kernel's rounding of the decoded plane cannot cull a hit the float box
    keeps), each axis uses at most 255 steps of its node's extent, codes are unchanged, and
    unused slots are inverted (lo 255 > hi 0) boxes.  `voxel` puts every plane of integer
    geometry on the grid."""
    sc = {"voxel": scenes.voxel_scene, "cloud": scenes.cloud_scene}.get(name, lambda: scenes.get_scene(name))()
    if sc.num_tris == 0:
        pytest.skip("sphere-only scene")
    bvh = hippt.Bvh(sc.verts, extent_hint=800.0)
    f, kids = _decode4(bvh.nodes4)
    q = bvh.nodes4q
    assert q.shape == (len(kids), 16)
    origin = q[:, 0:3].view(np.float32).astype(np.float64)
    scale = np.stack([q[:, 3], q[:, 10], q[:, 11]], axis=1).view(np.float32).astype(np.float64)
    m, e = np.frexp(scale)
    assert np.all(m == 0.5), "scales are powers of two"
    planes = q[:, 4:10].view(np.uint8).reshape(-1, 3, 2, 4).astype(np.float64)  # node, axis, lo/hi, slot
    assert np.array_equal(q[:, 12:16].view(np.int32), kids)
    for n in range(len(kids)):
        for c in range(4):
            unused = kids[n, c] == -1 and f[n, 0, 0, c] > 1e37
            if unused:
                assert np.all(planes[n, :, 0, c] == 255) and np.all(planes[n, :, 1, c] == 0)
                continue
            lo = origin[n] + planes[n, :, 0, c] * scale[n]
            hi = origin[n] + planes[n, :, 1, c] * scale[n]
            assert np.all(lo < f[n, :, 0, c].astype(np.float64))
            assert np.all(hi > f[n, :, 1, c].astype(np.float64))
        # the scale is (within a step for the origin's rounding) the smallest power of two whose
        # 253 steps cover the node's extent (one spare step below and above)
        used = [c for c in range(4) if not (kids[n, c] == -1 and f[n, 0, 0, c] > 1e37)]
        ext = f[n, :, 1, used].max(axis=0).astype(np.float64) - f[n, :, 0, used].min(axis=0).astype(np.float64)
        assert np.all(253 * scale[n] >= ext)
        assert np.all((ext == 0) | (253 * scale[n] / 4 < ext))


@pytest.mark.parametrize("big", [3.0e38, 3.4e38, -3.4e38])
def test_quantizer_terminates_near_float_max(big):
    """Boxes near +-FLT_MAX (the quantizer's scale search had no upper bound and spun
    forever once the grid origin overflowed): the build returns, the float trees are built, and
    the scene simply has no 8-bit tree (hipptBvh4QNodeCount 0) when no finite grid covers it.
    Runs in a subprocess under a timeout so that a regression fails instead of hanging."""
    import subprocess
    import sys
    import textwrap
    code = textwrap.dedent(f"""
        import numpy as np, hippt
        v = np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0], [{big}, 0, 0, {big}, 1, 0, {big}, 0, 1],
                      [5, 5, 5, 6, 5, 5, 5, 6, 5]], np.float32)
        b = hippt.Bvh(v)
        assert sorted(b.order.tolist()) == [0, 1, 2]
        assert b.nodes4.shape[0] >= 1
        print(b.nodes4q.shape[0])
    """)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    nq = int(out.stdout.strip().splitlines()[-1])
    # -3.4e38 - pad overflows to -inf: no 8-bit tree; the others still quantize (one node)
    assert nq == (0 if big < 0 else 1)
