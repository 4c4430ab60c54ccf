"""Synthetic scenes of SURVEY.md §8(d) as float32 triangle soups.

The reference ships no triangle scene (its CPU demo is ``random_scene`` of spheres,
RayTracer.h:599-643, and the GPU kernel hard-codes four spheres,
CudaPathTracerKernel.cu:113-116), so the benchmark scenes are defined here:

* ``cornell34`` — open-front Cornell-style box: floor, ceiling, back wall, left (x=0, green)
  and right (x=555, red) walls, plus two white axis-aligned boxes (12 triangles each);
  34 triangles.  The sky (RayTracer.h:593-595) is the only light, entering through the
  open front.
* ``blob70k`` — the Cornell walls (10 triangles) around a lat-long displaced sphere of
  256 x 136 quads (69,632 triangles; the pole rows are degenerate), 69,642 in total.

Camera (both): lookfrom (278, 278, -800) -> lookat (278, 278, 0), vup +y, vfov 40,
aperture 0, focus distance 10 (RayTracerFboItem.cpp:49-56 uses 10).

Scenes with spheres and the reference's other materials (RayTracer.h:490-540):

* ``random_scene`` — the recipe of RayTracer.h ``random_scene`` (:599-643: ground sphere,
  22 x 22 jittered small spheres, 80% Lambertian / 15% Metal / 5% Dielectric, three big
  spheres) drawn from a seeded numpy RNG (the reference's own RNG is nondeterministic,
  RayTracer.h:25-55), with RenderWorker::render's camera (RayTracerFboItem.cpp:50-56).
  ``load_scene_file(tests/golden/ref_random_scene.scene)`` is one scene the reference
  itself generated.
* ``cornell_mixed`` — the Cornell walls and the short box, a metal tall box, a glass
  sphere on the short box and a fuzzy metal sphere: triangles and spheres, all three
  materials.
"""
from __future__ import annotations

import dataclasses
import os
import struct

import numpy as np

WHITE = (0.73, 0.73, 0.73)
GREEN = (0.12, 0.45, 0.15)
RED = (0.65, 0.05, 0.05)

SCENE_MAGIC = 0x53505448      # v1: Lambertian triangles
SCENE_MAGIC_V2 = 0x32505448   # v2: triangles, spheres, material kinds

MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC = 0, 1, 2
# == hipptMaterial (include/hippt.h) == po_material (oracle/pt_oracle.h)
MATERIAL_DTYPE = np.dtype([("kind", "<i4"), ("albedo", "<f4", (3,)), ("fuzz", "<f4"), ("ir", "<f4")])


@dataclasses.dataclass
class Scene:
    name: str
    verts: np.ndarray          # (n, 9) float32: v0, v1, v2
    tri_mat: np.ndarray        # (n,) int32
    albedo: np.ndarray         # (k, 3) float32
    lookfrom: tuple = (278.0, 278.0, -800.0)
    lookat: tuple = (278.0, 278.0, 0.0)
    vup: tuple = (0.0, 1.0, 0.0)
    vfov: float = 40.0
    aperture: float = 0.0
    focus: float = 10.0
    spheres: np.ndarray = dataclasses.field(default_factory=lambda: np.zeros((0, 4), np.float32))  # cx cy cz r
    sph_mat: np.ndarray = dataclasses.field(default_factory=lambda: np.zeros(0, np.int32))
    mat_kind: np.ndarray = None  # (k,) int32, None = all Lambertian
    fuzz: np.ndarray = None      # (k,) float32 (Metal)
    ir: np.ndarray = None        # (k,) float32 (Dielectric)

    @property
    def num_tris(self) -> int:
        return int(self.verts.shape[0])

    @property
    def num_spheres(self) -> int:
        return int(np.asarray(self.spheres).reshape(-1, 4).shape[0])

    @property
    def lambertian_triangles(self) -> bool:
        """True when hipptUploadMesh / the v1 file format can carry the scene."""
        return self.num_spheres == 0 and (self.mat_kind is None or not np.any(np.asarray(self.mat_kind)))

    def materials(self) -> np.ndarray:
        """Structured array of MATERIAL_DTYPE, one per material."""
        k = int(np.asarray(self.albedo).reshape(-1, 3).shape[0])
        m = np.zeros(k, MATERIAL_DTYPE)
        m["albedo"] = np.asarray(self.albedo, np.float32).reshape(-1, 3)
        m["kind"] = 0 if self.mat_kind is None else np.asarray(self.mat_kind, np.int32)
        m["fuzz"] = 0.0 if self.fuzz is None else np.asarray(self.fuzz, np.float32)
        m["ir"] = 1.0 if self.ir is None else np.asarray(self.ir, np.float32)
        return m


def _quad(a, b, c, d):
    """Two triangles (a, b, c) and (a, c, d)."""
    return [a + b + c, a + c + d]


def _box(lo, hi):
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    p = {
        "000": (x0, y0, z0), "100": (x1, y0, z0), "110": (x1, y1, z0), "010": (x0, y1, z0),
        "001": (x0, y0, z1), "101": (x1, y0, z1), "111": (x1, y1, z1), "011": (x0, y1, z1),
    }
    faces = [
        ("000", "100", "110", "010"),  # z = z0
        ("001", "011", "111", "101"),  # z = z1
        ("000", "010", "011", "001"),  # x = x0
        ("100", "101", "111", "110"),  # x = x1
        ("000", "001", "101", "100"),  # y = y0
        ("010", "110", "111", "011"),  # y = y1
    ]
    tris = []
    for f in faces:
        tris += _quad(*(p[k] for k in f))
    return tris


def _walls():
    s = 555.0
    tris, mats = [], []
    for quad, m in (
        (((0, 0, 0), (s, 0, 0), (s, 0, s), (0, 0, s)), 0),      # floor
        (((0, s, 0), (0, s, s), (s, s, s), (s, s, 0)), 0),      # ceiling
        (((0, 0, s), (s, 0, s), (s, s, s), (0, s, s)), 0),      # back wall
        (((0, 0, 0), (0, 0, s), (0, s, s), (0, s, 0)), 1),      # left wall x = 0 (green)
        (((s, 0, 0), (s, s, 0), (s, s, s), (s, 0, s)), 2),      # right wall x = 555 (red)
    ):
        tris += _quad(*quad)
        mats += [m, m]
    return tris, mats


def cornell34() -> Scene:
    tris, mats = _walls()
    for lo, hi in (((130, 0, 65), (295, 165, 230)), ((265, 0, 295), (430, 330, 460))):
        b = _box(lo, hi)
        tris += b
        mats += [0] * len(b)
    return Scene(
        name="cornell34",
        verts=np.asarray(tris, dtype=np.float64).astype(np.float32),
        tri_mat=np.asarray(mats, dtype=np.int32),
        albedo=np.asarray([WHITE, GREEN, RED], dtype=np.float32),
    )


def blob_mesh(nu: int = 256, nv: int = 136, center=(278.0, 180.0, 278.0), radius: float = 150.0) -> np.ndarray:
    """Lat-long displaced sphere r = R (1 + 0.08 sin 7θ cos 5φ): nu*nv quads, 2*nu*nv tris."""
    th = np.pi * np.arange(nv + 1, dtype=np.float64) / nv
    ph = 2.0 * np.pi * np.arange(nu + 1, dtype=np.float64) / nu
    T, P = np.meshgrid(th, ph, indexing="ij")  # (nv+1, nu+1)
    r = radius * (1.0 + 0.08 * np.sin(7.0 * T) * np.cos(5.0 * P))
    X = center[0] + r * np.sin(T) * np.cos(P)
    Y = center[1] + r * np.cos(T)
    Z = center[2] + r * np.sin(T) * np.sin(P)
    V = np.stack([X, Y, Z], axis=-1).astype(np.float32)  # (nv+1, nu+1, 3)
    a = V[:-1, :-1]
    b = V[:-1, 1:]
    c = V[1:, 1:]
    d = V[1:, :-1]
    t1 = np.concatenate([a, b, c], axis=-1).reshape(-1, 9)
    t2 = np.concatenate([a, c, d], axis=-1).reshape(-1, 9)
    return np.stack([t1, t2], axis=1).reshape(-1, 9)


def blob70k() -> Scene:
    return blob_scene(256, 136, "blob70k")


def blob_scene(nu: int, nv: int, name: str | None = None) -> Scene:
    """blob70k's walls around a blob of nu x nv quads (blob70k: 256 x 136)."""
    tris, mats = _walls()
    walls = np.asarray(tris, dtype=np.float64).astype(np.float32)
    blob = blob_mesh(nu, nv)
    verts = np.concatenate([walls, blob], axis=0)
    tri_mat = np.concatenate([np.asarray(mats, np.int32), np.zeros(len(blob), np.int32)])
    return Scene(name=name or f"blob{nu}x{nv}", verts=np.ascontiguousarray(verts), tri_mat=tri_mat,
                 albedo=np.asarray([WHITE, GREEN, RED], dtype=np.float32))


def random_scene(seed: int = 2024) -> Scene:
    """RayTracer.h random_scene (:599-643) drawn from numpy's PCG64 (seeded), camera of
    RenderWorker::render (RayTracerFboItem.cpp:50-56: (13,2,3) -> 0, vfov 20, aperture 0.1,
    focus 10)."""
    rng = np.random.default_rng(seed)
    rd = rng.random
    spheres, mats = [], []

    def add(c, r, kind, albedo=(0.0, 0.0, 0.0), fuzz=0.0, ir=1.0):
        spheres.append((*c, r))
        mats.append((kind, albedo, min(fuzz, 1.0) if kind == MAT_METAL else fuzz, ir))

    add((0.0, -1000.0, 0.0), 1000.0, MAT_LAMBERTIAN, (0.5, 0.5, 0.5))
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rd()
            c = (a + 0.9 * rd(), 0.2, b + 0.9 * rd())
            if np.sqrt((c[0] - 4.0) ** 2 + (c[1] - 0.2) ** 2 + c[2] ** 2) <= 0.9:
                continue
            if choose < 0.8:
                alb = tuple(float(rd() * rd()) for _ in range(3))
                add(c, 0.2, MAT_LAMBERTIAN, alb)
            elif choose < 0.95:
                alb = tuple(float(0.5 + 0.5 * rd()) for _ in range(3))
                add(c, 0.2, MAT_METAL, alb, fuzz=0.5 * rd())
            else:
                add(c, 0.2, MAT_DIELECTRIC, (1.0, 1.0, 1.0), ir=1.5)
    add((0.0, 1.0, 0.0), 1.0, MAT_DIELECTRIC, (1.0, 1.0, 1.0), ir=1.5)
    add((-4.0, 1.0, 0.0), 1.0, MAT_LAMBERTIAN, (0.4, 0.2, 0.1))
    add((4.0, 1.0, 0.0), 1.0, MAT_METAL, (0.7, 0.6, 0.5), fuzz=0.0)
    return _sphere_scene("random_scene", spheres, mats)


def _sphere_scene(name, spheres, mats, verts=None, tri_mat=None, **cam) -> Scene:
    kw = dict(lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 0.0, 0.0), vup=(0.0, 1.0, 0.0), vfov=20.0, aperture=0.1,
              focus=10.0)
    kw.update(cam)
    return Scene(
        name=name,
        verts=np.zeros((0, 9), np.float32) if verts is None else np.ascontiguousarray(verts, np.float32),
        tri_mat=np.zeros(0, np.int32) if tri_mat is None else np.asarray(tri_mat, np.int32),
        albedo=np.asarray([m[1] for m in mats], np.float32).reshape(-1, 3),
        spheres=np.asarray(spheres, np.float64).astype(np.float32).reshape(-1, 4),
        sph_mat=np.arange(len(spheres), dtype=np.int32) if len(spheres) == len(mats) else None,
        mat_kind=np.asarray([m[0] for m in mats], np.int32),
        fuzz=np.asarray([m[2] for m in mats], np.float32),
        ir=np.asarray([m[3] for m in mats], np.float32),
        **kw,
    )


def cornell_mixed() -> Scene:
    """Cornell walls + short white box, metal tall box, glass and fuzzy-metal spheres."""
    tris, tmat = _walls()
    short = _box((130, 0, 65), (295, 165, 230))
    tall = _box((265, 0, 295), (430, 330, 460))
    tris = tris + short + tall
    tmat = tmat + [0] * len(short) + [3] * len(tall)
    mats = [(MAT_LAMBERTIAN, WHITE, 0.0, 1.0), (MAT_LAMBERTIAN, GREEN, 0.0, 1.0), (MAT_LAMBERTIAN, RED, 0.0, 1.0),
            (MAT_METAL, (0.8, 0.85, 0.88), 0.05, 1.0), (MAT_DIELECTRIC, (1.0, 1.0, 1.0), 0.0, 1.5),
            (MAT_METAL, (0.9, 0.6, 0.3), 0.3, 1.0)]
    sc = _sphere_scene("cornell_mixed", [], mats, verts=np.asarray(tris, np.float64).astype(np.float32),
                       tri_mat=tmat, lookfrom=(278.0, 278.0, -800.0), lookat=(278.0, 278.0, 0.0), vfov=40.0,
                       aperture=0.0, focus=10.0)
    sc.spheres = np.asarray([(212.5, 245.0, 147.5, 80.0), (420.0, 60.0, 150.0, 60.0)], np.float32)
    sc.sph_mat = np.asarray([4, 5], np.int32)
    return sc


def cloud_scene(n: int = 180, seed: int = 7) -> Scene:
    """Test scene for deep traversal stacks: the Cornell walls around a cloud of n small,
    randomly oriented triangles filling the box's middle.  Rays cross many overlapping child
    boxes (4-hit node visits are common), and it still fits the LDS scene copy at n <= 200."""
    rng = np.random.default_rng(seed)
    tris, mats = _walls()
    walls = np.asarray(tris, np.float64).astype(np.float32)
    c = rng.uniform(120.0, 435.0, size=(n, 1, 3))
    d = rng.normal(0.0, 18.0, size=(n, 3, 3))
    cloud = (c + d).reshape(n, 9).astype(np.float32)
    verts = np.concatenate([walls, cloud], axis=0)
    tri_mat = np.concatenate([np.asarray(mats, np.int32), np.zeros(n, np.int32)])
    return Scene(name=f"cloud{n}", verts=np.ascontiguousarray(verts), tri_mat=tri_mat,
                 albedo=np.asarray([WHITE, GREEN, RED], dtype=np.float32))


def voxel_scene(n: int = 6) -> Scene:
    """Test scene for the 8-bit child boxes: a staircase of unit cubes at integer coordinates
    (every box plane on a power-of-two quantisation grid, so floor/ceil add no slack) on an
    integer floor, seen from an integer camera position."""
    tris = []
    for i in range(n):
        for j in range(n):
            for k in range(max(1, n - i - j)):
                tris += _box((i, k, j), (i + 1, k + 1, j + 1))
    tris += _quad((-2, 0, -2), (-2, 0, n + 2), (n + 2, 0, n + 2), (n + 2, 0, -2))
    verts = np.asarray(tris, np.float64).astype(np.float32)
    tri_mat = (np.arange(len(tris)) // 12 % 3).astype(np.int32)
    return Scene(name=f"voxel{n}", verts=verts, tri_mat=tri_mat,
                 albedo=np.asarray([WHITE, GREEN, RED], dtype=np.float32),
                 lookfrom=(float(2 * n + 4), float(n + 2), float(2 * n + 6)), lookat=(0.0, 1.0, 0.0), vfov=40.0)


SCENES = {"cornell34": cornell34, "blob70k": blob70k, "random_scene": random_scene, "cornell_mixed": cornell_mixed}


def get_scene(name: str) -> Scene:
    try:
        return SCENES[name]()
    except KeyError:
        raise ValueError(f"unknown scene {name!r}; choose from {sorted(SCENES)}") from None


def write_scene_file(scene: Scene, path: str) -> None:
    """Binary scene file read by oracle/ref_harness.cpp (load_scene): v1 for Lambertian
    triangle scenes, v2 otherwise."""
    cam = list(scene.lookfrom) + list(scene.lookat) + list(scene.vup) + [scene.vfov, scene.aperture, scene.focus]
    with open(path, "wb") as f:
        if scene.lambertian_triangles:
            f.write(struct.pack("<3i", SCENE_MAGIC, scene.num_tris, len(scene.albedo)))
            f.write(np.ascontiguousarray(scene.verts, dtype="<f4").tobytes())
            f.write(np.ascontiguousarray(scene.tri_mat, dtype="<i4").tobytes())
            f.write(np.ascontiguousarray(scene.albedo, dtype="<f4").tobytes())
        else:
            mats = scene.materials()
            f.write(struct.pack("<4i", SCENE_MAGIC_V2, scene.num_tris, scene.num_spheres, len(mats)))
            f.write(np.ascontiguousarray(scene.verts, dtype="<f4").tobytes())
            f.write(np.ascontiguousarray(scene.tri_mat, dtype="<i4").tobytes())
            f.write(np.ascontiguousarray(scene.spheres, dtype="<f4").tobytes())
            f.write(np.ascontiguousarray(scene.sph_mat, dtype="<i4").tobytes())
            f.write(mats.tobytes())
        f.write(struct.pack("<12d", *cam))


def load_scene_file(path: str, name: str = None) -> Scene:
    """Reads a v1 or v2 scene file (write_scene_file, oracle/ref_harness.cpp random_scene)."""
    with open(path, "rb") as f:
        data = f.read()
    magic = struct.unpack_from("<i", data, 0)[0]
    off = 4
    if magic == SCENE_MAGIC:
        nt, nm = struct.unpack_from("<2i", data, off)
        ns = 0
        off += 8
    elif magic == SCENE_MAGIC_V2:
        nt, ns, nm = struct.unpack_from("<3i", data, off)
        off += 12
    else:
        raise ValueError(f"{path}: not a scene file")

    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(data, dtype=dtype, count=count, offset=off).copy()
        off += a.nbytes
        return a

    verts = take("<f4", nt * 9).reshape(-1, 9)
    tri_mat = take("<i4", nt)
    if magic == SCENE_MAGIC:
        albedo = take("<f4", nm * 3).reshape(-1, 3)
        mats = None
        spheres, sph_mat = np.zeros((0, 4), np.float32), np.zeros(0, np.int32)
    else:
        spheres = take("<f4", ns * 4).reshape(-1, 4)
        sph_mat = take("<i4", ns)
        mats = take(MATERIAL_DTYPE, nm)
        albedo = np.ascontiguousarray(mats["albedo"])
    cam = struct.unpack_from("<12d", data, off)
    sc = Scene(name=name or os.path.splitext(os.path.basename(path))[0], verts=verts, tri_mat=tri_mat, albedo=albedo,
               lookfrom=tuple(cam[0:3]), lookat=tuple(cam[3:6]), vup=tuple(cam[6:9]), vfov=cam[9], aperture=cam[10],
               focus=cam[11], spheres=spheres, sph_mat=sph_mat)
    if mats is not None:
        sc.mat_kind = np.ascontiguousarray(mats["kind"])
        sc.fuzz = np.ascontiguousarray(mats["fuzz"])
        sc.ir = np.ascontiguousarray(mats["ir"])
    return sc


def write_obj(scene: Scene, path: str, style: str = "plain") -> None:
    """Triangles of `scene` as a Wavefront OBJ file: one `usemtl m<k>` group per material,
    coordinates printed with 9 significant digits (they read back to the same float32).
    style "quads": consecutive same-material pairs (a, b, c) (a, c, d) — the layout of every
    quad here — become one quad `f a b/b c//c d/d/d`; "relative": negative vertex indices."""
    v = np.asarray(scene.verts, np.float32).reshape(-1, 3)
    mats = np.asarray(scene.tri_mat)
    nv = len(v)

    def ref(k):  # 1-based vertex k
        return str(k - nv - 1) if style == "relative" else str(k)

    with open(path, "w") as f:
        f.write(f"# {scene.name}: {scene.num_tris} triangles\n")
        for x, y, z in v:
            f.write(f"v {x:.9g} {y:.9g} {z:.9g}\n")
        cur, t, n = None, 0, scene.num_tris
        while t < n:
            if mats[t] != cur:
                cur = mats[t]
                f.write(f"usemtl m{cur}\n")
            a, b, c = 3 * t + 1, 3 * t + 2, 3 * t + 3
            if style == "quads" and t + 1 < n and mats[t + 1] == cur:
                d = 3 * t + 6
                f.write(f"f {a} {b}/{b} {c}//{c} {d}/{d}/{d}\n")
                t += 2
            else:
                f.write(f"f {ref(a)} {ref(b)} {ref(c)}\n")
                t += 1


def write_ply(scene: Scene, path: str, fmt: str = "binary_little_endian") -> None:
    """Triangles of `scene` as a PLY file (vertex x, y, z float; face list uchar int), one
    vertex per corner; fmt ascii / binary_little_endian / binary_big_endian."""
    v = np.asarray(scene.verts, np.float32).reshape(-1, 3)
    n = scene.num_tris
    head = (f"ply\nformat {fmt} 1.0\ncomment {scene.name}\nelement vertex {len(v)}\n"
            "property float x\nproperty float y\nproperty float z\n"
            f"element face {n}\nproperty list uchar int vertex_indices\nend_header\n")
    with open(path, "wb") as f:
        f.write(head.encode())
        if fmt == "ascii":
            lines = [f"{x:.9g} {y:.9g} {z:.9g}" for x, y, z in v]
            lines += [f"3 {3 * t} {3 * t + 1} {3 * t + 2}" for t in range(n)]
            f.write(("\n".join(lines) + "\n").encode())
        else:
            e = "<" if fmt == "binary_little_endian" else ">"
            f.write(v.astype(e + "f4").tobytes())
            face = np.zeros(n, dtype=[("c", "u1"), ("i", e + "i4", (3,))])
            face["c"] = 3
            face["i"] = np.arange(3 * n, dtype=np.int64).reshape(n, 3)
            f.write(face.tobytes())


def from_mesh_file(path: str, albedo=None, name: str = None, **camera) -> Scene:
    """Scene from an OBJ/PLY file read by libhippt (hipptReadMesh): one Lambertian material per
    OBJ `usemtl` group (albedo: (groups, 3), default white 0.73), camera keywords as Scene's
    (default: the Cornell camera)."""
    from hippt import read_mesh  # the library reader, no Python fallback
    verts, groups, names = read_mesh(path)
    k = max(1, len(names))
    alb = np.tile(np.float32(WHITE), (k, 1)) if albedo is None else np.asarray(albedo, np.float32).reshape(k, 3)
    return Scene(name=name or os.path.splitext(os.path.basename(path))[0], verts=verts,
                 tri_mat=groups.astype(np.int32), albedo=alb, **camera)
