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
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

WHITE = (0.73, 0.73, 0.73)
GREEN = (0.12, 0.45, 0.15)
RED = (0.65, 0.05, 0.05)

SCENE_MAGIC = 0x53505448


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

    @property
    def num_tris(self) -> int:
        return int(self.verts.shape[0])


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
    tris, mats = _walls()
    walls = np.asarray(tris, dtype=np.float64).astype(np.float32)
    blob = blob_mesh()
    verts = np.concatenate([walls, blob], axis=0)
    tri_mat = np.concatenate([np.asarray(mats, np.int32), np.zeros(len(blob), np.int32)])
    return Scene(name="blob70k", verts=np.ascontiguousarray(verts), tri_mat=tri_mat,
                 albedo=np.asarray([WHITE, GREEN, RED], dtype=np.float32))


SCENES = {"cornell34": cornell34, "blob70k": blob70k}


def get_scene(name: str) -> Scene:
    try:
        return SCENES[name]()
    except KeyError:
        raise ValueError(f"unknown scene {name!r}; choose from {sorted(SCENES)}") from None


def write_scene_file(scene: Scene, path: str) -> None:
    """Binary scene file read by oracle/ref_harness.cpp (load_scene)."""
    with open(path, "wb") as f:
        f.write(struct.pack("<3i", SCENE_MAGIC, scene.num_tris, len(scene.albedo)))
        f.write(np.ascontiguousarray(scene.verts, dtype="<f4").tobytes())
        f.write(np.ascontiguousarray(scene.tri_mat, dtype="<i4").tobytes())
        f.write(np.ascontiguousarray(scene.albedo, dtype="<f4").tobytes())
        cam = list(scene.lookfrom) + list(scene.lookat) + list(scene.vup) + [scene.vfov, scene.aperture, scene.focus]
        f.write(struct.pack("<12d", *cam))
