"""hipptReadMesh (qt-raytracer_amd/csrc/mesh_io.cpp): Wavefront OBJ and PLY triangle input,
the scene-ingestion row of SURVEY.md §8(f) (the reference itself has no mesh reader).

Host code of libhippt.so only, so these run without a GPU.  Round trips write the benchmark
scenes with hippt.scenes.write_obj / write_ply and read them back through the C ABI: the
triangles must come back bit-identical (9 significant digits print a float32 exactly), with
OBJ `usemtl` groups as material indices.
"""
import numpy as np
import pytest

import hippt
from hippt import scenes


def _tri_bits(v):
    return np.ascontiguousarray(v, np.float32).view(np.uint32)


@pytest.mark.parametrize("style", ["plain", "quads", "relative"])
def test_obj_round_trip_cornell(tmp_path, style):
    sc = scenes.cornell34()
    path = str(tmp_path / "cornell.obj")
    scenes.write_obj(sc, path, style=style)
    verts, groups, names = hippt.read_mesh(path)
    assert np.array_equal(_tri_bits(verts), _tri_bits(sc.verts))
    # groups in order of first use: m0, m1, m2 -> material index via the name
    mat = np.array([int(names[g][1:]) for g in groups])
    assert np.array_equal(mat, sc.tri_mat)


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
def test_ply_round_trip_blob(tmp_path, fmt):
    sc = scenes.blob70k()
    path = str(tmp_path / f"blob_{fmt}.ply")
    scenes.write_ply(sc, path, fmt)
    verts, groups, names = hippt.read_mesh(path)
    assert verts.shape == (sc.num_tris, 9)
    assert np.array_equal(_tri_bits(verts), _tri_bits(sc.verts))
    assert names == [""] and not groups.any()


def test_obj_polygons_and_index_forms(tmp_path):
    p = tmp_path / "poly.OBJ"
    p.write_text(
        "# pentagon + triangle, every index form\n"
        "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0.5 1.5 0\nv 0 1 0\n"
        "vt 0 0\nvn 0 0 1\n"
        "f 1/1/1 2//1 3/1 4 5\n"
        "usemtl glass\n"
        "f -5 -4 -3\n"
        "usemtl  \n"
        "f 1 3 5\n")
    verts, groups, names = hippt.read_mesh(str(p))
    v = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0.5, 1.5, 0], [0, 1, 0]], np.float32)
    want = np.stack([np.concatenate([v[0], v[1], v[2]]), np.concatenate([v[0], v[2], v[3]]),
                     np.concatenate([v[0], v[3], v[4]]), np.concatenate([v[0], v[1], v[2]]),
                     np.concatenate([v[0], v[2], v[4]])])
    assert np.array_equal(verts, want)
    # an empty usemtl returns to the unnamed group
    assert groups.tolist() == [0, 0, 0, 1, 0] and names == ["", "glass"]


def test_ply_with_extra_properties_and_elements(tmp_path):
    p = tmp_path / "extra.ply"
    head = ("ply\nformat ascii 1.0\ncomment extra props\nelement vertex 4\nproperty double x\n"
            "property uchar red\nproperty double y\nproperty double z\nproperty float confidence\n"
            "element face 1\nproperty list uchar uint vertex_index\nproperty int flags\n"
            "element edge 1\nproperty int vertex1\nproperty int vertex2\nend_header\n")
    body = "0 255 0 0 1\n1 0 0 0 1\n1 0 1 0 1\n0 0 1 0 1\n4 0 1 2 3 7\n0 1\n"
    p.write_text(head + body)
    verts, groups, _ = hippt.read_mesh(str(p))
    assert verts.shape == (2, 9) and groups.tolist() == [0, 0]
    assert verts[1].tolist() == [0, 0, 0, 1, 1, 0, 0, 1, 0]


@pytest.mark.parametrize("text,msg", [
    ("v 0 0 0\nv 1 0 0\nf 1 2\n", "at least 3"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n", "out of range"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 0\n", "bad face index"),
    ("v 0 x 0\n", "bad coordinate"),
    ("v 0 0 0\n", "no faces"),
])
def test_obj_errors(tmp_path, text, msg):
    p = tmp_path / "bad.obj"
    p.write_text(text)
    with pytest.raises(hippt.HipptError, match=msg):
        hippt.read_mesh(str(p))


def test_read_mesh_errors(tmp_path):
    with pytest.raises(hippt.HipptError, match="cannot open"):
        hippt.read_mesh(str(tmp_path / "missing.obj"))
    (tmp_path / "x.stl").write_text("solid x\n")
    with pytest.raises(hippt.HipptError, match="unknown mesh format"):
        hippt.read_mesh(str(tmp_path / "x.stl"))
    (tmp_path / "t.ply").write_bytes(b"ply\nformat binary_little_endian 1.0\nelement vertex 3\n"
                                     b"property float x\nproperty float y\nproperty float z\nend_header\n\x00\x00")
    with pytest.raises(hippt.HipptError, match="truncated"):
        hippt.read_mesh(str(tmp_path / "t.ply"))


def test_from_mesh_file_scene(tmp_path):
    path = str(tmp_path / "cornell.obj")
    scenes.write_obj(scenes.cornell34(), path, style="quads")
    sc = scenes.from_mesh_file(path, albedo=[scenes.WHITE, scenes.GREEN, scenes.RED])
    assert sc.num_tris == 34 and sc.lambertian_triangles
    assert np.array_equal(sc.tri_mat, scenes.cornell34().tri_mat)
