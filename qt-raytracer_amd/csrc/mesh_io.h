// mesh_io.h — host-side triangle mesh readers (Wavefront OBJ, PLY) for hipptReadMesh.
//
// The reference has no mesh input (its scenes are spheres built in code, RayTracer.h:599-643);
// SURVEY.md §8(f) asks for an OBJ/PLY reader so that meshes reach hipptUploadMesh /
// hipptUploadScene.  Output: a triangle soup (v0, v1, v2 per triangle, float32) and one
// group index per triangle (OBJ `usemtl` groups in order of first use; PLY: 0).
#pragma once

#include <string>
#include <vector>

namespace hippt {

struct MeshData {
    std::vector<float> verts;         // numTris * 9
    std::vector<int> group;           // numTris
    std::vector<std::string> groups;  // group names ("" = faces before any usemtl)
};

// Dispatches on the file extension (.obj / .ply, case-insensitive).  Polygons are
// fan-triangulated (v0, vi, vi+1).  On failure returns false with a message naming the
// file and, where it applies, the line.
bool read_mesh(const std::string &path, MeshData &out, std::string &err);
bool read_obj(const std::string &path, MeshData &out, std::string &err);
bool read_ply(const std::string &path, MeshData &out, std::string &err);

}  // namespace hippt
