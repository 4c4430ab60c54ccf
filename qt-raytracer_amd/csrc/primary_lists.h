// primary_lists.h — per-pixel candidate lists for the primary rays of a pinhole camera (host).
#pragma once

#include <cstdint>
#include <vector>

#include "hippt_device.h"

namespace hippt {

// For the pixels of rows y0, y0+stride, ... (rows of them) of a width x height image seen by the
// pinhole camera `cam` (lens_radius 0), the primitive slots (leaf order) whose projection
// overlaps each pixel's footprint widened by a margin: offsets[p]..offsets[p+1] index ids[] for
// band pixel p = k*width + x.  `tris` = numSlots device triangle records (12 floats each,
// MeshParams::tris).  Conservative: a primitive with a vertex at or behind the camera plane is a
// candidate of every pixel.  Returns false (lists empty) for a lens camera or a scene with
// spheres.
bool build_primary_lists(const float *tris, int numSlots, const CameraF &cam, int width, int height, int y0, int rows,
                         int stride, std::vector<uint32_t> &offsets, std::vector<uint32_t> &ids);

}  // namespace hippt
