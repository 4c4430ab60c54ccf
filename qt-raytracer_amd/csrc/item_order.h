// item_order.h — the order in which the megakernel's queues hand out a band's pixels (host).
#pragma once

#include <cstdint>
#include <vector>

#include "bvh_builder.h"
#include "hippt_device.h"

namespace hippt {

// An estimate of each run's sample length in segments, for the band's pixels (rows y0, y0+stride,
// ..., `rows` of them, of a width x height image) in runs of 64 consecutive band pixels: 1 for a
// run that sees the sky, up to maxDepth for one deep in the scene (item_order.cpp).  `tris`: the
// device primitive records of `bvh`'s leaf order (MeshParams::tris).  `threads` host threads share
// the runs (the result does not depend on it).
void run_costs(const Bvh4 &bvh, const float *tris, const CameraF &cam, int width, int height, int y0, int rows,
               int stride, int maxDepth, std::vector<float> &cost, int threads = 1);

// The queues' item table of a batch of `frames` frames of `bandPixels` band pixels: slot s =
// f*runs + r (run r of frame f, runs = cost.size()) is handed out as the 64 items starting at
// table[s].  Within each of the `queues` contiguous queue ranges (trace::queue_start) the slots
// come longest estimate first (stable), so that waves hold samples of similar length and each
// queue ends on the cheapest.  The order changes which lane traces a sample, never what it
// computes.
void build_item_table(const std::vector<float> &cost, unsigned bandPixels, unsigned frames, unsigned queues,
                      std::vector<uint32_t> &table);

}  // namespace hippt
