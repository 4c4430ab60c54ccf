// item_order.h — the order in which the megakernel's queues hand out a band's pixels (host).
#pragma once

#include <cstdint>
#include <vector>

#include "bvh_builder.h"
#include "hippt_device.h"

namespace hippt {

// The band's pixels (rows y0, y0+stride, ..., `rows` of them, of a width x height image) in runs
// of 64 consecutive band pixels: order[j] = the run handed out j-th within every frame.  Runs
// whose sample rays (4 pixel centres through the pinhole of `cam`) hit the scene come first and
// runs that see only the sky last, each group in image order, so that a queue's last items are
// the cheapest (the launch's tail); returns the number of runs that hit.  `tris`: the device primitive records of
// `bvh`'s leaf order (MeshParams::tris).  The order changes which lane traces a sample, never
// what it computes.
size_t build_run_order(const Bvh4 &bvh, const float *tris, const CameraF &cam, int width, int height, int y0, int rows,
                     int stride, std::vector<uint32_t> &order);

// The queues' item table of a batch of `frames` frames of `bandPixels` band pixels, from a frame's
// run order (build_run_order; its first `hitRuns` entries hit the scene): slot s = f*runs + r
// (run r of frame f, runs = bandPixels/64) is handed out as the 64 items starting at table[s].
// Within each of the kQueues contiguous queue ranges (trace::queue_start) the scene-hitting runs
// of all its frames come first and the sky's last, so the sky phase at a queue's end outlasts
// the paths started before it.
void build_item_table(const std::vector<uint32_t> &order, size_t hitRuns, unsigned bandPixels, unsigned frames,
                      unsigned queues, std::vector<uint32_t> &table);

}  // namespace hippt
