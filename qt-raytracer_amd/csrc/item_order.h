// item_order.h — the order in which the megakernel's queues hand out a band's pixels (host).
#pragma once

#include <cstdint>
#include <vector>

#include "bvh_builder.h"
#include "hippt_device.h"

namespace hippt {

// The band's runs of 64 pixels, the unit a table slot hands out (MeshParams::runOrder): with
// tileShift < 6, tiles of 2^tileShift columns x 2^(6 - tileShift) band rows over the band's whole
// strips of that many rows (a wave's camera rays then cover a compact patch of the image, and its
// bounces start from nearby points: fewer distinct tree lines per wave for a tree in global memory),
// then runs of 64 consecutive band pixels over the rest; tileShift 6: runs of 64 consecutive band
// pixels only.  Tiles need a width that is a multiple of the tile's (tile_shift_for falls back to 6).
struct RunLayout {
    unsigned width = 0, rows = 0, tileShift = 6;
};
// A table entry's flag: the run is a tile (its item k is at column k mod 2^tileShift, band row
// k >> tileShift of the tile; trace::order_item)
constexpr uint32_t kRunTile = 0x80000000u;
unsigned tile_shift_for(unsigned width, unsigned tileShift);
size_t run_count(const RunLayout &L);
// band pixel of run r's item 0, | kRunTile for a tile
uint32_t run_base(const RunLayout &L, size_t r);
// band pixel of item k of run r
uint32_t run_pixel(const RunLayout &L, size_t r, unsigned k);

// An estimate of each run's sample length in segments, for the band's pixels (rows y0, y0+stride,
// ..., `rows` of them, of a width x height image) in the runs of layout L: 1 for a run that sees
// the sky, up to maxDepth for one deep in the scene (item_order.cpp).  `tris`: the device
// primitive records of `bvh`'s leaf order (MeshParams::tris).  `threads` host threads share the
// runs (the result does not depend on it).
void run_costs(const Bvh4 &bvh, const float *tris, const CameraF &cam, const RunLayout &L, int height, int y0,
               int stride, int maxDepth, std::vector<float> &cost, int threads = 1);

// The queues' item table of a batch of `frames` frames of the band's L.width * L.rows pixels: slot
// s = f*runs + r (run r of frame f, runs = cost.size()), at queue position f*bandPixels + 64*r, is
// handed out as the 64 items of run r of frame f: table[s] = f*bandPixels + run_base(L, r).  Within
// each of the `queues` contiguous queue ranges of positions (trace::queue_start) the slots come
// longest estimate first (stable), so that waves hold samples of similar length and each queue ends
// on the cheapest.  The order changes which lane traces a sample, never what it computes.
void build_item_table(const std::vector<float> &cost, const RunLayout &L, unsigned frames, unsigned queues,
                      std::vector<uint32_t> &table);

}  // namespace hippt
