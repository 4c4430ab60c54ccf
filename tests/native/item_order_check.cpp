// item_order_check.cpp — host checks of the queues' item table (qt-raytracer_amd/csrc/item_order.cpp),
// built and run by tests/test_item_order.py: the table is a permutation of the batch's run slots
// for any band size, frame count and queue count; within a queue, the estimates never increase;
// the Cornell box's sky runs cost 1.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "item_order.h"

using namespace hippt;

// The table by definition: per queue, its slots stably sorted by estimate, longest first (the
// round-3 implementation; build_item_table must give the same table in O(slots)); slot s sits at
// queue position (s / runs) * bandPixels + 64 * (s % runs) and hands out run s % runs of its frame.
static void reference_table(const std::vector<float> &cost, const RunLayout &L, unsigned frames, unsigned queues,
                            std::vector<uint32_t> &table) {
    const unsigned bandPixels = L.width * L.rows;
    const size_t runs = cost.size(), slots = runs * frames;
    table.assign(slots, 0u);
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    auto pos = [&](size_t s) { return (unsigned long long)(s / runs) * bandPixels + 64 * (s % runs); };
    auto item = [&](size_t s) { return uint32_t((s / runs) * bandPixels) + run_base(L, s % runs); };
    size_t s = 0;
    std::vector<size_t> at, sorted;
    for (unsigned g = 0; g < queues && s < slots; ++g) {
        const unsigned long long end = total * (g + 1) / queues;
        at.clear();
        for (; s < slots && pos(s) < end; ++s) at.push_back(s);
        sorted = at;
        std::stable_sort(sorted.begin(), sorted.end(), [&](size_t a, size_t b) { return cost[a % runs] > cost[b % runs]; });
        for (size_t k = 0; k < at.size(); ++k) table[at[k]] = item(sorted[k]);
    }
    for (; s < slots; ++s) table[s] = item(s);
}

// the kernel's decode of a table entry's item k (trace::run_item)
static uint32_t run_item(uint32_t v, unsigned k, unsigned width, unsigned ts) {
    return (v & 0x7fffffffu) + ((v >> 31) ? (k & ((1u << ts) - 1u)) + (k >> ts) * width : k);
}

static int check_table(unsigned width, unsigned rows, unsigned frames, unsigned queues, unsigned tileShift) {
    RunLayout L{width, rows, tile_shift_for(width, tileShift)};
    const unsigned bandPixels = width * rows;
    const size_t runs = run_count(L);
    std::vector<float> cost(runs);
    for (size_t r = 0; r < runs; ++r) cost[r] = float((r * 7919) % 13) * 0.5f + 1.0f;
    std::vector<uint32_t> t, ref;
    build_item_table(cost, L, frames, queues, t);
    if (t.size() != runs * frames) return 1;
    reference_table(cost, L, frames, queues, ref);
    if (t != ref) return 4;
    // every (frame, band pixel) exactly once: the slots' 64 items each, then the positions past the
    // frame's whole runs as themselves (trace::order_item)
    std::vector<unsigned char> seen(size_t(bandPixels) * frames, 0);
    for (size_t k = 0; k < t.size(); ++k) {
        for (unsigned i = 0; i < 64; ++i) {
            const uint32_t it = run_item(t[k], i, width, L.tileShift);
            if (it >= seen.size() || seen[it]++) return 2;
        }
    }
    for (unsigned f = 0; f < frames; ++f)
        for (size_t q = runs * 64; q < bandPixels; ++q)
            if (seen[size_t(f) * bandPixels + q]++) return 2;
    for (unsigned char c : seen)
        if (c != 1) return 2;
    // within each queue range the estimates of the handed-out runs never increase
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    std::vector<size_t> runOf(bandPixels, 0);
    for (size_t r = 0; r < runs; ++r) runOf[run_base(L, r) & 0x7fffffffu] = r;
    for (unsigned g = 0; g < queues; ++g) {
        const unsigned long long lo = total * g / queues, hi = total * (g + 1) / queues;
        float prev = 1e30f;
        for (size_t k = 0; k < t.size(); ++k) {
            const unsigned long long pos = (k / runs) * bandPixels + 64 * (k % runs);
            if (pos < lo || pos >= hi) continue;
            const float c = cost[runOf[(t[k] & 0x7fffffffu) % bandPixels]];
            if (c > prev) return 3;
            prev = c;
        }
    }
    // tiles: item k of a tile run sits at column k mod 2^shift, row k >> shift of the tile
    if (L.tileShift < 6 && rows >= (64u >> L.tileShift) && runs) {
        const uint32_t b = run_base(L, 0);
        if (!(b & kRunTile) || run_pixel(L, 0, 63) != (63u & ((1u << L.tileShift) - 1u)) + (63u >> L.tileShift) * width)
            return 6;
    }
    return 0;
}

int main() {
    // width, band rows, frames, queues
    const unsigned shapes[][4] = {{640, 1, 1, 8}, {640, 1, 3, 8}, {650, 1, 7, 8}, {1920, 135, 64, 8}, {64, 1, 5, 8},
                                  {1000, 1, 13, 3}, {1920, 1080, 4, 8}, {1920, 1080, 64, 8}, {1920, 17, 9, 8},
                                  {128, 1, 64, 8}, {64, 7, 3, 5}, {45, 26, 6, 8}, {48, 37, 3, 8}, {96, 54, 4, 8}};
    for (const auto &sh : shapes)
        for (unsigned ts : {6u, 3u, 4u, 5u}) {
            const int e = check_table(sh[0], sh[1], sh[2], sh[3], ts);
            if (e) {
                std::printf("FAIL width %u rows %u frames %u queues %u tile shift %u: %d\n", sh[0], sh[1], sh[2],
                            sh[3], ts, e);
                return 1;
            }
        }
    std::printf("ok\n");
    return 0;
}
