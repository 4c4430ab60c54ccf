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
// round-3 implementation; build_item_table must give the same table in O(slots)).
static void reference_table(const std::vector<float> &cost, unsigned bandPixels, unsigned frames, unsigned queues,
                            std::vector<uint32_t> &table) {
    const size_t runs = cost.size(), slots = runs * frames;
    table.assign(slots, 0u);
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    auto item = [&](size_t s) { return uint32_t((s / runs) * bandPixels + 64 * (s % runs)); };
    size_t s = 0;
    std::vector<size_t> pos, sorted;
    for (unsigned g = 0; g < queues && s < slots; ++g) {
        const unsigned long long end = total * (g + 1) / queues;
        pos.clear();
        for (; s < slots && item(s) < end; ++s) pos.push_back(s);
        sorted = pos;
        std::stable_sort(sorted.begin(), sorted.end(), [&](size_t a, size_t b) { return cost[a % runs] > cost[b % runs]; });
        for (size_t k = 0; k < pos.size(); ++k) table[pos[k]] = item(sorted[k]);
    }
    for (; s < slots; ++s) table[s] = item(s);
}

static int check_table(unsigned bandPixels, unsigned frames, unsigned queues) {
    const size_t runs = bandPixels / 64;
    std::vector<float> cost(runs);
    for (size_t r = 0; r < runs; ++r) cost[r] = float((r * 7919) % 13) * 0.5f + 1.0f;
    std::vector<uint32_t> t, ref;
    build_item_table(cost, bandPixels, frames, queues, t);
    if (t.size() != runs * frames) return 1;
    reference_table(cost, bandPixels, frames, queues, ref);
    if (t != ref) return 4;
    std::vector<uint32_t> s = t;
    std::sort(s.begin(), s.end());
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i] != uint32_t((i / runs) * bandPixels + 64 * (i % runs))) return 2;
    // within each queue range the estimates of the handed-out runs never increase
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    for (unsigned g = 0; g < queues; ++g) {
        const unsigned long long lo = total * g / queues, hi = total * (g + 1) / queues;
        float prev = 1e30f;
        for (size_t k = 0; k < t.size(); ++k) {
            const unsigned long long pos = (k / runs) * bandPixels + 64 * (k % runs);
            if (pos < lo || pos >= hi) continue;
            const float c = cost[(t[k] % bandPixels) / 64];
            if (c > prev) return 3;
            prev = c;
        }
    }
    return 0;
}

int main() {
    const unsigned shapes[][3] = {{640, 1, 8}, {640, 3, 8}, {650, 7, 8}, {1920 * 135, 64, 8}, {64, 5, 8},
                                  {1000, 13, 3}, {1920 * 1080, 4, 8}, {1920 * 1080, 64, 8}, {1920 * 17, 9, 8},
                                  {128, 64, 8}, {64 * 7, 3, 5}};
    for (const auto &sh : shapes) {
        const int e = check_table(sh[0], sh[1], sh[2]);
        if (e) {
            std::printf("FAIL bandPixels %u frames %u queues %u: %d\n", sh[0], sh[1], sh[2], e);
            return 1;
        }
    }
    std::printf("ok\n");
    return 0;
}
