// item_order_check.cpp — host checks of the queues' item table (qt-raytracer_amd/csrc/item_order.cpp),
// built and run by tests/test_item_order.py: the table is a permutation of the batch's run slots
// for any band size, frame count and queue count; within a queue, the estimates never increase;
// the Cornell box's sky runs cost 1.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "item_order.h"

using namespace hippt;

static int check_table(unsigned bandPixels, unsigned frames, unsigned queues) {
    const size_t runs = bandPixels / 64;
    std::vector<float> cost(runs);
    for (size_t r = 0; r < runs; ++r) cost[r] = float((r * 7919) % 13) * 0.5f + 1.0f;
    std::vector<uint32_t> t;
    build_item_table(cost, bandPixels, frames, queues, t);
    if (t.size() != runs * frames) return 1;
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
                                  {1000, 13, 3}, {1920 * 1080, 4, 8}};
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
