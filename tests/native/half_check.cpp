// Host check of bvh_builder.cpp's half-precision planes (half_bvh4): the directed roundings against
// an exhaustive table of the 63,488 finite halves, and the node layout.  Prints "ok".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "bvh_builder.h"

using hippt::half_round_down;
using hippt::half_round_up;
using hippt::half_value;

static int fails = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c) && fails++ < 20) {                    \
            std::printf("FAIL %s: ", #c);              \
            std::printf(__VA_ARGS__);                  \
            std::printf("\n");                         \
        }                                              \
    } while (0)

int main() {
    // every half value in increasing order (-inf .. +inf, one zero)
    std::vector<float> vals;
    for (int h = 0xFC00; h > 0x8000; --h) vals.push_back(half_value(uint16_t(h)));
    for (int h = 0; h <= 0x7C00; ++h) vals.push_back(half_value(uint16_t(h)));
    for (size_t i = 1; i < vals.size(); ++i) CHECK(vals[i - 1] < vals[i], "order at %zu", i);
    auto check = [&](float x) {
        const float d = half_value(half_round_down(x)), u = half_value(half_round_up(x));
        // d = the largest half <= x, u = the smallest half >= x
        const auto it = std::upper_bound(vals.begin(), vals.end(), x);
        const float want_d = it == vals.begin() ? -INFINITY : *(it - 1);
        const auto jt = std::lower_bound(vals.begin(), vals.end(), x);
        const float want_u = jt == vals.end() ? INFINITY : *jt;
        CHECK(d == want_d && u == want_u, "x=%.9g down %.9g (want %.9g) up %.9g (want %.9g)", x, d, want_d, u,
              want_u);
    };
    for (float v : vals) {  // the halves themselves and their float neighbours
        check(v);
        check(std::nextafter(v, -INFINITY));
        check(std::nextafter(v, INFINITY));
    }
    std::mt19937 g(7);
    std::uniform_int_distribution<uint32_t> bits;
    for (int i = 0; i < 2000000; ++i) {
        uint32_t b = bits(g);
        float x;
        std::memcpy(&x, &b, 4);
        if (!std::isnan(x)) check(x);
    }
    check(3.4e38f);
    check(-3.4e38f);
    check(65504.0f);
    check(65519.99f);
    check(-65520.0f);
    check(1e-30f);
    check(-1e-30f);

    // layout: a node of distinct planes and codes
    std::vector<uint32_t> in(hippt::kNode4Words * 2, 0u);
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 4; ++i) {
                const float lo = 100.0f * k + 10.0f * a + i + 0.3f, hi = lo + 1.7f;
                std::memcpy(&in[k * 32 + 8 * a + i], &lo, 4);
                std::memcpy(&in[k * 32 + 8 * a + 4 + i], &hi, 4);
                in[k * 32 + 24 + i] = uint32_t(k * 1000 + i - 2);
            }
    std::vector<uint32_t> out;
    CHECK(hippt::half_bvh4(in.data(), 2, out), "in range");
    CHECK(out.size() == in.size(), "size");
    for (int k = 0; k < 2; ++k) {
        const unsigned char *n = reinterpret_cast<const unsigned char *>(out.data() + k * 32);
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 4; ++i) {
                float lo, hi;
                std::memcpy(&lo, &in[k * 32 + 8 * a + i], 4);
                std::memcpy(&hi, &in[k * 32 + 8 * a + 4 + i], 4);
                uint16_t h[16];
                std::memcpy(h, n + 32 * a, 32);
                // positive direction: the row at 32a = near (lo) halves then far (hi) halves;
                // negative: the row at 32a + 16 = near (hi) then far (lo)
                CHECK(half_value(h[i]) <= lo && half_value(h[i]) > lo - 0.25f, "lo");
                CHECK(half_value(h[4 + i]) >= hi && half_value(h[4 + i]) < hi + 0.25f, "hi");
                CHECK(h[8 + i] == h[4 + i] && h[12 + i] == h[i], "negative row");
            }
        uint32_t codes[4];
        std::memcpy(codes, n + 96, 16);
        for (int i = 0; i < 4; ++i) CHECK(codes[i] == uint32_t(k * 1000 + i - 2), "code");
        for (int b = 112; b < 128; ++b) CHECK(n[b] == 0, "pad");
    }
    // empty slots (lo = +inf, hi = -inf) stay infinite; a finite plane beyond the half range means no
    // half tree (it would become an infinite box)
    {
        std::vector<uint32_t> e = in, o;
        const float pinf = INFINITY, ninf = -INFINITY;
        for (int a = 0; a < 3; ++a) {
            std::memcpy(&e[8 * a + 3], &pinf, 4);
            std::memcpy(&e[8 * a + 4 + 3], &ninf, 4);
        }
        CHECK(hippt::half_bvh4(e.data(), 2, o) && o.size() == e.size(), "empty slots");
        const uint16_t *h = reinterpret_cast<const uint16_t *>(o.data());
        CHECK(h[3] == 0x7C00u && h[7] == 0xFC00u, "empty slot planes");
        for (float bad : {70000.0f, -70000.0f}) {
            std::vector<uint32_t> f = in;
            std::memcpy(&f[32 + 8 * 2 + (bad > 0 ? 4 : 0) + 1], &bad, 4);  // node 1, axis z, child 1
            CHECK(!hippt::half_bvh4(f.data(), 2, o) && o.empty(), "beyond the half range");
        }
        const float edge = 65504.0f, nedge = -65504.0f;
        std::vector<uint32_t> g = in;
        std::memcpy(&g[4], &edge, 4);
        std::memcpy(&g[0], &nedge, 4);
        CHECK(hippt::half_bvh4(g.data(), 2, o), "the largest half itself");
    }
    if (fails) return 1;
    std::printf("ok\n");
    return 0;
}
