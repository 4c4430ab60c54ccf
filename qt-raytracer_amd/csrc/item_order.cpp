// item_order.cpp — the order in which the megakernel's queues hand out a band's pixels.
//
// A wave's lanes advance in lock-step rounds and take new samples as theirs end, so a wave whose
// lanes hold samples of very different lengths (a sky pixel ends after one segment, a pixel deep
// in the box after up to maxDepth) runs its rounds with idle lanes.  The queues therefore hand out
// runs of 64 band pixels (a wave's camera-ray pool: neighbours, so the primary segment stays
// coherent) in order of an estimated sample length, longest first: a wave's lanes mostly hold
// samples of one kind, and the launch ends on the cheap ones.  The estimate comes from the host's
// copy of the tree: per run, 4 camera rays through pixel centres, and from each hit 8 fixed
// hemisphere directions, whose fraction e that escapes to the sky gives a Lambertian path's
// expected length ~1/e.  The order changes which lane traces a sample, never what it computes.
#include "item_order.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <utility>

namespace hippt {
namespace {

struct D3 {
    double x, y, z;
};
D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 mul(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 unit(D3 a) {
    const double l = std::sqrt(dot(a, a));
    return l > 0 ? mul(a, 1.0 / l) : D3{0, 0, 1};
}

constexpr double kTmin = 1e-3;

// t of the primitive record along the ray (INFINITY on a miss).
double prim_t(const float *rec, D3 o, D3 d) {
    uint32_t tag;
    std::memcpy(&tag, rec + 10, sizeof tag);
    if (tag != 0u) {  // sphere: (centre, r)
        const D3 oc = sub(o, D3{rec[0], rec[1], rec[2]});
        const double a = dot(d, d), hb = dot(oc, d), c = dot(oc, oc) - double(rec[3]) * rec[3];
        const double disc = hb * hb - a * c;
        if (disc < 0.0) return INFINITY;
        const double sq = std::sqrt(disc);
        const double t0 = (-hb - sq) / a, t1 = (-hb + sq) / a;
        return t0 > kTmin ? t0 : t1 > kTmin ? t1 : INFINITY;
    }
    const D3 v0{rec[0], rec[1], rec[2]}, e1{rec[3], rec[4], rec[5]}, e2{rec[6], rec[7], rec[8]};
    const D3 pv = cross(d, e2);
    const double det = dot(e1, pv);
    if (det == 0.0) return INFINITY;
    const D3 tv = sub(o, v0);
    const double u = dot(tv, pv) / det;
    const D3 qv = cross(tv, e1);
    const double v = dot(d, qv) / det;
    const double t = dot(e2, qv) / det;
    return u >= 0.0 && v >= 0.0 && u + v <= 1.0 && t > kTmin ? t : INFINITY;
}

// Closest hit along the ray over the 4-wide tree: t (INFINITY on a miss) and the primitive slot.
// An estimate for the order only: no result depends on it.
double closest(const Bvh4 &b, const float *tris, D3 o, D3 d, int &prim) {
    prim = -1;
    double best = INFINITY;
    if (b.nodes.empty()) return best;
    const double oa[3] = {o.x, o.y, o.z}, ia[3] = {1.0 / d.x, 1.0 / d.y, 1.0 / d.z};
    int stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const uint32_t *w = &b.nodes[size_t(stack[--sp]) * kNode4Words];
        float f[24];
        std::memcpy(f, w, sizeof f);
        for (int i = 0; i < 4; ++i) {
            double tn = kTmin, tf = best;
            const double lo[3] = {f[i], f[8 + i], f[16 + i]}, hi[3] = {f[4 + i], f[12 + i], f[20 + i]};
            for (int a = 0; a < 3; ++a) {
                double t0 = (lo[a] - oa[a]) * ia[a], t1 = (hi[a] - oa[a]) * ia[a];
                if (t0 > t1) std::swap(t0, t1);
                tn = std::fmax(tn, t0);
                tf = std::fmin(tf, t1);
            }
            if (!(tn <= tf)) continue;
            const int32_t c = int32_t(w[24 + i]);
            if (c >= 0) {
                if (sp < 256) stack[sp++] = c;
                continue;
            }
            const int first = (~c) >> 4, count = (~c) & 15;
            for (int k = first; k < first + count; ++k) {
                const double t = prim_t(tris + 12 * size_t(k), o, d);
                if (t < best) {
                    best = t;
                    prim = k;
                }
            }
        }
    }
    return best;
}

// Estimated segments of a sample along camera direction d: 1 on a miss; else 1 + the expected
// Lambertian bounces until a ray escapes, 1/e for an escape fraction e over 8 fixed hemisphere
// directions around the hit's normal, capped at maxDepth - 1.
double sample_cost(const Bvh4 &b, const float *tris, D3 o, D3 d, int maxDepth) {
    int prim;
    const double t = closest(b, tris, o, d, prim);
    if (prim < 0) return 1.0;
    const float *rec = tris + 12 * size_t(prim);
    const D3 p = add(o, mul(d, t));
    uint32_t tag;
    std::memcpy(&tag, rec + 10, sizeof tag);
    D3 n = tag ? unit(sub(p, D3{rec[0], rec[1], rec[2]}))
               : unit(cross(D3{rec[3], rec[4], rec[5]}, D3{rec[6], rec[7], rec[8]}));
    if (dot(n, d) > 0) n = mul(n, -1.0);
    // an orthonormal frame around n and 8 directions at 30 and 60 degrees from it
    const D3 a = std::fabs(n.x) < 0.9 ? D3{1, 0, 0} : D3{0, 1, 0};
    const D3 u = unit(cross(n, a)), v = cross(n, u);
    const D3 start = add(p, mul(n, 1e-3 * (1.0 + std::sqrt(dot(p, p)))));
    int escaped = 0;
    for (int j = 0; j < 8; ++j) {
        const double phi = 0.785398163397 * j, th = (j & 1) ? 1.0471975512 : 0.523598775598;
        const D3 dir = add(mul(n, std::cos(th)),
                           add(mul(u, std::sin(th) * std::cos(phi)), mul(v, std::sin(th) * std::sin(phi))));
        int q;
        if (!std::isfinite(closest(b, tris, start, dir, q))) ++escaped;
    }
    const double bounces = escaped ? 8.0 / escaped : double(maxDepth);
    return 1.0 + std::min(bounces, double(maxDepth - 1));
}

}  // namespace

unsigned tile_shift_for(unsigned width, unsigned tileShift) {
    if (tileShift >= 6) return 6;
    return width % (1u << tileShift) == 0 ? tileShift : 6;
}

size_t run_count(const RunLayout &L) { return size_t(L.rows) * size_t(L.width) / 64; }

uint32_t run_base(const RunLayout &L, size_t r) {
    if (L.tileShift >= 6) return uint32_t(64 * r);
    const size_t tw = size_t(1) << L.tileShift, th = 64 / tw;
    const size_t perStrip = L.width / tw, tileRuns = (L.rows / th) * perStrip;
    if (r < tileRuns) return uint32_t(((r / perStrip) * th * L.width + (r % perStrip) * tw)) | kRunTile;
    return uint32_t(tileRuns * 64 + 64 * (r - tileRuns));
}

uint32_t run_pixel(const RunLayout &L, size_t r, unsigned k) {
    const uint32_t b = run_base(L, r);
    if (!(b & kRunTile)) return b + k;
    return (b & ~kRunTile) + (k & ((1u << L.tileShift) - 1u)) + (k >> L.tileShift) * L.width;
}

void run_costs(const Bvh4 &bvh, const float *tris, const CameraF &cam, const RunLayout &L, int height, int y0,
               int stride, int maxDepth, std::vector<float> &cost, int threads) {
    cost.clear();
    const int width = int(L.width);
    if (width <= 0 || L.rows <= 0) return;
    const size_t runs = run_count(L);
    const double sw = double(std::max(1, width - 1)), sh = double(std::max(1, height - 1));
    const D3 O{cam.origin[0], cam.origin[1], cam.origin[2]};
    cost.assign(runs, 0.0f);
    auto span = [&](size_t r0, size_t r1) {
        for (size_t r = r0; r < r1; ++r) {
            double c = 0.0;
            for (int j = 0; j < 4; ++j) {
                const size_t p = run_pixel(L, r, unsigned(21 * j));  // the run's items 0, 21, 42, 63
                const double x = double(p % size_t(width)) + 0.5;
                const double y = double(y0 + int(p / size_t(width)) * stride) + 0.5;
                const double s = x / sw, t = y / sh;
                const D3 d{cam.llc[0] + s * cam.horizontal[0] + t * cam.vertical[0] - O.x,
                           cam.llc[1] + s * cam.horizontal[1] + t * cam.vertical[1] - O.y,
                           cam.llc[2] + s * cam.horizontal[2] + t * cam.vertical[2] - O.z};
                c += sample_cost(bvh, tris, O, d, std::max(1, maxDepth));
            }
            cost[r] = float(c / 4.0);
        }
    };
    // each run's estimate is independent of the others: contiguous spans per thread (same values
    // for any thread count)
    const size_t nt = std::min<size_t>(size_t(std::max(1, threads)), std::max<size_t>(1, runs / 256));
    if (nt <= 1) {
        span(0, runs);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    size_t k = 1;
    try {
        for (; k < nt; ++k) pool.emplace_back(span, runs * k / nt, runs * (k + 1) / nt);
    } catch (...) {  // no more threads: the rest here (joinable threads must not be destroyed)
        for (; k < nt; ++k) span(runs * k / nt, runs * (k + 1) / nt);
    }
    span(0, runs / nt);
    for (auto &t : pool) t.join();
}

void build_item_table(const std::vector<float> &cost, const RunLayout &L, unsigned frames, unsigned queues,
                      std::vector<uint32_t> &table) {
    const size_t runs = cost.size(), slots = runs * frames;
    table.assign(slots, 0u);
    if (!slots) return;
    const unsigned bandPixels = L.width * L.rows;
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    // slot s: queue position pos(s) (which queue hands it out), items from item(s)
    auto pos = [&](size_t s) { return (unsigned long long)(s / runs) * bandPixels + 64 * (s % runs); };
    auto item = [&](size_t s) { return uint32_t((s / runs) * bandPixels) + run_base(L, s % runs); };
    // A stable sort of each queue's slots (s = f*runs + r, ascending) by cost[r], longest first, in
    // O(slots): the runs by (cost descending, r ascending) once; a queue then takes each group of
    // equal-cost runs frame by frame (ascending slot order within a group is frame-major).
    std::vector<uint32_t> ranked(runs);
    for (size_t r = 0; r < runs; ++r) ranked[r] = uint32_t(r);
    std::stable_sort(ranked.begin(), ranked.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    std::vector<size_t> group{0};  // group k: ranked[group[k] .. group[k+1])
    for (size_t k = 1; k < runs; ++k)
        if (cost[ranked[k]] != cost[ranked[k - 1]]) group.push_back(k);
    group.push_back(runs);
    size_t s0 = 0;
    for (unsigned g = 0; g < queues && s0 < slots; ++g) {
        const unsigned long long end = total * (g + 1) / queues;
        size_t s1 = s0;
        while (s1 < slots && pos(s1) < end) ++s1;  // the queue's slots [s0, s1)
        if (s1 == s0) continue;
        const size_t f0 = s0 / runs, f1 = (s1 - 1) / runs;
        size_t out = s0;
#ifdef HIPPT_EXP_ORDER_CYCLES
        // experiment: the queue's frames in HIPPT_EXP_ORDER_CYCLES consecutive parts, each walked
        // longest first on its own (a big batch ordered like a chain of small ones)
        const size_t parts = HIPPT_EXP_ORDER_CYCLES, nf = f1 - f0 + 1;
        for (size_t c = 0; c < parts; ++c) {
            const size_t fa = f0 + nf * c / parts, fb = f0 + nf * (c + 1) / parts;
            for (size_t k = 0; k + 1 < group.size(); ++k)
                for (size_t f = fa; f < fb; ++f)
                    for (size_t q = group[k]; q < group[k + 1]; ++q) {
                        const size_t sl = f * runs + ranked[q];
                        if (sl >= s0 && sl < s1) table[out++] = item(sl);
                    }
        }
#else
        for (size_t k = 0; k + 1 < group.size(); ++k)
            for (size_t f = f0; f <= f1; ++f)
                for (size_t q = group[k]; q < group[k + 1]; ++q) {
                    const size_t sl = f * runs + ranked[q];
                    if (sl >= s0 && sl < s1) table[out++] = item(sl);
                }
#endif
        s0 = s1;
    }
    for (; s0 < slots; ++s0) table[s0] = item(s0);
}

}  // namespace hippt
