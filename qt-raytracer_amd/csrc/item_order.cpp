// item_order.cpp — the order in which the megakernel's queues hand out a band's pixels.
//
// The persistent grid takes its work in chunks from per-XCD queues; once the queues are empty a
// wave still finishes what it holds (its claimed chunk, its camera-ray pool, its paths in
// flight), and the launch ends with the slowest such wave.  In image order the last items of a
// queue are whatever the last rows show: on Cornell the box interior, whose samples take ~6
// segments at ~25 us per round while sky samples take one.  Handing out the runs that hit the
// scene first and the sky runs last makes the work left at the drain cheap.  Runs of 64 band
// pixels keep a wave's camera rays neighbours (the coherence of the primary segment).
#include "item_order.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <utility>

namespace hippt {
namespace {

struct D3 {
    double x, y, z;
};
D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

constexpr double kTmin = 1e-3;

bool prim_hit(const float *rec, D3 o, D3 d) {
    uint32_t tag;
    std::memcpy(&tag, rec + 10, sizeof tag);
    if (tag != 0u) {  // sphere: (centre, r)
        const D3 oc = sub(o, D3{rec[0], rec[1], rec[2]});
        const double a = dot(d, d), hb = dot(oc, d), c = dot(oc, oc) - double(rec[3]) * rec[3];
        const double disc = hb * hb - a * c;
        if (disc < 0.0) return false;
        const double sq = std::sqrt(disc);
        return (-hb - sq) / a > kTmin || (-hb + sq) / a > kTmin;
    }
    const D3 v0{rec[0], rec[1], rec[2]}, e1{rec[3], rec[4], rec[5]}, e2{rec[6], rec[7], rec[8]};
    const D3 pv = cross(d, e2);
    const double det = dot(e1, pv);
    if (det == 0.0) return false;
    const D3 tv = sub(o, v0);
    const double u = dot(tv, pv) / det;
    const D3 qv = cross(tv, e1);
    const double v = dot(d, qv) / det;
    return u >= 0.0 && v >= 0.0 && u + v <= 1.0 && dot(e2, qv) / det > kTmin;
}

// Any hit along the ray (an estimate for the order only: no result depends on it).
bool any_hit(const Bvh4 &b, const float *tris, D3 o, D3 d) {
    if (b.nodes.empty()) return false;
    const D3 inv{1.0 / d.x, 1.0 / d.y, 1.0 / d.z};
    int stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const uint32_t *w = &b.nodes[size_t(stack[--sp]) * kNode4Words];
        float f[24];
        std::memcpy(f, w, sizeof f);
        for (int i = 0; i < 4; ++i) {
            double tn = kTmin, tf = INFINITY;
            const double lo[3] = {f[i], f[8 + i], f[16 + i]}, hi[3] = {f[4 + i], f[12 + i], f[20 + i]};
            const double oa[3] = {o.x, o.y, o.z}, ia[3] = {inv.x, inv.y, inv.z};
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
            for (int k = first; k < first + count; ++k)
                if (prim_hit(tris + 12 * size_t(k), o, d)) return true;
        }
    }
    return false;
}

}  // namespace

size_t build_run_order(const Bvh4 &bvh, const float *tris, const CameraF &cam, int width, int height, int y0, int rows,
                       int stride, std::vector<uint32_t> &order) {
    order.clear();
    if (width <= 0 || rows <= 0) return 0;
    const size_t runs = size_t(rows) * size_t(width) / 64;
    const double sw = double(std::max(1, width - 1)), sh = double(std::max(1, height - 1));
    const D3 O{cam.origin[0], cam.origin[1], cam.origin[2]};
    std::vector<uint32_t> sky;
    order.reserve(runs);
    for (size_t r = 0; r < runs; ++r) {
        bool hit = false;
        for (int j = 0; j < 4 && !hit; ++j) {
            const size_t p = 64 * r + size_t(21 * j);  // band pixels 0, 21, 42, 63 of the run
            const double x = double(p % size_t(width)) + 0.5;
            const double y = double(y0 + int(p / size_t(width)) * stride) + 0.5;
            const double s = x / sw, t = y / sh;
            const D3 d{cam.llc[0] + s * cam.horizontal[0] + t * cam.vertical[0] - O.x,
                       cam.llc[1] + s * cam.horizontal[1] + t * cam.vertical[1] - O.y,
                       cam.llc[2] + s * cam.horizontal[2] + t * cam.vertical[2] - O.z};
            hit = any_hit(bvh, tris, O, d);
        }
        (hit ? order : sky).push_back(uint32_t(r));
    }
    const size_t hits = order.size();
    order.insert(order.end(), sky.begin(), sky.end());
    return hits;
}

void build_item_table(const std::vector<uint32_t> &order, size_t hitRuns, unsigned bandPixels, unsigned frames,
                      unsigned queues, std::vector<uint32_t> &table) {
    const size_t runs = order.size(), slots = runs * frames;
    table.assign(slots, 0u);
    if (!slots) return;
    std::vector<uint8_t> hit(runs, 0);
    for (size_t j = 0; j < hitRuns; ++j) hit[order[j]] = 1;
    const unsigned long long total = (unsigned long long)bandPixels * frames;
    auto item = [&](size_t s) { return uint32_t((s / runs) * bandPixels + 64 * (s % runs)); };
    // slots by queue (the queue holding a slot's first item), in order
    size_t s = 0;
    std::vector<size_t> pos, hitSlots, skySlots;
    for (unsigned g = 0; g < queues && s < slots; ++g) {
        const unsigned long long end = total * (g + 1) / queues;
        pos.clear();
        hitSlots.clear();
        skySlots.clear();
        for (; s < slots && item(s) < end; ++s) {
            pos.push_back(s);
            (hit[s % runs] ? hitSlots : skySlots).push_back(s);
        }
        size_t k = 0;
        for (size_t h : hitSlots) table[pos[k++]] = item(h);
        for (size_t h : skySlots) table[pos[k++]] = item(h);
    }
    for (; s < slots; ++s) table[s] = item(s);
}

}  // namespace hippt
