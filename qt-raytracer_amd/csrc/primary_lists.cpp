// primary_lists.cpp — per-pixel candidate lists for primary rays of a pinhole camera.
//
// A camera ray of pixel (x, y) (RenderWorker::render's u/v, RayTracerFboItem.cpp:109-110, and
// Camera::get_ray with a zero lens radius, RayTracer.h:563-567) starts at the camera origin O and
// has the direction d(X, Y) = (llc - O) + X/(W-1) * horizontal + Y/(H-1) * vertical for some
// (X, Y) in the pixel's footprint [x, x+1] x [y, y+1], whatever the jitter.  The closest hit is
// the argmin (t, primitive id) over every primitive the FP32 Möller–Trumbore test reports as hit
// (the oracle's brute force, pt_oracle.c scene_closest; the BVH traversals return the same).  So a
// list per pixel that holds every primitive whose FP32 test can pass for some ray through the
// pixel gives the same closest hit: extra primitives cannot change an argmin they do not win, and
// the kernel tests the list with the same arithmetic (hippt_trace.h primary_hit).
//
// Which primitives can pass.  The test's three edge values un = dot(d, e2 x tv), vn =
// dot(d, tv x e1) and det - un - vn (tv = O - v0, det = dot(d, e2 x e1)) are linear in d, hence
// affine in (X, Y): their zero lines are the projected triangle's edges.  Their FP32 values are
// within E of the exact ones: C eps |a||b||d| for the test's own roundings (two for the cross
// product, three for fdot, one for tv: ~7.5, C = 16) plus the FP32 direction's distance from the
// exact d(X, Y) (dominated by the fmaf results ~llc when the camera is far from the world origin:
// ~0.02 pixel for the headline scenes).  When the camera
// origin is off the triangle's plane by more than the error of t's numerator (|h| > 2 E_t) and the
// vertices are in front of the camera, every FP32 hit with t >= 0 has det of the cone's sign s, so
// the three values satisfy s*g >= -E: the pixel's footprint must meet the triangle whose edges are
// pushed out by E/|grad g|.  Otherwise (a vertex at or behind the camera plane, the origin near the
// plane, triangles degenerate in FP64 but not in FP32 such as the blob's poles) a pass still needs
// |un|, |vn|, |det - un - vn| <= |det|: three strips around the projected edge lines.  Non-finite
// values make the primitive a candidate of every pixel.  The pixel test uses the footprint widened
// by 1/32 pixel on top, for the rounding of X/(W-1) (~4e-4 pixel).
#include "primary_lists.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace hippt {
namespace {

struct V3 {
    double x, y, z;
};
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
double norm(V3 a) { return std::sqrt(dot(a, a)); }

struct Affine {  // g(X, Y) = a + b X + c Y over pixel coordinates
    double a, b, c;
};

constexpr double kMarginPx = 1.0 / 32.0;
constexpr double kEps = 1.0 / 16777216.0;  // 2^-24: FP32 round to nearest
constexpr double kC = 16.0;  // the test's own roundings: ~7.5 eps |a||b||d|, taken twice

}  // namespace

bool build_primary_lists(const float *tris, int numSlots, const CameraF &cam, int width, int height, int y0, int rows,
                         int stride, std::vector<uint32_t> &offsets, std::vector<uint32_t> &ids) {
    offsets.clear();
    ids.clear();
    if (cam.lens_radius != 0.0f || width <= 0 || height <= 0 || rows < 0 || stride < 1) return false;
    for (int k = 0; k < numSlots; ++k) {
        uint32_t tag;
        std::memcpy(&tag, tris + 12 * size_t(k) + 10, sizeof tag);
        if (tag != 0u) return false;  // a sphere (type tag): not handled here
    }
    const V3 O{cam.origin[0], cam.origin[1], cam.origin[2]};
    const V3 hor{cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]};
    const V3 ver{cam.vertical[0], cam.vertical[1], cam.vertical[2]};
    const V3 w = sub(V3{cam.llc[0], cam.llc[1], cam.llc[2]}, O);
    const double sw = double(std::max(1, width - 1)), sh = double(std::max(1, height - 1));
    // |d| over the image (its corners, widened) and the bound of the direction's own rounding
    double dmax = 0.0;
    for (double X : {-1.0, double(width) + 1.0})
        for (double Y : {-1.0, double(height) + 1.0}) {
            const V3 d{w.x + X / sw * hor.x + Y / sh * ver.x, w.y + X / sw * hor.y + Y / sh * ver.y,
                       w.z + X / sw * hor.z + Y / sh * ver.z};
            dmax = std::max(dmax, norm(d));
        }
    // per component, the FP32 direction's distance from the exact d(X, Y) of its pixel point: the
    // roundings of s and t (3 eps each, times horizontal / vertical), of the two fmaf (their
    // results are ~llc) and of the origin's subtraction (~d), taken twice
    double dErr[3];
    const float *llcF = cam.llc, *horF = cam.horizontal, *verF = cam.vertical;
    for (int i = 0; i < 3; ++i)
        dErr[i] = 2.0 * kEps *
                  (2.0 * std::fabs(double(llcF[i])) + 5.0 * std::fabs(double(horF[i])) +
                   2.0 * std::fabs(double(verF[i])) + dmax);
    auto dirErr = [&](const V3 &n) { return dErr[0] * std::fabs(n.x) + dErr[1] * std::fabs(n.y) + dErr[2] * std::fabs(n.z); };
    // the image-plane depth of a point: its coefficient along w in the basis (hor, ver, w)
    const V3 depthN = cross(hor, ver);
    const double depthW = dot(w, depthN);
    if (!std::isfinite(dmax) || !(std::fabs(depthW) > 0.0)) return false;

    const size_t pixels = size_t(rows) * size_t(width);
    std::vector<uint32_t> count(pixels + 1, 0u);
    auto visit = [&](int k, auto &&emit) {
        const float *t = tris + 12 * size_t(k);  // (v0, e1.x) (e1.yz, e2.xy) (e2.z, id, tag, -)
        const V3 v0{t[0], t[1], t[2]}, e1{t[3], t[4], t[5]}, e2{t[6], t[7], t[8]};
        if (e1.x == 0 && e1.y == 0 && e1.z == 0 && e2.x == 0 && e2.y == 0 && e2.z == 0) return;  // det = 0
        const V3 tv = sub(O, v0);
        const V3 nu = cross(e2, tv), nv = cross(tv, e1), nd = cross(e2, e1);
        const double h = -dot(tv, nd);  // dot(v0 - O, e2 x e1): det's sign inside the cone
        const double l1 = norm(e1), l2 = norm(e2), lt = norm(tv);
        const double Et = kC * kEps * l1 * l2 * lt;
        const double Eu = kC * kEps * lt * l2 * dmax + dirErr(nu), Ev = kC * kEps * lt * l1 * dmax + dirErr(nv);
        const double Ed = kC * kEps * l1 * l2 * dmax + dirErr(nd), Ew = 2.0 * (Eu + Ev + Ed);
        // un, vn, det and det - un - vn as affine functions of the pixel coordinates
        const V3 nrm[3] = {nu, nv, nd};
        Affine raw[4];
        for (int e = 0; e < 3; ++e) raw[e] = {dot(w, nrm[e]), dot(hor, nrm[e]) / sw, dot(ver, nrm[e]) / sh};
        raw[3] = {raw[2].a - raw[0].a - raw[1].a, raw[2].b - raw[0].b - raw[1].b, raw[2].c - raw[0].c - raw[1].c};
        bool finite = std::isfinite(h) && std::isfinite(Ew);
        for (const Affine &f : raw) finite = finite && std::isfinite(f.a) && std::isfinite(f.b) && std::isfinite(f.c);
        if (!finite) {
            for (size_t p = 0; p < pixels; ++p) emit(p, uint32_t(k));
            return;
        }
        bool signedCase = std::fabs(h) > 2.0 * Et;
        for (int i = 0; i < 3 && signedCase; ++i) {  // every vertex strictly in front of the camera plane
            const V3 v = i == 0 ? v0 : i == 1 ? V3{v0.x + e1.x, v0.y + e1.y, v0.z + e1.z}
                                              : V3{v0.x + e2.x, v0.y + e2.y, v0.z + e2.z};
            const double depth = dot(sub(v, O), depthN) / depthW;
            signedCase = depth > 1e-9 * norm(sub(v, O)) / std::max(1e-300, norm(w));
        }
        // Constraints "g >= 0 somewhere in the pixel's widened footprint".  Signed case: the three
        // edge values with det's sign s, pushed out by their errors.  Otherwise (a vertex at or
        // behind the camera plane, the origin near the plane, a triangle degenerate in FP64): any
        // FP32 pass has |un|, |vn|, |det - un - vn| <= |det| (us, vs >= 0 and us + vs <= |det|),
        // so each lies within |exact det| + errors of zero: three strips, bounded per row by the
        // row's largest |det|.
        const double sg = h > 0 ? 1.0 : -1.0;
        const Affine g[3] = {{sg * raw[0].a + Eu, sg * raw[0].b, sg * raw[0].c},
                             {sg * raw[1].a + Ev, sg * raw[1].b, sg * raw[1].c},
                             {sg * raw[3].a + Ew, sg * raw[3].b, sg * raw[3].c}};
        double ylo = -1.0, yhi = double(height);
        if (signedCase) {  // rows: the relaxed triangle's vertices (pairwise intersections of its edges)
            bool bounded = true;
            double vyMin = INFINITY, vyMax = -INFINITY;
            for (int e = 0; e < 3 && bounded; ++e) {
                const Affine &A = g[e], &B = g[(e + 1) % 3], &Cc = g[(e + 2) % 3];
                const double det2 = A.b * B.c - A.c * B.b;
                const double scale = std::max(std::fabs(A.b * B.c), std::fabs(A.c * B.b));
                if (!(std::fabs(det2) > 1e-9 * scale)) {
                    bounded = false;
                    break;
                }
                const double X = (-A.a * B.c + A.c * B.a) / det2, Y = (-A.b * B.a + A.a * B.b) / det2;
                // a vertex of a bounded region satisfies the third constraint
                if (!std::isfinite(X) || !std::isfinite(Y) ||
                    Cc.a + Cc.b * X + Cc.c * Y < -1e-9 * (1.0 + std::fabs(Cc.a)))
                    bounded = false;
                vyMin = std::min(vyMin, Y);
                vyMax = std::max(vyMax, Y);
            }
            if (bounded) {
                ylo = std::max(ylo, vyMin);
                yhi = std::min(yhi, vyMax);
            }
        }
        // band rows whose widened footprint [y - m, y + 1 + m] meets [ylo, yhi]
        const double ya = std::floor(ylo - 1.0 - kMarginPx), yb = std::ceil(yhi + kMarginPx);
        if (ya > double(height) || yb < 0.0) return;
        const long long yA = ya < 0.0 ? 0LL : (long long)ya, yB = yb > double(height - 1) ? height - 1LL : (long long)yb;
        if (yB < y0) return;
        const long long ky0 = std::max(0LL, (yA - y0 + stride - 1) / stride);
        const long long ky1 = std::min((long long)rows - 1, (yB - y0) / stride);
        for (long long ky = ky0; ky <= ky1; ++ky) {
            const double yl = double(y0 + ky * stride) - kMarginPx, yh = double(y0 + ky * stride) + 1.0 + kMarginPx;
            Affine cs[6];
            int n = 0;
            if (signedCase) {
                for (int e = 0; e < 3; ++e) cs[n++] = g[e];
            } else {
                double md = 0.0;  // the row's largest |det|
                for (double X : {-1.0 - kMarginPx, double(width) + kMarginPx})
                    for (double Y : {yl, yh}) md = std::max(md, std::fabs(raw[2].a + raw[2].b * X + raw[2].c * Y));
                const double E[3] = {Eu + Ed, Ev + Ed, Ew};
                const int idx[3] = {0, 1, 3};
                for (int e = 0; e < 3; ++e) {
                    const Affine &f = raw[idx[e]];
                    cs[n++] = {f.a + md + E[e], f.b, f.c};
                    cs[n++] = {-f.a + md + E[e], -f.b, -f.c};
                }
            }
            // x range: for each constraint, max over the footprint box of g >= 0
            double xlo = 0.0, xhi = double(width - 1);
            bool any = true;
            for (int e = 0; e < n && any; ++e) {
                const Affine &f = cs[e];
                const double A = f.a + std::max(f.c * yl, f.c * yh);
                if (f.b > 0.0) {
                    xlo = std::max(xlo, -A / f.b - 1.0 - kMarginPx);  // A + b (x + 1 + m) >= 0
                } else if (f.b < 0.0) {
                    xhi = std::min(xhi, -A / f.b + kMarginPx);  // A + b (x - m) >= 0
                } else {
                    any = A >= 0.0;
                }
            }
            if (!any || !(xlo <= xhi)) continue;
            const long long xa = std::max(0LL, (long long)std::ceil(xlo - 1e-9 * (1.0 + std::fabs(xlo))));
            const long long xb = std::min((long long)width - 1, (long long)std::floor(xhi + 1e-9 * (1.0 + std::fabs(xhi))));
            for (long long x = xa; x <= xb; ++x) emit(size_t(ky) * size_t(width) + size_t(x), uint32_t(k));
        }
    };
    for (int k = 0; k < numSlots; ++k) visit(k, [&](size_t p, uint32_t) { ++count[p + 1]; });
    for (size_t p = 0; p < pixels; ++p) count[p + 1] += count[p];
    offsets.assign(count.begin(), count.end());
    ids.resize(offsets.back());
    std::vector<uint32_t> fill(offsets.begin(), offsets.end() - 1);
    for (int k = 0; k < numSlots; ++k) visit(k, [&](size_t p, uint32_t id) { ids[fill[p]++] = id; });
    return true;
}

}  // namespace hippt
