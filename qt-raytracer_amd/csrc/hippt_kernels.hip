// hippt_kernels.hip — gfx950 (MI355X, CDNA4) path-tracing kernels.
//
// Three kernels:
//   sphere4_kernel  the reference CUDA megakernel's semantics (CudaPathTracerKernel.cu:23-179)
//                   for the legacy built-in 4-sphere scene; one lane per pixel.
//   mesh_kernel     the triangle/BVH megakernel (new capability; shading model of
//                   RayTracer.h ray_color :579-596 + Lambertian :473-488 in FP32, hash RNG of
//                   CudaPathTracerKernel.cu:23-35,144).  Persistent grid; each lane owns one
//                   (pixel, frame) sample at a time and pulls the next one from a wave-pooled
//                   global queue the moment its path ends (wave64 ballot + mbcnt compaction),
//                   so no lane idles while its wave still has paths to trace.  BVH traversal is
//                   iterative with a per-lane stack in LDS; a wave leaves the traversal loop to
//                   shade once fewer than `waveThreshold` of its lanes are still traversing.
//   combine_kernel  the running-average accumulation + tonemap (CudaPathTracerKernel.cu:157-178)
//                   over a batch of per-sample radiances, in frame order (bit-identical to one
//                   launch per frame).
//
// Arithmetic contract: this file is compiled with -ffp-contract=off; the only fused
// multiply-adds are the explicit fmaf() calls, placed exactly where oracle/pt_oracle.c
// places them, and divisions/sqrt are IEEE correctly rounded (hipcc default), so every
// result-defining value is bit-identical to the CPU restatement.  The BVH box test is NOT
// result-defining (boxes are padded; the closest hit is argmin (t, original index)), so it
// uses the fast reciprocal and FMA slab form.
#include "bvh_builder.h"
#include "hippt_device.h"

#pragma clang fp contract(off)

namespace hippt {
namespace {

constexpr unsigned kNone = 0xffffffffu;
constexpr int kDone = int(0x80000000);

// ---- RNG: CudaPathTracerKernel.cu:23-35 --------------------------------------------------
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// float(state) / 4294967295.0f: the literal rounds to 2^32, so this is the exact product.
__device__ __forceinline__ float rand01(uint32_t &s) {
    s = hash32(s);
    return float(s) * 0x1p-32f;
}

// Rejection loops leave a short RNG cycle: after every 64 consecutive rejections the state is
// xored with 0x9E3779B9 (pt_oracle.c PO_ESCAPE; the reference loops forever there, e.g. on
// the 2-cycle {160893342, 357741884} seeded by pixel (1750,1610) frame 17 at 3840x2160).
__device__ __forceinline__ void escape_cycle(uint32_t &s, unsigned tries) {
    if ((tries & 63u) == 0u) s ^= 0x9E3779B9u;
}

// CudaPathTracerKernel.cu:144 in uint32 wrap-around.
__device__ __forceinline__ uint32_t pixel_seed(uint32_t x, uint32_t y, uint32_t w, uint32_t f) {
    return (x + y * w) * 9781u + (f + 1u) * 6271u;
}

__device__ __forceinline__ float fdot(float ax, float ay, float az, float bx, float by, float bz) {
    return fmaf(ax, bx, fmaf(ay, by, az * bz));
}

// n = q*d + r for n < 2^31, d >= 1: float estimate (relative error < 2^-22, so off by at
// most one for quotients < 2^20) and one exact integer correction — a few VALU instead of
// the ~30-instruction generic unsigned division.
__device__ __forceinline__ void divmod(unsigned n, unsigned d, float rcp, unsigned &q, unsigned &r) {
    q = unsigned(float(n) * rcp);
    int rem = int(n - q * d);
    if (rem < 0) {
        --q;
        rem += int(d);
    } else if (rem >= int(d)) {
        ++q;
        rem -= int(d);
    }
    r = unsigned(rem);
}

__device__ __forceinline__ unsigned q8(float c) {
    return unsigned(sqrtf(fminf(fmaxf(c, 0.0f), 1.0f)) * 255.0f);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// =========================================================================================
// Legacy scene: literal restatement of CudaPathTracerKernel.cu:37-179 (no contraction).
// =========================================================================================
struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

__device__ __forceinline__ V3 normalize3(V3 v) {  // :53-59
    float len = sqrtf(dot(v, v));
    if (len <= 1e-6f) return mk(0.0f, 0.0f, 0.0f);
    return mk(v.x / len, v.y / len, v.z / len);
}

__device__ __forceinline__ V3 rius_legacy(uint32_t &st) {  // :61-68 + short-cycle escape
    for (unsigned tries = 1;; ++tries) {
        float x = rand01(st) * 2.0f - 1.0f;
        float y = rand01(st) * 2.0f - 1.0f;
        float z = rand01(st) * 2.0f - 1.0f;
        V3 p = mk(x, y, z);
        if (dot(p, p) < 1.0f) return p;
        escape_cycle(st, tries);
    }
}

__device__ __forceinline__ bool hit_sphere(V3 c, float r, V3 ro, V3 rd, float &t, V3 &n, V3 &alb) {  // :70-98
    V3 oc = sub(ro, c);
    float a = dot(rd, rd);
    float b = dot(oc, rd);
    float cc = dot(oc, oc) - r * r;
    float d = b * b - a * cc;
    if (d < 0.0f) return false;
    float s = sqrtf(d);
    float t0 = (-b - s) / a;
    float t1 = (-b + s) / a;
    t = t0 > 0.001f ? t0 : t1;
    if (t <= 0.001f) return false;
    V3 p = add(ro, mul(rd, t));
    n = normalize3(sub(p, c));
    if (r > 50.0f) alb = mk(0.8f, 0.8f, 0.0f);
    else if (c.x < -0.5f) alb = mk(0.8f, 0.3f, 0.3f);
    else if (c.x > 0.5f) alb = mk(0.3f, 0.8f, 0.3f);
    else alb = mk(0.75f, 0.75f, 0.75f);
    return true;
}

__global__ __launch_bounds__(256) void sphere4_kernel(Sphere4Params P) {
    const int idx = int(blockIdx.x) * 256 + int(threadIdx.x);
    unsigned long long segs = 0;
    if (idx < P.rows * P.width) {
        const int yb = idx / P.width;
        const int x = idx - yb * P.width;
        const int y = P.y0 + yb;
        float4 acc = P.accum[idx];
        uint32_t outp = 0;
        const float wd = float(max(1, P.width - 1));
        const float hd = float(max(1, P.height - 1));
        const float aspect = float(P.width) / float(P.height);
        const V3 origin = mk(0.0f, 0.3f, 1.2f);
        const V3 ll = mk(-aspect, -1.0f, -1.0f);
        const V3 hor = mk(2.0f * aspect, 0.0f, 0.0f);
        const V3 ver = mk(0.0f, 2.0f, 0.0f);
        for (int fi = 0; fi < P.frames; ++fi) {
            const int frame = P.firstFrame + fi;
            uint32_t seed = pixel_seed(uint32_t(x), uint32_t(y), uint32_t(P.width), uint32_t(frame));
            float u = (float(x) + rand01(seed)) / wd;
            float v = (float(y) + rand01(seed)) / hd;
            V3 rd = normalize3(sub(add(add(ll, mul(hor, u)), mul(ver, v)), origin));
            V3 ro = origin;
            // traceRay, :100-134
            V3 thr = mk(1.0f, 1.0f, 1.0f), rad = mk(0.0f, 0.0f, 0.0f);
            for (int depth = 0; depth < P.maxDepth; ++depth) {
                ++segs;
                float bt = 1e20f;
                V3 bn = mk(0.0f, 0.0f, 0.0f), ba = mk(0.0f, 0.0f, 0.0f);
                bool hit = false;
                float t;
                V3 n, a;
                if (hit_sphere(mk(0.0f, -100.5f, -1.0f), 100.0f, ro, rd, t, n, a) && t < bt) { bt = t; bn = n; ba = a; hit = true; }
                if (hit_sphere(mk(0.0f, 0.0f, -1.0f), 0.5f, ro, rd, t, n, a) && t < bt) { bt = t; bn = n; ba = a; hit = true; }
                if (hit_sphere(mk(-1.0f, 0.0f, -1.4f), 0.5f, ro, rd, t, n, a) && t < bt) { bt = t; bn = n; ba = a; hit = true; }
                if (hit_sphere(mk(1.0f, 0.0f, -1.2f), 0.5f, ro, rd, t, n, a) && t < bt) { bt = t; bn = n; ba = a; hit = true; }
                if (!hit) {
                    V3 un = normalize3(rd);
                    float al = 0.5f * (un.y + 1.0f);
                    V3 sky = add(mul(mk(1.0f, 1.0f, 1.0f), 1.0f - al), mul(mk(0.5f, 0.7f, 1.0f), al));
                    rad = add(rad, mulv(thr, sky));
                    break;
                }
                V3 hp = add(ro, mul(rd, bt));
                V3 sd = normalize3(add(bn, rius_legacy(seed)));
                ro = add(hp, mul(bn, 0.001f));
                rd = sd;
                thr = mulv(thr, ba);
            }
            // :157-178
            const float ff = float(frame), fc = float(frame + 1);
            acc.x = (acc.x * ff + rad.x) / fc;
            acc.y = (acc.y * ff + rad.y) / fc;
            acc.z = (acc.z * ff + rad.z) / fc;
            acc.w = 1.0f;
            outp = (255u << 24) | (q8(acc.x) << 16) | (q8(acc.y) << 8) | q8(acc.z);
        }
        if (P.frames > 0) {
            P.accum[idx] = acc;
            P.out[idx] = outp;
        }
    }
    segs = wave_sum(segs);
    if ((threadIdx.x & 63) == 0 && segs) atomicAdd(&P.stats[0], segs);
}

// =========================================================================================
// Triangle-mesh megakernel.
// =========================================================================================

// Pulls one item per requesting lane from a wave-private pool refilled `chunk` items at a
// time from the global queue (one atomic per chunk, not per lane).  Must be called by the
// whole wave (uniform control flow); pool bounds are wave-uniform.
__device__ __forceinline__ unsigned wave_fetch(bool req, unsigned &poolNext, unsigned &poolEnd,
                                               unsigned *queue, unsigned chunk, unsigned total) {
    const unsigned long long mask = __ballot(req);
    const unsigned n = unsigned(__popcll(mask));
    const unsigned rank = __builtin_amdgcn_mbcnt_hi(unsigned(mask >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(mask), 0u));
    const unsigned avail = poolEnd - poolNext;
    unsigned item;
    if (n <= avail) {
        item = poolNext + rank;
        poolNext += n;
    } else {
        unsigned base = 0;
        if (__lane_id() == 0) base = atomicAdd(queue, chunk);
        base = __builtin_amdgcn_readfirstlane(base);
        item = rank < avail ? poolNext + rank : base + (rank - avail);
        poolNext = base + (n - avail);
        poolEnd = base + chunk;
    }
    return (req && item < total) ? item : kNone;
}

// Phase profiling (STATS build only): pc[2k] counts wave-level passes of phase k (by the
// first active lane), pc[2k+1] lane-level passes; SIMD efficiency = lanes / (64 * waves).
// Phases: 0 outer iteration, 1 camera-ray generation, 2 traversal do-while, 3 interior node
// loop, 4 leaf loop, 5 triangle loop, 6 shading, 7 unit-sphere rejection loop.
#define HIPPT_PROF(k)                                                                     \
    do {                                                                                  \
        if (STATS) {                                                                      \
            ++pc[2 * (k) + 1];                                                            \
            if (__lane_id() == unsigned(__ffsll((unsigned long long)__ballot(1)) - 1)) ++pc[2 * (k)]; \
        }                                                                                 \
    } while (0)

// Build knob (experiments): minimum waves per SIMD the register allocator must allow.
#ifndef HIPPT_MESH_WAVES_PER_EU
#define HIPPT_MESH_WAVES_PER_EU 1
#endif

// LDS-resident scene (small scenes): nodes at an 80-byte stride (20 dwords: 16 nodes start on
// 16 distinct 4-bank groups, so ds_read_b128 of different nodes in a lane group do not
// conflict), triangles at 48 bytes (12 dwords, likewise), shading records at 16 bytes.
constexpr int kLdsNodeF4 = 5;

template <bool STATS, bool LDS_SCENE>
__global__ __launch_bounds__(kMeshBlock, HIPPT_MESH_WAVES_PER_EU) void mesh_kernel(MeshParams P) {
    // Per-lane traversal stack, P.stackDepth (= BVH interior levels) entries per lane, sized
    // at launch so shallow BVHs do not cap occupancy.  Entry k of lane t at stk[k*256 + t]:
    // a wave's lanes hit 64 consecutive dwords, conflict-free for any mix of depths.
    extern __shared__ int stk[];
    int *const my = stk + threadIdx.x;
    const float tmin = 0.001f;

    const float4 *nodes = P.nodes, *tris = P.tris, *shade = P.shade;
    if (LDS_SCENE) {
        float4 *sNodes = reinterpret_cast<float4 *>(stk + (P.stackDepth + 1) * kMeshBlock);
        float4 *sTris = sNodes + P.numNodes * kLdsNodeF4;
        float4 *sShade = sTris + P.numTris * 3;
        for (int i = threadIdx.x; i < P.numNodes * 4; i += kMeshBlock)
            sNodes[(i >> 2) * kLdsNodeF4 + (i & 3)] = P.nodes[i];
        for (int i = threadIdx.x; i < P.numTris * 3; i += kMeshBlock) sTris[i] = P.tris[i];
        for (int i = threadIdx.x; i < P.numTris; i += kMeshBlock) sShade[i] = P.shade[i];
        __syncthreads();
        nodes = sNodes;
        tris = sTris;
        shade = sShade;
    }
    constexpr int nodeF4 = LDS_SCENE ? kLdsNodeF4 : 4;

    unsigned poolNext = 0, poolEnd = 0;

    unsigned item = kNone;
    uint32_t rng = 0;
    int depth = 0;
    float ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0;
    float ix = 0, iy = 0, iz = 0, oix = 0, oiy = 0, oiz = 0;
    float tr = 1, tg = 1, tb = 1;
    int cur = kDone;
    int sp = 0;    // stack depth * kMeshBlock (element offset of the next free slot in `my`)
    int leaf = 0;  // postponed leaf code (< 0) or 0 = none
    float bestT = INFINITY;
    int bestI = -1, bestO = 0x7fffffff;
    bool need = true;
    unsigned long long segs = 0, samples = 0, nvis = 0, ntest = 0;
    unsigned pc[16] = {0};

    auto begin_traversal = [&]() {
        // Fast reciprocal; |d| clamped so that o*inv stays finite (box test only).
        const float cx = copysignf(fmaxf(fabsf(dx), 1e-20f), dx);
        const float cy = copysignf(fmaxf(fabsf(dy), 1e-20f), dy);
        const float cz = copysignf(fmaxf(fabsf(dz), 1e-20f), dz);
        ix = __builtin_amdgcn_rcpf(cx);
        iy = __builtin_amdgcn_rcpf(cy);
        iz = __builtin_amdgcn_rcpf(cz);
        oix = ox * ix;
        oiy = oy * iy;
        oiz = oz * iz;
        cur = 0;
        sp = 0;
        bestT = INFINITY;
        bestI = -1;
        bestO = 0x7fffffff;
    };

    for (;;) {
        HIPPT_PROF(0);
        // ---- refill: every lane whose sample ended takes the next (pixel, frame) -------------
        if (__ballot(need)) {
            const unsigned it = wave_fetch(need, poolNext, poolEnd, P.queue, P.chunk, P.totalItems);
            if (need) {
                need = false;
                item = it;
                if (it != kNone) {
                    HIPPT_PROF(1);
                    // RenderWorker::render u/v (RayTracerFboItem.cpp:109-110), Camera::get_ray
                    // (RayTracer.h:563-567), seed per CudaPathTracerKernel.cu:144.
                    unsigned fl, p, yb, x;
                    divmod(it, P.bandPixels, P.rcpBandPixels, fl, p);
                    divmod(p, unsigned(P.width), P.rcpWidth, yb, x);
                    const unsigned y = unsigned(P.y0) + yb;
                    rng = pixel_seed(x, y, unsigned(P.width), unsigned(P.firstFrame) + fl);
                    const float s = (float(x) + rand01(rng)) * P.invW;
                    const float t = (float(y) + rand01(rng)) * P.invH;
                    float qx, qy;
                    for (unsigned tries = 1;; ++tries) {  // random_in_unit_disk, RayTracer.h:163-169
                        qx = fmaf(2.0f, rand01(rng), -1.0f);
                        qy = fmaf(2.0f, rand01(rng), -1.0f);
                        if (fmaf(qx, qx, qy * qy) < 1.0f) break;
                        escape_cycle(rng, tries);
                    }
                    const CameraF &C = P.cam;
                    const float rx = C.lens_radius * qx, ry = C.lens_radius * qy;
                    const float fx = fmaf(C.v[0], ry, C.u[0] * rx);
                    const float fy = fmaf(C.v[1], ry, C.u[1] * rx);
                    const float fz = fmaf(C.v[2], ry, C.u[2] * rx);
                    ox = C.origin[0] + fx;
                    oy = C.origin[1] + fy;
                    oz = C.origin[2] + fz;
                    dx = (fmaf(t, C.vertical[0], fmaf(s, C.horizontal[0], C.llc[0])) - C.origin[0]) - fx;
                    dy = (fmaf(t, C.vertical[1], fmaf(s, C.horizontal[1], C.llc[1])) - C.origin[1]) - fy;
                    dz = (fmaf(t, C.vertical[2], fmaf(s, C.horizontal[2], C.llc[2])) - C.origin[2]) - fz;
                    tr = tg = tb = 1.0f;
                    depth = 0;
                    begin_traversal();
                }
            }
        }
        if (!__any(cur != kDone)) break;

        // ---- traversal: while-while over the BVH; leave once few lanes remain -------------
        do {
            HIPPT_PROF(2);
            while (cur >= 0) {
                HIPPT_PROF(3);
                const float4 *nd = nodes + __umul24(unsigned(cur), unsigned(nodeF4));  // full-rate 24-bit mul
                const float4 a = nd[0], b = nd[1], c = nd[2];
                const int4 e = *reinterpret_cast<const int4 *>(nd + 3);
                if (STATS) ++nvis;
                const float l0x = fmaf(a.x, ix, -oix), h0x = fmaf(a.w, ix, -oix);
                const float l0y = fmaf(a.y, iy, -oiy), h0y = fmaf(b.x, iy, -oiy);
                const float l0z = fmaf(a.z, iz, -oiz), h0z = fmaf(b.y, iz, -oiz);
                const float l1x = fmaf(b.z, ix, -oix), h1x = fmaf(c.y, ix, -oix);
                const float l1y = fmaf(b.w, iy, -oiy), h1y = fmaf(c.z, iy, -oiy);
                const float l1z = fmaf(c.x, iz, -oiz), h1z = fmaf(c.w, iz, -oiz);
                const float n0 = fmaxf(fmaxf(fminf(l0x, h0x), fminf(l0y, h0y)), fmaxf(fminf(l0z, h0z), tmin));
                const float f0 = fminf(fminf(fmaxf(l0x, h0x), fmaxf(l0y, h0y)), fminf(fmaxf(l0z, h0z), bestT));
                const float n1 = fmaxf(fmaxf(fminf(l1x, h1x), fminf(l1y, h1y)), fmaxf(fminf(l1z, h1z), tmin));
                const float f1 = fminf(fminf(fmaxf(l1x, h1x), fmaxf(l1y, h1y)), fminf(fmaxf(l1z, h1z), bestT));
                const bool hit0 = n0 <= f0, hit1 = n1 <= f1;
                // Branch-free child selection: near child first; the far child is written to
                // the slot above the top unconditionally (one spare slot per lane), kept only
                // when both children are hit; the top is read unconditionally and used only
                // when neither is.
                const bool take0 = hit0 & (!hit1 | (n0 <= n1));  // bitwise: no exec-mask branches
                const int nearC = take0 ? e.x : e.y;
                const int farC = take0 ? e.y : e.x;
                my[sp] = farC;
                const int top = my[max(sp - kMeshBlock, 0)];
                // (logical, not bitwise, operators here: measured 4.5% faster on gfx950)
                const bool none = !(hit0 || hit1);
                sp += (hit0 && hit1) ? kMeshBlock : 0;
                cur = none ? (sp > 0 ? top : kDone) : nearC;
                sp -= (none && sp > 0) ? kMeshBlock : 0;
                // Speculative traversal (Aila & Laine 2009): postpone the first leaf reached and
                // keep descending, so the wave enters the leaf loop only once every lane still
                // in this loop holds a leaf.
                if (cur < 0 && cur != kDone && leaf == 0) {
                    leaf = cur;
                    cur = sp > 0 ? my[sp -= kMeshBlock] : kDone;
                }
                if (!__any(leaf == 0)) break;
            }
            while (leaf != 0) {
                HIPPT_PROF(4);
                const int code = ~leaf;
                const int first = code >> 4, last = first + (code & 15);
                for (int i = first; i < last; ++i) {
                    const float4 *tp = tris + 3 * i;
                    const float4 A = tp[0], B = tp[1], Cc = tp[2];
                    HIPPT_PROF(5);
                    if (STATS) ++ntest;
                    // Möller–Trumbore, division-free edge tests (pt_oracle.c po_tri_hit)
                    const float e1x = A.w, e1y = B.x, e1z = B.y;
                    const float e2x = B.z, e2y = B.w, e2z = Cc.x;
                    const float pvx = fmaf(dy, e2z, -(dz * e2y));
                    const float pvy = fmaf(dz, e2x, -(dx * e2z));
                    const float pvz = fmaf(dx, e2y, -(dy * e2x));
                    const float det = fdot(e1x, e1y, e1z, pvx, pvy, pvz);
                    const float tvx = ox - A.x, tvy = oy - A.y, tvz = oz - A.z;
                    const float un = fdot(tvx, tvy, tvz, pvx, pvy, pvz);
                    const float qvx = fmaf(tvy, e1z, -(tvz * e1y));
                    const float qvy = fmaf(tvz, e1x, -(tvx * e1z));
                    const float qvz = fmaf(tvx, e1y, -(tvy * e1x));
                    const float vn = fdot(dx, dy, dz, qvx, qvy, qvz);
                    const bool neg = det < 0.0f;
                    const float us = neg ? -un : un, vs = neg ? -vn : vn;
                    if (det != 0.0f && us >= 0.0f && vs >= 0.0f && us + vs <= fabsf(det)) {
                        const float tt = fdot(e2x, e2y, e2z, qvx, qvy, qvz) / det;
                        const int orig = __float_as_int(Cc.y);
                        if (tt >= tmin && (tt < bestT || (tt == bestT && orig < bestO))) {
                            bestT = tt;
                            bestI = i;
                            bestO = orig;
                        }
                    }
                }
                // a leaf that was next in line is processed in the same loop
                leaf = 0;
                if (cur < 0 && cur != kDone) {
                    leaf = cur;
                    cur = sp > 0 ? my[sp -= kMeshBlock] : kDone;
                }
            }
        } while (__popcll(__ballot(cur != kDone)) > unsigned(P.waveThreshold));

        // ---- shading: lanes whose traversal finished (ray_color step, RayTracer.h:579-596) ----
        if (item != kNone && cur == kDone) {
            HIPPT_PROF(6);
            ++segs;
            bool finished = false;
            float Lr = 0.0f, Lg = 0.0f, Lb = 0.0f;
            if (bestI < 0) {
                const float uy = (1.0f / sqrtf(fdot(dx, dy, dz, dx, dy, dz))) * dy;
                const float al = 0.5f * (uy + 1.0f);
                const float bl = 1.0f - al;
                Lr = tr * fmaf(al, 0.5f, bl);
                Lg = tg * fmaf(al, 0.7f, bl);
                Lb = tb * fmaf(al, 1.0f, bl);
                finished = true;
            } else if (++depth >= P.maxDepth) {
                finished = true;  // depth exhausted: contributes 0 (RayTracer.h:582-583)
            } else {
                const float4 sh = shade[bestI];
                float nx = sh.x, ny = sh.y, nz = sh.z;
                const float px = fmaf(bestT, dx, ox), py = fmaf(bestT, dy, oy), pz = fmaf(bestT, dz, oz);
                if (!(fdot(dx, dy, dz, nx, ny, nz) < 0.0f)) {  // set_face_normal, :215-218
                    nx = -nx;
                    ny = -ny;
                    nz = -nz;
                }
                float rx, ry, rz, r2;
                for (unsigned tries = 1;; ++tries) {  // random_in_unit_sphere, :155-161
                    HIPPT_PROF(7);
                    rx = fmaf(2.0f, rand01(rng), -1.0f);
                    ry = fmaf(2.0f, rand01(rng), -1.0f);
                    rz = fmaf(2.0f, rand01(rng), -1.0f);
                    r2 = fmaf(rx, rx, fmaf(ry, ry, rz * rz));
                    if (r2 < 1.0f) break;
                    escape_cycle(rng, tries);
                }
                const float inv = 1.0f / sqrtf(r2);  // unit_vector = (1/len)*v, :137-139,151-153
                float sx = nx + rx * inv, sy = ny + ry * inv, sz = nz + rz * inv;
                if (fdot(sx, sy, sz, sx, sy, sz) < 1e-8f) {  // Lambertian degenerate direction, :479-480
                    sx = nx;
                    sy = ny;
                    sz = nz;
                }
                const float4 alb = P.albedo[__float_as_int(sh.w)];
                tr *= alb.x;
                tg *= alb.y;
                tb *= alb.z;
                ox = px;
                oy = py;
                oz = pz;
                dx = sx;
                dy = sy;
                dz = sz;
                begin_traversal();
            }
            if (finished) {
                P.scratch[item] = Lr;
                P.scratch[size_t(P.totalItems) + item] = Lg;
                P.scratch[2 * size_t(P.totalItems) + item] = Lb;
                ++samples;
                item = kNone;
                need = true;
            }
        }
    }

    segs = wave_sum(segs);
    samples = wave_sum(samples);
    if (STATS) {
        nvis = wave_sum(nvis);
        ntest = wave_sum(ntest);
    }
    if (__lane_id() == 0) {
        atomicAdd(&P.stats[0], segs);
        atomicAdd(&P.stats[1], samples);
        if (STATS) {
            atomicAdd(&P.stats[2], nvis);
            atomicAdd(&P.stats[3], ntest);
        }
    }
    if (STATS) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const unsigned long long v = wave_sum(pc[k]);
            if (__lane_id() == 0) atomicAdd(&P.stats[4 + k], v);
        }
    }
}
#undef HIPPT_PROF

// Running average in frame order, then ARGB (CudaPathTracerKernel.cu:157-178).
__global__ __launch_bounds__(256) void combine_kernel(CombineParams P) {
    const unsigned stride = gridDim.x * 256u;
    for (unsigned p = blockIdx.x * 256u + threadIdx.x; p < P.bandPixels; p += stride) {
        float4 acc = P.accum[p];
        for (int fl = 0; fl < P.frames; ++fl) {
            const size_t k = size_t(fl) * P.bandPixels + p;
            const int f = P.firstFrame + fl;
            const float ff = float(f), fc = float(f + 1);
            acc.x = fmaf(acc.x, ff, P.scratch[k]) / fc;
            acc.y = fmaf(acc.y, ff, P.scratch[size_t(P.totalItems) + k]) / fc;
            acc.z = fmaf(acc.z, ff, P.scratch[2 * size_t(P.totalItems) + k]) / fc;
        }
        acc.w = 1.0f;
        P.accum[p] = acc;
        P.out[p] = (255u << 24) | (q8(acc.x) << 16) | (q8(acc.y) << 8) | q8(acc.z);
    }
}

}  // namespace

hipError_t launch_sphere4(const Sphere4Params &p, hipStream_t s) {
    const long long n = (long long)p.rows * p.width;
    if (n <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n + 255) / 256);
    hipLaunchKernelGGL(sphere4_kernel, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// Stack: one spare slot per lane above the deepest level for the speculative far-child
// write; then (LDS_SCENE) the scene copy.
size_t mesh_lds_bytes(int stackDepth, int ldsNodes, int ldsTris) {
    return size_t(stackDepth + 1) * kMeshBlock * sizeof(int) + size_t(ldsNodes) * kLdsNodeF4 * 16 +
           size_t(ldsTris) * (3 + 1) * 16;
}

size_t mesh_lds_scene_limit() { return 24u << 10; }

using MeshFn = void (*)(MeshParams);
static MeshFn mesh_fn(bool count, bool lds) {
    if (count) return lds ? mesh_kernel<true, true> : mesh_kernel<true, false>;
    return lds ? mesh_kernel<false, true> : mesh_kernel<false, false>;
}

hipError_t launch_mesh(const MeshParams &p, int blocks, bool countTraversal, hipStream_t s) {
    if (p.stackDepth < 1 || p.stackDepth > kStackDepth) return hipErrorInvalidValue;
    const bool lds = p.ldsScene != 0;
    const size_t bytes = mesh_lds_bytes(p.stackDepth, lds ? p.numNodes : 0, lds ? p.numTris : 0);
    hipLaunchKernelGGL(mesh_fn(countTraversal, lds), dim3(blocks), dim3(kMeshBlock), bytes, s, p);
    return hipGetLastError();
}

hipError_t launch_combine(const CombineParams &p, hipStream_t s) {
    if (p.bandPixels == 0) return hipSuccess;
    unsigned blocks = (p.bandPixels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(combine_kernel, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

int mesh_blocks_per_cu(bool countTraversal, int stackDepth, int ldsNodes, int ldsTris) {
    int n = 0;
    const bool lds = ldsNodes > 0;
    const size_t bytes = mesh_lds_bytes(stackDepth, ldsNodes, ldsTris);
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mesh_fn(countTraversal, lds), kMeshBlock, bytes);
    if (e != hipSuccess || n <= 0) n = 1;
    return n;
}

}  // namespace hippt
