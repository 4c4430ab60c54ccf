// hippt_kernels.hip — gfx950 (MI355X, CDNA4) path-tracing kernels.
//
// Three kernels:
//   sphere4_kernel  the reference CUDA megakernel's semantics (CudaPathTracerKernel.cu:23-179)
//                   for the legacy built-in 4-sphere scene; one lane per pixel.
//   mesh_kernel     the BVH megakernel over triangles and spheres (new capability; shading
//                   model of RayTracer.h ray_color :579-596 with Lambertian/Metal/Dielectric
//                   :473-540 in FP32, hash RNG of CudaPathTracerKernel.cu:23-35,144).
//                   Persistent grid; each lane owns one (pixel, frame) sample at a time and
//                   pulls the next one from a wave-pooled global queue the moment its path ends
//                   (wave64 ballot + mbcnt compaction), so no lane idles while its wave still
//                   has paths to trace.  BVH traversal is iterative with a per-lane stack in
//                   LDS; a wave leaves the traversal loop to shade once fewer than
//                   `waveThreshold` of its lanes are still traversing.  FULL=false is the
//                   Lambertian-triangle specialisation.
//   combine_kernel  the running-average accumulation + tonemap (CudaPathTracerKernel.cu:157-178)
//                   over a batch of per-sample radiances, in frame order (bit-identical to one
//                   launch per frame).
//
// Arithmetic contract: see hippt_trace.h (shared with oracle/pt_oracle.c).
#include "hippt_trace.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace hippt {
namespace {
using namespace trace;

__device__ __forceinline__ unsigned q8(float c) {
    return unsigned(sqrtf(fminf(fmaxf(c, 0.0f), 1.0f)) * 255.0f);
}

// The displayed pixel of an accumulated colour.  kPixelArgb: the CUDA backend's word
// (CudaPathTracerKernel.cu:171-178): 0xAARRGGBB, channel = uint(sqrt(clamp(c, 0, 1)) * 255)
// truncated.  kPixelRgba8: the GL / Vulkan backends' RGBA8 UNORM image texel
// (GpuPathTracer.cpp:284-285, pathtrace_vulkan.comp:113-114): bytes R, G, B, A in memory
// (0xAABBGGRR), channel = sqrt(clamp(c, 0, 1)) * 255 rounded to nearest, ties to even.
__device__ __forceinline__ uint32_t pack_pixel(float r, float g, float b, int format) {
    if (format == kPixelRgba8) {
        const auto u8 = [](float c) { return unsigned(rintf(sqrtf(fminf(fmaxf(c, 0.0f), 1.0f)) * 255.0f)); };
        return (255u << 24) | (u8(b) << 16) | (u8(g) << 8) | u8(r);
    }
    return (255u << 24) | (q8(r) << 16) | (q8(g) << 8) | q8(b);
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
        const int y = P.y0 + yb * P.rowStride;
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
            outp = pack_pixel(acc.x, acc.y, acc.z, P.format);
        }
        if (P.frames > 0) {
            P.accum[idx] = acc;
            P.out[idx] = outp;
            // a blocking frame's word also straight into the caller's pinned frame (full-frame
            // row y): the PCIe writes stream out while other waves still trace
            if (P.hostOut) P.hostOut[size_t(y) * size_t(P.width) + size_t(x)] = outp;
        }
    }
    segs = wave_sum(segs);
    if ((threadIdx.x & 63) == 0 && segs) atomicAdd(&stat_slot(P.stats)[0], segs);
}

// =========================================================================================
// Mesh megakernel.
// =========================================================================================

// Build knob (experiments): minimum waves per SIMD the register allocator must allow.  The
// general (FULL) kernel is held to 7 (<= 72 VGPRs, as many waves as the SGPR budget allows)
// instead of the 6 its 73 VGPRs would give.
#ifndef HIPPT_MESH_WAVES_PER_EU
#define HIPPT_MESH_WAVES_PER_EU 1
#endif

// LDS-resident scene (small scenes): node strides kLdsNodeF4 / kLdsNode4F4 (hippt_device.h),
// primitives at 48 bytes (12 dwords: conflict-free likewise), shading records at 16 bytes.

#ifdef HIPPT_DEBUG_TIMELINE
// per wave: [0] start, [1] first drained fetch, [2] end (s_memrealtime, 100 MHz), [3] items,
// [4] HW_ID, [5] XCC_ID
__device__ unsigned long long g_timeline[65536 * 8];
#endif
#ifdef HIPPT_DEBUG_RATE
// per 10 us bucket of a launch (from each wave's own start): [0] samples finished, [1] segments,
// [2] wave rounds, [3] live-lane rounds (lanes holding a sample), [4] waves running
// (kRateSlots copies, by wave id, summed on the host: one address per bucket serialised the atomics)
constexpr int kRateBuckets = 1024, kRateSlots = 256;
__device__ unsigned long long g_rate[kRateSlots * kRateBuckets * 5];
#endif

// SGPR budget.  A wave's SGPR allocation (granule 16) plus the 16 the trap handler reserves
// must fit 7 waves in a SIMD's 800 SGPRs: <= 96.  Unbounded, the compiler used 97-100, the
// hardware then held 6 blocks per CU while the occupancy query (which does not count the trap
// reservation) reported 7 — 1/7 of the persistent grid started only when others finished
// (per-wave timeline, tools/timeline.py) and ran as a tail.  At 96: all blocks resident,
// Cornell +0.5%, blob +1.3%.
#ifndef HIPPT_NUM_SGPR
#define HIPPT_NUM_SGPR 96
#endif
#define HIPPT_SGPR_ATTR __attribute__((amdgpu_num_sgpr(HIPPT_NUM_SGPR)))

// Lambertian-triangle kernels: a shading pass runs at most this many tries of the unit-sphere
// draw; a lane whose draw is still rejecting stays on its hit and resumes the same chain in the
// next pass (0: the whole draw in one pass).
#ifndef HIPPT_REJECT_CAP
#define HIPPT_REJECT_CAP 0
#endif

// LDS-resident 4-wide trees sort packed child keys (trace::child_key_p: codes in the keys' low
// bits, the sorting network as unsigned min/max pairs); 0: keys and codes sorted as pairs
#ifndef HIPPT_PACKED_KEYS
#define HIPPT_PACKED_KEYS 1
#endif

// Build knob (experiment): the camera sample's and item order's arguments loaded where a wave
// generates camera rays instead of held in registers across the kernel (trace::late_arg_at).
#ifndef HIPPT_LATE_CAM
#define HIPPT_LATE_CAM 0
#endif
#ifndef HIPPT_WIDE_WAVES_PER_EU
#define HIPPT_WIDE_WAVES_PER_EU 7
#endif
// Running average in frame order, then the output word (CudaPathTracerKernel.cu:157-178), of band
// pixel p over a batch of per-sample radiances.
template <int UNROLL, bool HOST = false>
__device__ __forceinline__ void combine_pixel(const CombineParams &P, unsigned p, const HostFrame &H = HostFrame{}) {
    float4 acc = P.accum[p];
#pragma unroll UNROLL
    for (int fl = 0; fl < P.frames; ++fl) {
        const size_t k = size_t(fl) * P.bandPixels + p;
        const int f = P.firstFrame + fl;
        const float ff = float(f), fc = float(f + 1);
        const float3 L = *reinterpret_cast<const float3 *>(P.scratch + 3 * k);
        acc.x = fmaf(acc.x, ff, L.x) / fc;
        acc.y = fmaf(acc.y, ff, L.y) / fc;
        acc.z = fmaf(acc.z, ff, L.z) / fc;
    }
    acc.w = 1.0f;
    P.accum[p] = acc;
    const uint32_t word = pack_pixel(acc.x, acc.y, acc.z, P.format);
    P.out[p] = word;
    if (HOST && H.host) {
        const unsigned yb = p / unsigned(H.width), x = p - yb * unsigned(H.width);
        H.host[size_t(unsigned(H.y0) + yb * unsigned(H.stride)) * unsigned(H.width) + x] = word;
    }
}

// One 64-pixel chunk of the previous batch's combine (MeshParams::comb) for the whole wave; false
// once every chunk is claimed.  Wave-uniform.  The frame loop is not unrolled here: unrolled 8x
// at the kernel's two call sites it cost blob70k 3% even with the combine off (r3g/r3h; none
// without the unroll, r3i).
__device__ __forceinline__ bool combine_chunk(const MeshParams &P) {
    unsigned base = 0;
    if (__lane_id() == 0) base = atomicAdd(P.combCtr, 64u);
    base = __builtin_amdgcn_readfirstlane(base);
    if (base >= P.comb.bandPixels) return false;
    const unsigned p = base + __lane_id();
    if (p < P.comb.bandPixels) combine_pixel<1>(P.comb, p);
    return true;
}

// Chained batches (hippt_trace.h): the running average of band pixel p over the run's batches
// [c0, c1] in order (batch b: frames C.firstFrame + b*step + fl, its samples in ring slot b % slots).
template <int UNROLL, bool HOST = false>
__device__ __forceinline__ void combine_pixel_chain(const CombineParams &C, const float *scratch, unsigned p, int c0,
                                                    int c1, unsigned slots, unsigned shift, int step,
                                                    const HostFrame &H = HostFrame{}) {
    float4 acc = C.accum[p];
    for (int b = c0; b <= c1; ++b) {
        const float *scr = scratch + 3 * ((size_t(unsigned(b) & (slots - 1u)) << shift) + p);
        const int f0 = C.firstFrame + b * step;
#pragma unroll UNROLL
        for (int fl = 0; fl < C.frames; ++fl) {
            const float3 L = *reinterpret_cast<const float3 *>(scr + 3 * size_t(fl) * C.bandPixels);
            const float ff = float(f0 + fl), fc = float(f0 + fl + 1);
            acc.x = fmaf(acc.x, ff, L.x) / fc;
            acc.y = fmaf(acc.y, ff, L.y) / fc;
            acc.z = fmaf(acc.z, ff, L.z) / fc;
        }
    }
    acc.w = 1.0f;
    C.accum[p] = acc;
    const uint32_t word = pack_pixel(acc.x, acc.y, acc.z, C.format);
    C.out[p] = word;
    if (HOST && H.host) {
        const unsigned yb = p / unsigned(H.width), x = p - yb * unsigned(H.width);
        H.host[size_t(unsigned(H.y0) + yb * unsigned(H.stride)) * unsigned(H.width) + x] = word;
    }
}

// combine_chunk of a CHAIN launch: 64 pixels over its combine range (ChainWave::c0..c1), chunks from
// the launch's epoch-parity counter; arguments loaded where they are used.
__device__ __forceinline__ bool combine_chunk_chain(const ChainWave *cw) {
    unsigned *const ctl = late_field(chainCtl);
    const unsigned e = late_field(chainEpoch);
    const unsigned bandPixels = late_field(comb.bandPixels);
    unsigned base = 0;
    if (__lane_id() == 0) base = atomicAdd(ctl + kChainCtlWord + 64u + 32u * (e & 1u), 64u);
    base = __builtin_amdgcn_readfirstlane(base);
    if (base >= bandPixels) return false;
    const unsigned p = base + __lane_id();
    const int c0 = int(__builtin_amdgcn_readfirstlane(cw->c0)), c1 = int(__builtin_amdgcn_readfirstlane(cw->c1));
    if (p < bandPixels)
        combine_pixel_chain<8>(late_field(comb), late_field(scratch), p, c0, c1, late_field(chainSlots),
                               late_field(chainShift), max(0, late_field(chainStep)));
    if (unsigned *const audit = late_field(chainAudit)) {
        const bool v = p < bandPixels;
        audit_combine(audit, c0, c1, unsigned(__popcll(__ballot(v))), wave_sum(v ? audit_hash(p) : 0ull), e,
                      late_field(comb.firstFrame), max(0, late_field(chainStep)));
    }
    return true;
}

// Camera-ray pool (POOL, HIPPT_OPT_CAMERA_POOL): a refill happens when a lane's path ends, so only
// the lanes whose paths ended together generate camera rays, at ~30% SIMD efficiency (Cornell,
// tools/phase_profile.py).  With the pool, the wave generates the camera rays of its next 64 work
// items with all lanes at once into LDS (one entry per lane, fields 64 words apart: conflict-free),
// and refilling lanes take the next entries in order; the pool is regenerated when a refill needs
// more entries than it holds (those lanes take the rest of the old pool first, then the new one).
// Items are claimed from the work queue in the same order as without the pool and every claimed
// item is traced, so the results are the same.
template <bool POOL>
__device__ __forceinline__ void pool_take(const MeshParams &P, const float *pool, unsigned k, unsigned &item, Ray &r,
                                          uint32_t &rng) {
    item = __float_as_uint(pool[k]);
    if (item == kNone) return;
    rng = __float_as_uint(pool[64 + k]);
    r.dx = pool[128 + k];
    r.dy = pool[192 + k];
    r.dz = pool[256 + k];
    if (P.poolWords == kPoolWordsFull) {
        r.ox = pool[320 + k];
        r.oy = pool[384 + k];
        r.oz = pool[448 + k];
    } else {
        r.ox = P.cam.origin[0];
        r.oy = P.cam.origin[1];
        r.oz = P.cam.origin[2];
    }
}

// CHAIN: chained batches (hippt_trace.h; camera-pool kernels over 4-wide float nodes only)
template <bool STATS, bool LDS_SCENE, bool FULL, bool WIDE, bool QUANT, bool SPILL = true, bool POOL = false,
          bool HYBRID = false, bool HALF = false, bool CHAIN = false>
__global__ __launch_bounds__(kMeshBlock, (FULL || WIDE) ? HIPPT_WIDE_WAVES_PER_EU : HIPPT_MESH_WAVES_PER_EU) HIPPT_SGPR_ATTR void mesh_kernel(MeshParams P) {
    static_assert(!QUANT || (WIDE && !LDS_SCENE), "quantized nodes: 4-wide global-memory traversal only");
    static_assert(!CHAIN || (POOL && WIDE && !QUANT && !HYBRID && !HALF && !STATS), "chained batches: pool kernels");
#ifdef HIPPT_DEBUG_TIMELINE
    const unsigned tlw = blockIdx.x * 4u + (threadIdx.x >> 6);
    unsigned long long tlDrained = 0, tlItems = 0, tlRounds = 0, tlLate = 0;
    if (__lane_id() == 0 && tlw < 65536) {
        g_timeline[8 * tlw] = __builtin_amdgcn_s_memrealtime();
        g_timeline[8 * tlw + 4] = __builtin_amdgcn_s_getreg(0xF804);  // HW_REG_HW_ID
        g_timeline[8 * tlw + 5] = __builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
    }
#endif
    // Per-lane traversal stack, P.stackDepth (= BVH interior levels) entries per lane, sized
    // at launch so shallow BVHs do not cap occupancy.  Entry k of lane t at stk[k*256 + t]:
    // a wave's lanes hit 64 consecutive dwords, conflict-free for any mix of depths.
    // LDS-resident scenes put the node copy at LDS address 0 (node rows are then addressed by
    // their byte offset alone: no base add per row read), then the stack, primitives, shading.
    extern __shared__ int lds[];
    constexpr int ldsNodeF4 = WIDE ? kLdsNode4F4 : kLdsNodeF4;
    // Trees in global memory (4-wide): the top of the tree (P.topBytes of the node array) at LDS
    // address 0, then the stack.
    constexpr bool TOP = WIDE && !LDS_SCENE;
    // packed child keys over LDS-resident 4-wide trees (Cornell +0.8%; the general kernel lost
    // 4.3% with them under the round-2 loop exits and gains 0.6% under the current ones,
    // cornell_mixed, round 3 A/Bs)
    constexpr bool PACKED = WIDE && LDS_SCENE && bool(HIPPT_PACKED_KEYS);
    int *const stk = LDS_SCENE ? lds + P.numNodes * ldsNodeF4 * 4 : lds + (TOP ? (P.topBytes >> 2) : 0u);
    int *const my = stk + threadIdx.x;

    const float4 *nodes = P.nodes, *tris = P.tris, *shade = P.shade, *mats = P.mats;
    if (LDS_SCENE) {
        float4 *sNodes = reinterpret_cast<float4 *>(lds);
        float4 *sTris = reinterpret_cast<float4 *>(stk + (P.stackDepth + 1) * kMeshBlock);
        float4 *sShade = sTris + P.numTris * 3;
        // the materials too: a shading step's shade-record -> material chain then stays in LDS
        float4 *sMats = sShade + P.numTris;
        for (int i = threadIdx.x; i < P.numMats * 2; i += kMeshBlock) sMats[i] = P.mats[i];
        mats = sMats;
        if (WIDE) {
            // packed keys: the copy's code rows hold each code's low refBits bits (child_key_p merges
            // them into the key with one v_and_or)
            const unsigned refMask = PACKED ? (1u << P.refBits) - 1u : ~0u;
            for (int i = threadIdx.x; i < P.numNodes * kLdsNode4F4; i += kMeshBlock) {
                float4 v = P.nodes[i];
                if (PACKED && (i & 7) == 6) {
                    v.x = __uint_as_float(__float_as_uint(v.x) & refMask);
                    v.y = __uint_as_float(__float_as_uint(v.y) & refMask);
                    v.z = __uint_as_float(__float_as_uint(v.z) & refMask);
                    v.w = __uint_as_float(__float_as_uint(v.w) & refMask);
                }
                sNodes[i] = v;
            }
        } else {
            for (int i = threadIdx.x; i < P.numNodes * 4; i += kMeshBlock)
                sNodes[(i >> 2) * kLdsNodeF4 + (i & 3)] = P.nodes[i];
        }
        for (int i = threadIdx.x; i < P.numTris * 3; i += kMeshBlock) sTris[i] = P.tris[i];
        for (int i = threadIdx.x; i < P.numTris; i += kMeshBlock) sShade[i] = P.shade[i];
        __syncthreads();
        nodes = sNodes;
        tris = sTris;
        shade = sShade;
    }
    if (TOP && P.topBytes) {
        float4 *sTop = reinterpret_cast<float4 *>(lds);
        for (unsigned i = threadIdx.x; i < (P.topBytes >> 4); i += kMeshBlock) sTop[i] = P.nodes[i];
        __syncthreads();
    }
    constexpr int nodeF4 = LDS_SCENE ? ldsNodeF4 : (WIDE ? (QUANT ? 4 : 8) : 4);
    const SpillArea S{P.spill, (blockIdx.x * unsigned(kMeshBlock) + threadIdx.x) * unsigned(P.spillCap), P.stackCap};

    // this wave's camera-ray pool (POOL): entries [poolNext, 64) not taken yet (wave-uniform).  Each
    // wave's pool block starts with its kWaveWords state words (WaveWords: work queue, segment count,
    // chain state), so that their address is the pool's minus a constant.
    constexpr unsigned kWW = POOL ? kWaveWords : 0u;
    float *const pool = reinterpret_cast<float *>(reinterpret_cast<char *>(lds) + P.poolOffset) +
                        (threadIdx.x >> 6) * unsigned(P.poolWords * 64 + kWW) + kWW;
    unsigned poolNext = 64;
    WaveWords *const ww = reinterpret_cast<WaveWords *>(pool - kWW);
    ChainWave *const cw = &ww->cw;
    WaveWords *const bw = reinterpret_cast<WaveWords *>(reinterpret_cast<char *>(lds) + P.poolOffset);
    ChainView *const view = &bw->view;
    unsigned *const drained = POOL ? bw->drained : nullptr;  // the block's drained-queue words
    // CHAIN kernels keep the work queue and the segment count in LDS (ww->Q, ww->segs), the others in
    // registers
    WorkQueue Q;
    if (POOL && threadIdx.x == 0) bw->drained[0] = bw->drained[1] = 0u;
    if constexpr (CHAIN) {
        chain_begin(Q, cw, view);
        store_queue(&ww->Q, Q);
        if (__lane_id() == 0) ww->segs = 0;
    } else {
        queue_begin(Q, P.totalItems, P.chunk);
    }
    if (POOL) __syncthreads();  // the block's words (its first wave's: mailbox view, drained queues)
    unsigned item = kNone;
    uint32_t rng = 0;
    int depth = 0;
    Ray r{};
    Trav T;
    T.cur = kDone;
    T.sp = 0;
    T.leaf = 0;
    T.bestT = INFINITY;
    T.bestI = -1;
    T.bestO = 0x7fffffff;
    float tr = 1, tg = 1, tb = 1;
    bool need = true, fresh = false;
    constexpr unsigned CAP = FULL ? 0u : unsigned(HIPPT_REJECT_CAP);
    unsigned pend = 0;  // tries so far of a pending unit-sphere draw (CAP), 0 = none
    // per-lane counts fit 32 bits (a lane traces a few thousand segments per launch); widened
    // for the wave sum
    unsigned segs = 0, samples = 0;
    unsigned long long nvis = 0, ntest = 0;
    unsigned pc[kProfSlots] = {0};

    // The previous batch's combine (memory-bound) beside this batch's paths (VALU-bound): one wave
    // in 8 starts with it while the others trace, and every wave takes what is left when its
    // paths run out (the launch's tail, where the traversal leaves SIMDs idle).  Not inside the
    // path loop: with the paths' state live it costs registers.
    // Tail finish (the camera-pool kernel over a tree in global memory): once the wave has found
    // the queues drained, its traversal rounds run until no lane traverses (no wave-threshold
    // exit), so its last iterations are not one node visit each: the slowest 1/8 blob70k share
    // 3.36 -> 3.27 ms, full size unchanged; LDS scenes lose 1% on the share and keep the exit
    // (DESIGN_LOG.md §A.1)
    constexpr bool FINISH = POOL && !LDS_SCENE;
#ifdef HIPPT_DEBUG_RATE
    const unsigned long long rtStart = __builtin_amdgcn_s_memrealtime();
    unsigned rtBucket = 0, rtSegs0 = 0, rtSamples0 = 0;
    unsigned long long rtRounds = 0, rtLive = 0;
    auto rt_flush = [&](unsigned nb) {
        const unsigned long long a = wave_sum((unsigned long long)(samples - rtSamples0));
        const unsigned wsegs = CHAIN ? __builtin_amdgcn_readfirstlane(ww->segs) : 0u;
        const unsigned long long b = CHAIN ? (unsigned long long)(wsegs - rtSegs0) : wave_sum((unsigned long long)(segs - rtSegs0));
        rtSamples0 = samples;
        rtSegs0 = CHAIN ? wsegs : segs;
        if (__lane_id() == 0) {
            const unsigned k = ((blockIdx.x * 4u + (threadIdx.x >> 6)) % unsigned(kRateSlots) * unsigned(kRateBuckets) +
                                min(rtBucket, unsigned(kRateBuckets - 1))) * 5u;
            atomicAdd(&g_rate[k], a);
            atomicAdd(&g_rate[k + 1], b);
            atomicAdd(&g_rate[k + 2], rtRounds);
            atomicAdd(&g_rate[k + 3], rtLive);
            atomicAdd(&g_rate[k + 4], 1ull);
        }
        rtRounds = rtLive = 0;
        rtBucket = nb;
    };
#endif
    unsigned waveThr = unsigned(P.waveThreshold);
    bool combLeft = CHAIN ? int(__builtin_amdgcn_readfirstlane(cw->c1)) >= int(__builtin_amdgcn_readfirstlane(cw->c0))
                          : P.comb.bandPixels != 0;
    auto comb_step = [&]() { return CHAIN ? combine_chunk_chain(cw) : combine_chunk(P); };
    if (combLeft && (blockIdx.x & 1u) == 0 && threadIdx.x < 64u)
        while (combLeft) combLeft = comb_step();
    for (;;) {
        prof<STATS>(pc, 0);
#ifdef HIPPT_DEBUG_TIMELINE
        if (tlDrained) ++tlRounds;
#endif
#ifdef HIPPT_DEBUG_RATE
        {
            const unsigned nb = unsigned((__builtin_amdgcn_s_memrealtime() - rtStart) / 1000ull);
            if (nb != rtBucket) rt_flush(nb);
            ++rtRounds;
            rtLive += __popcll(__ballot(item != kNone));
        }
#endif
        // ---- refill: every lane whose sample ended takes the next (pixel, frame) -------------
        if (POOL) {
            const unsigned long long m = __ballot(need);
            if (m) {
                const unsigned n = unsigned(__popcll(m));
                const unsigned rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
                const unsigned avail = 64u - poolNext;
                const bool took = need;
                if (need && rank < avail) {
                    need = false;
                    pool_take<POOL>(P, pool, poolNext + rank, item, r, rng);
                }
                if (n > avail) {
                    // the camera rays of the wave's next 64 items, every lane at once
                    unsigned it;
                    Ray c{};
                    uint32_t crng = 0;
                    if constexpr (CHAIN) {
                        // items of the wave's batch (ChainWave::t); a drained batch moves the wave into
                        // the run's next one (chain_next) and the lanes still without an item take its
                        // items, so that a refill spans batches and no lane waits for a batch's end
                        WorkQueue Q = load_queue(&ww->Q);
                        unsigned raw = kNone, tItem = 0;
                        bool want = true;
                        for (;;) {
                            const unsigned t = __builtin_amdgcn_readfirstlane(cw->t);
                            // the own group's queue (ChainWave::stat) spans its batches' items
                            const bool grp = t == __builtin_amdgcn_readfirstlane(cw->stat);
                            const unsigned nb = grp ? late_field(chainGroup) : 1u;
                            const unsigned got =
                                queue_fetch(want, Q, chain_block(late_field(chainCtl), t, late_field(chainSlots)),
                                            late_field(totalItems) * nb, late_field(chunk), grp, drained, t);
                            if (want && got != kNone) {
                                // a group position: the group walks the one-batch order once
                                chain::group_item(got, t, nb, raw, tItem);
                                want = false;
                            }
                            if (!__ballot(want) || !chain_next(Q, cw, view)) break;
                        }
                        store_queue(&ww->Q, Q);
                        it = order_item_late(raw);
                        if (it != kNone) {
                            // the item's frames: its batch's offset from the launch's own batch's
                            const int step = int(__builtin_amdgcn_readfirstlane(unsigned(cw->step)));
                            const unsigned fAdd = chain::frame_add(tItem, late_field(chainSeq), step);
                            camera_sample(cam_args_late(), it, c, crng, fAdd);
                            if (unsigned *const audit = late_field(chainAudit))
                                audit_trace(audit, tItem, it, unsigned(late_field(firstFrame)) + fAdd,
                                            late_field(chainEpoch));
                            it |= (tItem & (late_field(chainSlots) - 1u)) << late_field(chainShift);
                        }
                    } else {
                        it = HIPPT_LATE_CAM ? order_item_late(queue_fetch(true, Q, P.queue, P.totalItems, P.chunk, true, drained))
                                            : order_item(P, queue_fetch(true, Q, P.queue, P.totalItems, P.chunk, true, drained));
                        if (it != kNone) {
                            if (HIPPT_LATE_CAM)
                                camera_sample(cam_args_late(), it, c, crng);
                            else
                                camera_sample(P, it, c, crng);
                        }
                    }
#ifdef HIPPT_DEBUG_TIMELINE
                    if (!tlDrained && __ballot(it == kNone)) tlDrained = __builtin_amdgcn_s_memrealtime();
                    tlItems += __popcll(__ballot(it != kNone));
#endif
                    if (it != kNone) prof<STATS>(pc, 1);
                    const unsigned k = __lane_id();
                    pool[k] = __uint_as_float(it);
                    pool[64 + k] = __uint_as_float(crng);
                    pool[128 + k] = c.dx;
                    pool[192 + k] = c.dy;
                    pool[256 + k] = c.dz;
                    if (P.poolWords == kPoolWordsFull) {
                        pool[320 + k] = c.ox;
                        pool[384 + k] = c.oy;
                        pool[448 + k] = c.oz;
                    }
                    poolNext = n - avail;
                    if (need) {
                        need = false;
                        pool_take<POOL>(P, pool, rank - avail, item, r, rng);
                    }
                } else {
                    poolNext += n;
                }
                if (took && item != kNone) {
                    tr = tg = tb = 1.0f;
                    depth = 0;
                    fresh = true;
                }
                if (FINISH && __ballot(took && item == kNone)) waveThr = 0u;
            }
        } else if (__ballot(need)) {
            const unsigned it = HIPPT_LATE_CAM ? order_item_late(queue_fetch(need, Q, P.queue, P.totalItems, P.chunk))
                                               : order_item(P, queue_fetch(need, Q, P.queue, P.totalItems, P.chunk));
#ifdef HIPPT_DEBUG_TIMELINE
            if (!tlDrained && __ballot(need && it == kNone)) tlDrained = __builtin_amdgcn_s_memrealtime();
            tlItems += __popcll(__ballot(it != kNone));
#endif
            if (need) {
                need = false;
                item = it;
                if (it != kNone) {
                    prof<STATS>(pc, 1);
                    if (HIPPT_LATE_CAM)
                        camera_sample(cam_args_late(), it, r, rng);
                    else
                        camera_sample(P, it, r, rng);
                    tr = tg = tb = 1.0f;
                    depth = 0;
                    fresh = true;
                }
            }
        }
        // new rays (refilled or scattered): one place, so a pass with lanes of both kinds runs
        // the reciprocals once
        if (fresh) {
            fresh = false;
            prepare(r);
            begin(T);
        }
        if (!__any(busy(T) || pend != 0u)) break;

        // ---- traversal: while-while over the BVH; leave once few lanes remain -------------
        if (!CAP || __any(busy(T))) do {
            prof<STATS>(pc, 2);
            if (WIDE)
                traverse_round_wide<nodeF4, STATS, FULL, QUANT, SPILL, LDS_SCENE, TOP, HYBRID, PACKED, HALF>(
                    T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit, S, P.topBytes, P.refBits);
            else
                traverse_round<nodeF4, STATS, FULL>(T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit);
        } while (__popcll(__ballot(busy(T))) > (FINISH ? waveThr : unsigned(P.waveThreshold)));

        // ---- shading: lanes whose traversal finished (ray_color step, RayTracer.h:579-596) ----
        // (a lane resuming a pending draw continues its segment; CHAIN kernels count the wave's
        // segments in ww->segs, one LDS add per round)
        if constexpr (CHAIN) {
            const unsigned long long sm = __ballot(item != kNone && !busy(T) && !(CAP && pend != 0u));
            if (__lane_id() == 0 && sm) atomicAdd(&ww->segs, unsigned(__popcll(sm)));
        }
        if (item != kNone && !busy(T)) {
            prof<STATS>(pc, 6);
            const bool cont = CAP && pend != 0u;  // resumes a pending draw: same segment
            if (!CHAIN && !cont) ++segs;
            bool finished = false;
            float Lr = 0.0f, Lg = 0.0f, Lb = 0.0f;
            if (!FULL) {
                // Lambertian triangles: the sky's 1/sqrt(|d|^2) and the scatter's 1/sqrt(|q|^2) as one
                // sequence for both kinds of lanes (the draw first: no other draw precedes it)
                const bool miss = !cont && T.bestI < 0;
                // depth exhausted: contributes 0 (RayTracer.h:582-583)
                const bool scat = cont || (!miss && ++depth < P.maxDepth);
                float qx = 0.0f, qy = 0.0f, qz = 0.0f;
                float x = fdot(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz);
                bool drawn = true;
                if (scat) {
                    if (CAP && !P.rngTable) {
                        const float q2 = rius_capped<STATS>(rng, qx, qy, qz, pend, CAP, pc);
                        drawn = q2 >= 0.0f;
                        if (drawn) {
                            x = q2;
                            pend = 0;
                        }
                    } else {
                        x = rius<STATS>(rng, qx, qy, qz, pc, P.rngTable);
                    }
                }
                const float inv = rsqrt_rn(x);
                if (miss) sky_inv(r, inv, tr, tg, tb, Lr, Lg, Lb);
                if (scat && drawn) {
                    lambert_apply(r, T.bestT, T.bestI, shade, mats, qx, qy, qz, inv, tr, tg, tb);
                    fresh = true;
                }
                finished = !scat;
            } else if (T.bestI < 0) {
                sky(r, tr, tg, tb, Lr, Lg, Lb);
                finished = true;
            } else if (++depth >= P.maxDepth) {
                finished = true;  // depth exhausted: contributes 0 (RayTracer.h:582-583)
            } else if (scatter<FULL, STATS>(r, T.bestT, T.bestI, shade, tris, mats, rng, tr, tg, tb, pc,
                                            P.rngTable)) {
                fresh = true;
            } else {
                finished = true;  // absorbed: contributes 0 (RayTracer.h:590)
            }
            if (finished) {
                store_radiance(P.scratch, item, Lr, Lg, Lb);
                if (!CHAIN) ++samples;  // (CHAIN batches: every item is one sample, counted by the host)
#ifdef HIPPT_DEBUG_TIMELINE
                if (tlDrained) ++tlLate;
#endif
                item = kNone;
                need = true;
            }
        }
    }
    while (combLeft) combLeft = comb_step();
#ifdef HIPPT_DEBUG_RATE
    rt_flush(0);
#endif

#ifdef HIPPT_DEBUG_TIMELINE
    if (__lane_id() == 0 && tlw < 65536) {
        g_timeline[8 * tlw + 1] = tlDrained;
        g_timeline[8 * tlw + 2] = __builtin_amdgcn_s_memrealtime();
        g_timeline[8 * tlw + 3] = tlItems;
        g_timeline[8 * tlw + 6] = tlRounds;  // loop iterations after the wave saw the queues drained
        g_timeline[8 * tlw + 7] = tlLate;    // samples lane 0 finished after that
    }
#endif
    const unsigned long long segsW = CHAIN ? (unsigned long long)__builtin_amdgcn_readfirstlane(ww->segs) : wave_sum(segs);
    const unsigned long long samplesW = CHAIN ? 0ull : wave_sum(samples);
    if (STATS) {
        nvis = wave_sum(nvis);
        ntest = wave_sum(ntest);
    }
    unsigned long long *const st = stat_slot(P.stats);
    if (__lane_id() == 0) {
        atomicAdd(&st[0], segsW);
        atomicAdd(&st[1], samplesW);
        if (STATS) {
            atomicAdd(&st[2], nvis);
            atomicAdd(&st[3], ntest);
        }
    }
    if (STATS) {
#pragma unroll
        for (int k = 0; k < kProfSlots; ++k) {
            const unsigned long long v = wave_sum(pc[k]);
            if (__lane_id() == 0) atomicAdd(&st[4 + k], v);
        }
    }
}

// Running average in frame order, then ARGB (CudaPathTracerKernel.cu:157-178).
__global__ __launch_bounds__(256) void combine_kernel(CombineParams P, HostFrame H) {
    const unsigned stride = gridDim.x * 256u;
    for (unsigned p = blockIdx.x * 256u + threadIdx.x; p < P.bandPixels; p += stride) combine_pixel<8, true>(P, p, H);
}

// The chain's final combine (ChainFlushParams): every batch of the run no launch combined, in order.
__global__ __launch_bounds__(256) void chain_flush_kernel(ChainFlushParams P) {
    const int c0 = int(P.ctl[kChainCtlWord + 32u * ((P.epoch + 1u) & 1u)]);  // (written by an earlier launch)
    const int c1 = int(P.lastSeq);
    if (c1 < c0) return;
    const unsigned stride = gridDim.x * 256u;
    // whole waves per step (the audit's wave sums)
    for (unsigned base = blockIdx.x * 256u + (threadIdx.x & ~63u); base < P.comb.bandPixels; base += stride) {
        const unsigned p = base + __lane_id();
        const bool v = p < P.comb.bandPixels;
        if (v) combine_pixel_chain<8>(P.comb, P.scratch, p, c0, c1, P.slots, P.shift, P.step);
        if (P.audit)
            audit_combine(P.audit, c0, c1, unsigned(__popcll(__ballot(v))), wave_sum(v ? audit_hash(p) : 0ull), P.epoch,
                          P.comb.firstFrame, P.step);
    }
}

// table[s] for s = 0 .. 2^32-1: the state from which random_in_unit_sphere, entered with state s,
// draws the candidate it accepts (the loop of trace::rius, escape included).
__global__ __launch_bounds__(256) void rng_table_kernel(uint32_t *table, uint32_t base) {
    const uint32_t s0 = base + blockIdx.x * 256u + threadIdx.x;
    uint32_t s = s0;
    for (unsigned tries = 1;; ++tries) {
        const uint32_t from = s;
        const float x = rand_pm1(s), y = rand_pm1(s), z = rand_pm1(s);
        if (fmaf(x, x, fmaf(y, y, z * z)) < 1.0f) {
            table[s0] = from;
            return;
        }
        escape_cycle(s, tries);
    }
}

}  // namespace

hipError_t launch_rng_table(uint32_t *table, hipStream_t s) {
    // a grid dimension holds fewer than 2^32 work-items: 4 launches of 2^30 states
    for (uint32_t q = 0; q < 4; ++q) {
        hipLaunchKernelGGL(rng_table_kernel, dim3(1u << 22), dim3(256), 0, s, table, q << 30);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#ifdef HIPPT_DEBUG_TIMELINE
extern "C" int hipptDebugTimeline(unsigned long long *out, int maxWaves) {
    const int n = maxWaves < 65536 ? maxWaves : 65536;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_timeline), size_t(n) * 8 * sizeof(unsigned long long)) == hipSuccess
               ? n
               : -1;
}
#endif

#ifdef HIPPT_DEBUG_RATE
extern "C" int hipptDebugRate(unsigned long long *out, int reset) {
    static unsigned long long buf[kRateSlots * kRateBuckets * 5];
    if (out) {
        if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_rate), sizeof(buf)) != hipSuccess) return -1;
        for (int i = 0; i < kRateBuckets * 5; ++i) {
            unsigned long long v = 0;
            for (int k = 0; k < kRateSlots; ++k) v += buf[size_t(k) * kRateBuckets * 5 + i];
            out[i] = v;
        }
    }
    if (reset) {
        std::fill(buf, buf + kRateSlots * kRateBuckets * 5, 0ull);
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_rate), buf, sizeof(buf)) != hipSuccess) return -1;
    }
    return kRateBuckets;
}
#endif

hipError_t launch_sphere4(const Sphere4Params &p, hipStream_t s) {
    const long long n = (long long)p.rows * p.width;
    if (n <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n + 255) / 256);
    hipLaunchKernelGGL(sphere4_kernel, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// Stack: one spare slot per lane above the deepest level for the speculative far-child
// write; then (LDS_SCENE) the scene copy.
size_t mesh_lds_bytes(int stackDepth, int ldsNodes, int ldsTris, bool wide, unsigned topBytes, int ldsMats,
                      int poolWords) {
    return size_t(stackDepth + 1) * kMeshBlock * sizeof(int) +
           size_t(ldsNodes) * (wide ? kLdsNode4F4 : kLdsNodeF4) * 16 + size_t(ldsTris) * (3 + 1) * 16 + topBytes +
           size_t(ldsMats) * 2 * 16 +
           (poolWords ? (size_t(poolWords) * 64 + kWaveWords) * (kMeshBlock / 64) * sizeof(float) : 0);
}

size_t mesh_lds_scene_limit() { return 24u << 10; }

// waves a SIMD holds under the SGPR budget: 800 SGPRs per SIMD, 16 of them reserved per wave
// for the trap handler (one block = 4 waves = one wave per SIMD)
static constexpr int kMaxResidentBlocks = 800 / (HIPPT_NUM_SGPR + 16) < 8 ? 800 / (HIPPT_NUM_SGPR + 16) : 8;

// 160 KiB of LDS per CU shared by the resident blocks, in 512-byte allocation granules
size_t mesh_lds_block_budget() { return (size_t(160u << 10) / kMaxResidentBlocks) & ~size_t(511); }

using MeshFn = void (*)(MeshParams);
// node formats (MeshParams::wide): 2-wide, 4-wide float, 4-wide quantized, 4-wide hybrid (float
// top in LDS, quantized below it), 4-wide half planes; the last three are for global-memory trees only
// 4-wide trees whose stack bound fits the LDS capacity run a variant without the spill/refill
// code (timed builds; the counting builds keep one variant, the results are the same)
// (the camera-ray pool: 4-wide float-node kernels)
template <bool STATS, bool FULL, bool SPILL, bool POOL>
static MeshFn mesh_fn_wide(bool lds, int fmt) {
    if (lds) return mesh_kernel<STATS, true, FULL, true, false, SPILL, POOL>;
    if (fmt == kWideHybrid) return mesh_kernel<STATS, false, FULL, true, true, SPILL, false, true>;
    if (fmt == kWideHalf) return mesh_kernel<STATS, false, FULL, true, false, SPILL, POOL, false, true>;
    return fmt == kWideQuant ? mesh_kernel<STATS, false, FULL, true, true, SPILL>
                             : mesh_kernel<STATS, false, FULL, true, false, SPILL, POOL>;
}
template <bool STATS, bool FULL>
static MeshFn mesh_fn_fmt(bool lds, int fmt, bool spill, bool pool) {
    if (fmt == kWide2) return lds ? mesh_kernel<STATS, true, FULL, false, false> : mesh_kernel<STATS, false, FULL, false, false>;
    if (STATS || spill)
        return pool ? mesh_fn_wide<STATS, FULL, true, true>(lds, fmt) : mesh_fn_wide<STATS, FULL, true, false>(lds, fmt);
    return pool ? mesh_fn_wide<STATS, FULL, false, true>(lds, fmt) : mesh_fn_wide<STATS, FULL, false, false>(lds, fmt);
}
// chained batches (MeshParams::chainCtl): the timed camera-pool kernels over 4-wide float nodes
template <bool FULL, bool SPILL>
static MeshFn mesh_fn_chain(bool lds) {
    return lds ? mesh_kernel<false, true, FULL, true, false, SPILL, true, false, false, true>
               : mesh_kernel<false, false, FULL, true, false, SPILL, true, false, false, true>;
}
static MeshFn mesh_fn(bool count, bool lds, bool full, int fmt, bool spill, bool pool, bool chain = false) {
    if (chain) {
        if (count || fmt != kWideFloat || !pool) return nullptr;
        if (full) return spill ? mesh_fn_chain<true, true>(lds) : mesh_fn_chain<true, false>(lds);
        return spill ? mesh_fn_chain<false, true>(lds) : mesh_fn_chain<false, false>(lds);
    }
    if (count)
        return full ? mesh_fn_fmt<true, true>(lds, fmt, spill, pool) : mesh_fn_fmt<true, false>(lds, fmt, spill, pool);
    return full ? mesh_fn_fmt<false, true>(lds, fmt, spill, pool) : mesh_fn_fmt<false, false>(lds, fmt, spill, pool);
}

hipError_t launch_mesh(const MeshParams &p, int blocks, bool countTraversal, hipStream_t s) {
    if (p.stackDepth < 1 || p.stackDepth > kStackDepth) return hipErrorInvalidValue;
    if (p.wide && (p.stackCap < 1 || p.stackCap + 2 > p.stackDepth)) return hipErrorInvalidValue;
    const bool lds = p.ldsScene != 0;
    if (p.wide < kWide2 || p.wide > kWideHalf || (lds && p.wide >= kWideQuant)) return hipErrorInvalidValue;
    // the top of the tree: whole nodes of the LDS-read format (8-bit nodes only for kWideQuant)
    if (p.topBytes && (lds || p.wide == kWide2 || p.topBytes % (p.wide == kWideQuant ? 64u : 128u) ||
                       p.topBytes > (unsigned(p.numNodes) << (p.wide == kWideQuant ? 6 : 7))))
        return hipErrorInvalidValue;
    if (p.wide == kWideHybrid && !p.topBytes) return hipErrorInvalidValue;  // hybrid trees start in LDS
    if (lds && p.wide == kWideFloat && (p.refBits < 8 || p.refBits > 20)) return hipErrorInvalidValue;
    const bool pool = p.poolWords != 0;
    if (pool && ((p.wide != kWideFloat && p.wide != kWideHalf) || (p.poolWords != kPoolWordsPinhole && p.poolWords != kPoolWordsFull)))
        return hipErrorInvalidValue;
    const bool chain = p.chainCtl != nullptr;
    if (chain && (!p.chainBox || p.chainSlots < 2 || p.chainSlots > kChainSlotsMax || (p.chainSlots & (p.chainSlots - 1)) ||
                  p.chainShift > kChainMaxShift || p.totalItems > (1u << p.chainShift) || p.chainCap < 1 ||
                  p.chainCap >= p.chainSlots || p.chainPosted < p.chainSeq || p.chainPosted - p.chainSeq >= p.chainCap ||
                  p.chainGroup < 1 || p.chainGroup > p.chainCap || p.chainPosted - p.chainSeq + 1 < p.chainGroup ||
                  (p.chainGroup > 1 && p.totalItems % 64u) ||
                  p.comb.bandPixels != p.bandPixels || p.comb.frames != p.frames))
        return hipErrorInvalidValue;
    const size_t bytes = mesh_lds_bytes(p.stackDepth, lds ? p.numNodes : 0, lds ? p.numTris : 0, p.wide != 0, p.topBytes,
                                        lds ? p.numMats : 0, p.poolWords);
    if (pool && p.poolOffset != bytes - (size_t(p.poolWords) * 64 + kWaveWords) * (kMeshBlock / 64) * sizeof(float))
        return hipErrorInvalidValue;
    const MeshFn fn = mesh_fn(countTraversal, lds, p.full != 0, p.wide, p.spill != nullptr, pool, chain);
    if (!fn) return hipErrorInvalidValue;
    if (p.wide && (lds || p.topBytes || pool)) {
        const hipError_t e = check_lds_at_zero(reinterpret_cast<const void *>(fn));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(kMeshBlock), bytes, s, p);
    return hipGetLastError();
}

hipError_t launch_combine(const CombineParams &p, hipStream_t s, const HostFrame &h) {
    if (p.bandPixels == 0) return hipSuccess;
    unsigned blocks = (p.bandPixels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(combine_kernel, dim3(blocks), dim3(256), 0, s, p, h);
    return hipGetLastError();
}

hipError_t launch_chain_flush(const ChainFlushParams &p, hipStream_t s) {
    if (p.comb.bandPixels == 0) return hipSuccess;
    if (!p.ctl || p.slots < 2 || p.slots > kChainSlotsMax || (p.slots & (p.slots - 1)) || p.shift > kChainMaxShift)
        return hipErrorInvalidValue;
    unsigned blocks = (p.comb.bandPixels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(chain_flush_kernel, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

int mesh_blocks_per_cu(bool countTraversal, bool full, int fmt, int stackDepth, int ldsNodes, int ldsTris, bool spill,
                       unsigned topBytes, int ldsMats, int poolWords, bool chain) {
    int n = 0;
    const bool lds = ldsNodes > 0;
    const size_t bytes = mesh_lds_bytes(stackDepth, ldsNodes, ldsTris, fmt != kWide2, topBytes, ldsMats, poolWords);
    const MeshFn fn = mesh_fn(countTraversal, lds, full, lds && fmt >= kWideQuant ? kWideFloat : fmt, spill,
                              poolWords != 0, chain);
    if (!fn) return 1;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kMeshBlock, bytes);
    if (e != hipSuccess || n <= 0) n = 1;
    // the query ignores the trap handler's SGPRs (kMaxResidentBlocks): a larger persistent grid
    // leaves blocks waiting for a slot until others finish
    return std::min(n, kMaxResidentBlocks);
}

}  // namespace hippt
