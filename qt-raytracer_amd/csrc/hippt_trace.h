// hippt_trace.h — device building blocks of the mesh path tracer, shared by the megakernel
// (hippt_kernels.hip) and the wavefront kernels (hippt_wavefront.hip): RNG, camera ray,
// BVH traversal round, primitive tests, sky and material scatter.
//
// Arithmetic contract (oracle/pt_oracle.c): compiled with -ffp-contract=off; the only fused
// multiply-adds are the explicit fmaf() calls, placed where the oracle places them, and
// division/sqrt are IEEE correctly rounded (hipcc default), so every result-defining value is
// bit-identical to the CPU restatement.  The BVH box test is NOT result-defining (boxes are
// padded; the closest hit is argmin (t, primitive id)), so it uses the fast reciprocal.
#pragma once

#include "bvh_builder.h"
#include "hippt_chain_logic.h"
#include "hippt_device.h"

#pragma clang fp contract(off)

namespace hippt {
namespace trace {

constexpr unsigned kNone = 0xffffffffu;
constexpr int kDone = int(0x80000000);

__device__ __forceinline__ uint32_t hash32(uint32_t x) {  // CudaPathTracerKernel.cu:23-30
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float rand01(uint32_t &s) {  // :32-35 (÷4294967295.0f == ×2^-32)
    s = hash32(s);
    return float(s) * 0x1p-32f;
}

// 2*rand01 - 1 (fmaf(2, u, -1) of the contract) in one FMA: u = float(s)*2^-32 is an exact
// power-of-two scaling, so fmaf(float(s), 2^-31, -1) rounds the same exact value 2u - 1.
__device__ __forceinline__ float rand_pm1(uint32_t &s) {
    s = hash32(s);
    return fmaf(float(s), 0x1p-31f, -1.0f);
}

// Correctly rounded square root and reciprocal as short sequences (the IEEE expansions hipcc
// emits for sqrtf and 1.0f/x are 15 and 11 instructions: denormal scaling, class tests,
// v_div_scale/fmas/fixup).  Both are checked against hipcc's IEEE sqrtf / 1.0f/x on EVERY float
// bit pattern on gfx950 (tools/micro/rn_check.hip, tests/test_gpu_rounding.py):
//   sqrt_fix(x) == sqrtf(x)                   for every x except the denormals (x >= 2^-104)
//   rcp_nr(x)   == 1.0f / x                   for 2^-126 <= |x| < 2^126
//   rcp_nr(sqrt_fix(x)) == 1.0f / sqrtf(x)    for 2^-105 <= x < +inf
// v_sqrt_f32 is within one ulp, so the correctly rounded root is s or a neighbour, picked by
// the signs of the exact residuals x - s'*s (one fma each); v_rcp_f32 is within one ulp and one
// Newton step rounds correctly.
__device__ __forceinline__ float sqrt_fix(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = s;
    if (fmaf(-sm, s, x) <= 0.0f) r = sm;
    if (fmaf(-sp, s, x) > 0.0f) r = sp;
    return r;
}

__device__ __forceinline__ float rcp_nr(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, y, 1.0f), y, y);
}

// 1.0f / sqrtf(x), bit for bit, for any x: the short sequence inside its verified range, the IEEE
// expansion outside (a branch no lane takes for real rays: x = |d|^2 of a ray direction).
__device__ __forceinline__ float rsqrt_rn(float x) {
    if (x >= 0x1p-105f && x < INFINITY) return rcp_nr(sqrt_fix(x));
    return 1.0f / sqrtf(x);
}

// 1.0f / sqrtf(r2) for the unit-sphere draw's r2 = |p|^2 < 1: a coordinate 2u - 1 of the draw is
// 0 or at least 2^-24 in magnitude (u = float(s)*2^-32, float(s) a multiple of 128 near 2^31),
// so r2 is +0 or >= 2^-48 (a sum of squares, never -0), inside the verified range apart from +0
// (1/+0 = +inf).
__device__ __forceinline__ float rsqrt_unit_draw(float r2) {
    return r2 == 0.0f ? INFINITY : rcp_nr(sqrt_fix(r2));
}

// Short-cycle escape of the rejection loops (pt_oracle.c PO_ESCAPE).
__device__ __forceinline__ void escape_cycle(uint32_t &s, unsigned tries) {
    if ((tries & 63u) == 0u) s ^= 0x9E3779B9u;
}

__device__ __forceinline__ uint32_t pixel_seed(uint32_t x, uint32_t y, uint32_t w, uint32_t f) {
    return (x + y * w) * 9781u + (f + 1u) * 6271u;  // :144, uint32 wrap-around
}

__device__ __forceinline__ float fdot(float ax, float ay, float az, float bx, float by, float bz) {
    return fmaf(ax, bx, fmaf(ay, by, az * bz));
}

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

// This block's copy of the launch counters (kStatSlots).
__device__ __forceinline__ unsigned long long *stat_slot(unsigned long long *stats) {
    return stats + (blockIdx.x % unsigned(kStatSlots)) * unsigned(kStatWords);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// Wave-pooled grab from a global counter (see hippt_kernels.hip wave_fetch).  Whole wave,
// uniform control flow.
__device__ __forceinline__ unsigned wave_fetch(bool req, unsigned &poolNext, unsigned &poolEnd, unsigned *queue,
                                               unsigned chunk, unsigned total) {
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

// Work distribution of the persistent megakernel over items [0, total).  The items are split
// into kQueues contiguous queues, one per XCD (block b is dispatched to XCD b % 8), each with
// its counter on its own 128-byte line (queue[g * kQueueStride]).  A wave's first chunk is
// assigned statically (no atomic at kernel start, where all waves would contend), further
// chunks come from its home queue's counter, chunks shrink to kTailChunk items once the queue
// is within one chunk per wave of its end (a short tail), and a wave whose home queue is
// drained moves on to the others.  Counters start at 0 and count dynamically claimed items.
// (Claiming exactly the requesting lanes' count in the tail instead: neutral, DESIGN_LOG.md §A.1.)
#ifndef HIPPT_TAIL_CHUNK
#define HIPPT_TAIL_CHUNK 64
#endif
constexpr unsigned kQueues = kMeshQueues, kQueueStride = 32, kTailChunk = HIPPT_TAIL_CHUNK;

struct WorkQueue {
    unsigned g, left;  // current queue, queues not yet found drained
    unsigned next, end;  // this wave's pool [next, end) (all items of queue g)
    unsigned qEnd, dynBase, waves;  // queue g: end, first dynamically claimed item, home waves
};

__device__ __forceinline__ unsigned queue_start(unsigned total, unsigned g) {
    return unsigned((unsigned long long)total * g / kQueues);
}

__device__ __forceinline__ void queue_select(WorkQueue &Q, unsigned g, unsigned total, unsigned chunk) {
    Q.g = g;
    Q.qEnd = queue_start(total, g + 1);
    Q.waves = 4u * ((gridDim.x + kQueues - 1 - g) / kQueues);  // blocks b = g mod 8, 4 waves each
    Q.dynBase = queue_start(total, g) + Q.waves * chunk;
}

__device__ __forceinline__ void queue_begin(WorkQueue &Q, unsigned total, unsigned chunk) {
    queue_select(Q, blockIdx.x % kQueues, total, chunk);
    Q.left = kQueues;
    const unsigned wid = (blockIdx.x / kQueues) * 4u + (threadIdx.x >> 6);
    Q.next = min(queue_start(total, Q.g) + wid * chunk, Q.qEnd);
    Q.end = min(Q.next + chunk, Q.qEnd);
}

// A queue found drained, for the block (LDS word drained[t & 1] = t << 8 | one bit per queue of
// batch t), so that the block's other waves skip it: at a batch's end every wave otherwise learns
// each queue's end by one failing atomic on its counter, and those atomics serialise on the
// counter's line (~11 ns each, MI355X_MICROARCH.md "dequeue"): 7168 waves x 8 queues held a chained
// launch's waves ~50 us at each batch boundary (r5k rate timeline).
__device__ __forceinline__ void block_drained_set(unsigned *drained, unsigned t, unsigned g) {
    unsigned *const w = &drained[t & 1u];
    unsigned old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
        if ((old >> 8) > t) return;  // the word holds a later batch
        const unsigned nw = ((old >> 8) == t ? old : (t << 8)) | (1u << g);
        if (nw == old ||
            __hip_atomic_compare_exchange_strong(w, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            return;
    }
}

// One item per requesting lane (kNone once every queue is drained).  Whole wave, uniform
// control flow; the pool and queue state are wave-uniform.  stat: the queues have static first
// chunks (queue_begin); a chained batch a launch moves into has none (chain_select).  drained
// (camera-pool kernels): the block's drained-queue words (block_drained_set) for batch t.
__device__ __forceinline__ unsigned queue_fetch(bool req, WorkQueue &Q, unsigned *ctr, unsigned total,
                                                unsigned chunk, bool stat = true, unsigned *drained = nullptr,
                                                unsigned t = 0) {
    unsigned item = kNone;
    bool want = req;
    unsigned long long m = __ballot(want);
    unsigned rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
    unsigned avail = Q.end - Q.next;
    if (want && rank < avail) {
        item = Q.next + rank;
        want = false;
    }
    Q.next += min(unsigned(__popcll(m)), avail);
    while (Q.left && __ballot(want)) {
        m = __ballot(want);
        rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
        bool gone = false, got = false;
        if (drained) {
            const unsigned w = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&drained[t & 1u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            gone = (w >> 8) == t && ((w >> Q.g) & 1u);
        }
        if (!gone) {
            const unsigned c = Q.qEnd - min(Q.end, Q.qEnd) < Q.waves * chunk ? kTailChunk : chunk;
            unsigned base = 0;
            if (__lane_id() == 0) base = atomicAdd(&ctr[Q.g * kQueueStride], c);
            base = __builtin_amdgcn_readfirstlane(base) + Q.dynBase;
            if (base < Q.qEnd) {
                got = true;
                Q.next = base;
                Q.end = min(base + c, Q.qEnd);
                avail = Q.end - Q.next;
                if (want && rank < avail) {
                    item = Q.next + rank;
                    want = false;
                }
                Q.next += min(unsigned(__popcll(m)), avail);
            } else if (drained && __lane_id() == 0) {
                block_drained_set(drained, t, Q.g);
            }
        }
        if (!got && --Q.left) {
            queue_select(Q, Q.g + 1 == kQueues ? 0u : Q.g + 1, total, chunk);
            if (!stat) Q.dynBase = queue_start(total, Q.g);
            Q.next = Q.end = 0;
        }
    }
    return item;
}

// Wave-aggregated append of one entry per requesting lane to queue[] (one atomic per wave).
__device__ __forceinline__ void wave_append(bool req, unsigned value, unsigned *queue, unsigned *count) {
    const unsigned long long mask = __ballot(req);
    if (!mask) return;
    const unsigned n = unsigned(__popcll(mask));
    const unsigned rank = __builtin_amdgcn_mbcnt_hi(unsigned(mask >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(mask), 0u));
    const int leader = __ffsll((unsigned long long)mask) - 1;
    unsigned base = 0;
    if (int(__lane_id()) == leader) base = atomicAdd(count, n);
    base = __builtin_amdgcn_readlane(base, leader);
    if (req) queue[base + rank] = value;
}

// Phase profiling (STATS builds): pc[2k] counts wave-level passes of phase k (by the first
// active lane), pc[2k+1] lane-level passes; SIMD efficiency = lanes / (64 * waves).  Phases:
// 0 outer iteration, 1 camera ray, 2 traversal round, 3 interior node loop, 4 leaf loop,
// 5 primitive test, 6 shading, 7 unit-sphere rejection loop.  pc[kNhHist + h] (4-wide trees)
// counts node visits with h = 0..4 hit children; pc[kNhHist + 5] those with none hit only
// because of the closest hit found since the node was pushed (float 4-wide nodes); pc[kTopVisits]
// the visits served by the LDS copy of the top of a global-memory tree.
constexpr int kProfPhases = 8, kNhHist = 2 * kProfPhases, kTopVisits = kNhHist + 6, kProfSlots = kNhHist + 7;
template <bool STATS>
__device__ __forceinline__ void prof(unsigned *pc, int k) {
    if (STATS) {
        ++pc[2 * k + 1];
        if (__lane_id() == unsigned(__ffsll((unsigned long long)__ballot(1)) - 1)) ++pc[2 * k];
    }
}

struct Ray {
    float ox, oy, oz, dx, dy, dz;
    float ix, iy, iz, oix, oiy, oiz;  // box-test reciprocals (fast rcp; not result-defining)
};

__device__ __forceinline__ void prepare(Ray &r) {
    const float cx = copysignf(fmaxf(fabsf(r.dx), 1e-20f), r.dx);
    const float cy = copysignf(fmaxf(fabsf(r.dy), 1e-20f), r.dy);
    const float cz = copysignf(fmaxf(fabsf(r.dz), 1e-20f), r.dz);
    r.ix = __builtin_amdgcn_rcpf(cx);
    r.iy = __builtin_amdgcn_rcpf(cy);
    r.iz = __builtin_amdgcn_rcpf(cz);
    r.oix = r.ox * r.ix;
    r.oiy = r.oy * r.iy;
    r.oiz = r.oz * r.iz;
}

// A MeshParams field (the kernels' only argument, at kernarg offset 0) loaded where it is used: the
// opaque kernarg address keeps the compiler from loading it at kernel entry and holding it in
// registers (SGPRs, or VGPR lanes once those run out) across the whole kernel.  Taking the
// parameter's address instead would copy the whole block to scratch.
template <typename T>
__device__ __forceinline__ T late_arg_at(unsigned offset) {
    typedef const char __attribute__((address_space(4))) *KPtr;
    typedef const unsigned __attribute__((address_space(4))) *KWords;
    static_assert(sizeof(T) % 4 == 0, "whole words");
    KPtr k = (KPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    const KWords w = reinterpret_cast<KWords>(k + offset);
    T v;
    unsigned *d = reinterpret_cast<unsigned *>(&v);
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; ++i) d[i] = w[i];
    return v;
}

// MeshParams from `cam` through `rcpWidth`: the camera sample's and the item order's arguments.
// HIPPT_LATE_CAM builds load them where a wave generates camera rays (late_arg_at) instead of
// holding ~30 uniform values across the kernel.
struct CamArgs {
    CameraF cam;
    float invW, invH;
    int width, height, y0, bandRows, rowStride;
    int firstFrame, frames, maxDepth;
    unsigned bandPixels, totalItems;
    float rcpBandPixels, rcpWidth;
};
static_assert(offsetof(MeshParams, rcpWidth) - offsetof(MeshParams, cam) == offsetof(CamArgs, rcpWidth),
              "CamArgs mirrors MeshParams");
__device__ __forceinline__ CamArgs cam_args_late() { return late_arg_at<CamArgs>(unsigned(offsetof(MeshParams, cam))); }

// Camera sample for work item `it`: RenderWorker::render u/v (RayTracerFboItem.cpp:109-110) and
// Camera::get_ray (RayTracer.h:563-567, disk draw always consumed).
// The work item at queue position `it` (MeshParams::runOrder, item_order.h build_item_table):
// the 64-item slot of (frame, run) handed out as the slot the table names, the offset within
// the run kept; positions outside whole runs and kNone stay as they are.
// A table entry's item k: consecutive band pixels, or (flag bit 31, item_order.h kRunTile) column
// k mod 2^tileShift, band row k >> tileShift of a tile.
__device__ __forceinline__ unsigned run_item(unsigned v, unsigned k, unsigned width, unsigned tileShift) {
    return (v & 0x7fffffffu) + ((v >> 31) ? (k & ((1u << tileShift) - 1u)) + (k >> tileShift) * width : k);
}

__device__ __forceinline__ unsigned order_item(const MeshParams &P, unsigned it) {
    if (it == kNone || !P.runOrder) return it;
    unsigned fl, q;
    divmod(it, P.bandPixels, P.rcpBandPixels, fl, q);
    const unsigned run = q >> 6;
    return run < P.runCount ? run_item(P.runOrder[fl * P.runCount + run], q & 63u, unsigned(P.width), P.runTileShift)
                            : it;
}

// order_item with its arguments loaded where it runs (HIPPT_LATE_CAM)
__device__ __forceinline__ unsigned order_item_late(unsigned it) {
    if (it == kNone) return it;
    const unsigned *order = late_arg_at<const unsigned *>(unsigned(offsetof(MeshParams, runOrder)));
    if (!order) return it;
    const CamArgs A = cam_args_late();
    const unsigned runs = late_arg_at<unsigned>(unsigned(offsetof(MeshParams, runCount)));
    unsigned fl, q;
    divmod(it, A.bandPixels, A.rcpBandPixels, fl, q);
    const unsigned run = q >> 6;
    return run < runs ? run_item(order[fl * runs + run], q & 63u, unsigned(A.width),
                                 late_arg_at<unsigned>(unsigned(offsetof(MeshParams, runTileShift))))
                      : it;
}

// ---- chained batches (MeshParams::chain*, CHAIN kernels) ----------------------------
// A launch whose batch is drained goes on with the batches of its run the host has posted behind it,
// so that a run of batches pays the launch's tail (the last paths finishing at falling lane use,
// ~0.2-0.3 ms) once per chainCap batches instead of once per batch; batches that arrive while the
// run's last launch has not started are held on the host and launched as one group
// (MeshParams::chainGroup: the launch's own batches, one set of queues over their items).  The rules
// that keep it exact:
//  * a launch starts after the previous one on the stream has ended, so every batch before its own
//    is finished, and so is every batch an earlier launch moved into (a wave leaves a batch only once
//    all of its queues are drained, and a launch ends only when its waves have finished their paths):
//    an earlier launch's marker in the batch's ring slot says so;
//  * a launch combines (running average + tonemap, in frame order per pixel) every finished batch not
//    yet combined, [c0, c1], beside its own tracing (the fused combine of one batch before), and
//    records c1 + 1 for the next launch (by epoch parity: the next launch reads it, this one's late
//    waves do not see it);
//  * it traces from u = c1 + 1 (its own batch or group when no earlier launch took it: the first
//    chunks then static, as unchained) up to min(c0 + slots - 1, u + chainCap - 1), so that it never
//    writes a ring slot it combines or one a batch not yet combined holds; the host posts a batch
//    launched on its own in the mailbox before its launch is enqueued, never a held one, and a launch
//    takes a later batch only once the mailbox shows it;
//  * the counters of the slots it combines are zeroed at its start for the batches that reuse them
//    (no wave of the launch reads them: it traces only past c1);
//  * the run's last combines are the final flush (launch_chain_flush), before anything reads or
//    resets the image, and a new run starts from a zeroed control block.
// Per wave, in LDS (WaveWords::cw):
struct ChainWave {
    unsigned t;         // the batch the wave's queue serves (its items carry its ring slot above chainShift)
    unsigned spare;
    unsigned tLim;      // the last batch this launch may trace
    unsigned posted;    // batches before this one are known posted
    int step;           // frames from one batch to the next (-1: not known yet)
    unsigned c0, c1;    // this launch's combine range (c1 < c0: none)
    unsigned stat;      // the own batch (group) whose queues have static first chunks (~0u: none)
};

// The block's view of the mailbox (in its first wave's WaveWords; chain_next): batches up to `last`
// are posted (frames apart when `consec`; none after them when `closed`: the host is on a later run),
// as learnt at `stamp` (low 32 bits of the 100 MHz clock) by the block's querier; `busy` while one
// wave asks the device copy for the block, so that the block's other waves wait in LDS.
struct ChainView {
    unsigned last;
    unsigned flags;  // bit 0: consecutive frames; bit 1: closed
    unsigned stamp;
    unsigned busy;
};

#define late_field(f) late_arg_at<decltype(MeshParams::f)>(unsigned(offsetof(MeshParams, f)))

// The camera-pool kernels' per-wave state kept in LDS between uses, kWaveWords words at the start of
// each wave's pool block: the work queue (read and written back at each pool refill, once per 64
// items), the wave's segment count and the chain state.  In registers they would be live across the
// whole path loop, which has none to spare: the loop's peak is the node visit with every lane's path
// state live, and the chained kernels spilled the path throughput to scratch until these moved out.
struct WaveWords {
    WorkQueue Q;
    unsigned segs;
    ChainWave cw;
    ChainView view;       // (the block's first wave's only)
    unsigned drained[2];  // (the block's first wave's only: queue_fetch's block_drained_set words)
};
static_assert(sizeof(WaveWords) == kWaveWords * 4, "per-wave LDS words");

__device__ __forceinline__ WorkQueue load_queue(const WorkQueue *q) {
    WorkQueue Q;
    Q.g = __builtin_amdgcn_readfirstlane(q->g);
    Q.left = __builtin_amdgcn_readfirstlane(q->left);
    Q.next = __builtin_amdgcn_readfirstlane(q->next);
    Q.end = __builtin_amdgcn_readfirstlane(q->end);
    Q.qEnd = __builtin_amdgcn_readfirstlane(q->qEnd);
    Q.dynBase = __builtin_amdgcn_readfirstlane(q->dynBase);
    Q.waves = __builtin_amdgcn_readfirstlane(q->waves);
    return Q;
}
__device__ __forceinline__ void store_queue(WorkQueue *q, const WorkQueue &Q) {
    if (__lane_id() == 0) *q = Q;
}

__device__ __forceinline__ unsigned *chain_block(unsigned *ctl, unsigned t, unsigned slots) {
    return ctl + (t & (slots - 1u)) * kChainBlockWords;
}

// Cross-launch words (markers, the combined-through word, counter resets) are plain loads and stores:
// a launch reads only what earlier launches wrote (the kernel boundary writes the L2s back and
// invalidates them), and every wave of a launch writes the same value.  Uncached (agent-scope) loads
// of one line by every wave of a launch serialise at the memory side: ~0.3 ms per launch (r5g).

// Batch t taken by launch `epoch` (lane 0; every wave that moves into t stores the same word).
__device__ __forceinline__ void chain_mark(unsigned *ctl, unsigned t, unsigned slots, unsigned epoch) {
    if (__lane_id() == 0)
        *reinterpret_cast<unsigned long long *>(chain_block(ctl, t, slots) + kChainMarkerWord) = chain::marker(t, epoch);
}

// queue_select for a batch with (stat) or without static first chunks
__device__ __forceinline__ void chain_select(WorkQueue &Q, unsigned g, unsigned total, unsigned chunk, bool stat) {
    queue_select(Q, g, total, chunk);
    if (!stat) Q.dynBase = queue_start(total, g);
}

// Kernel start of a CHAIN launch (whole wave): the combine range, the first batch to trace and the
// wave's queue (static first chunk when that batch is the launch's own), state into *cw; the block's
// first wave also initialises the block's mailbox view.
__device__ __forceinline__ void chain_begin(WorkQueue &Q, ChainWave *cw, ChainView *view) {
    unsigned *const ctl = late_field(chainCtl);
    const unsigned e = late_field(chainEpoch), own = late_field(chainSeq), R = late_field(chainSlots);
    const unsigned posted = late_field(chainPosted);
    const unsigned total = late_field(totalItems), chunk = late_field(chunk), group = late_field(chainGroup);
    // the first batch not combined by an earlier launch (written at the previous launch's start)
    const unsigned c0 = __builtin_amdgcn_readfirstlane(ctl[kChainCtlWord + 32u * ((e + 1u) & 1u)]);
    // lane k: batch t0 + k finished by an earlier launch (its slot's marker), within the ring's window
    const unsigned t0 = chain::begin_t0(c0, own);
    bool fin = false;
    if (chain::begin_lane_in_window(__lane_id(), t0, c0, R)) {
        const unsigned t = t0 + __lane_id();
        fin = chain::marker_finished(
            *reinterpret_cast<const unsigned long long *>(chain_block(ctl, t, R) + kChainMarkerWord), t, e);
    }
    const unsigned nfin = unsigned(__builtin_ctzll(~__ballot(fin)));
    const chain::BeginPlan plan = chain::begin_plan(c0, own, nfin, R, late_field(chainCap));
    const int c1 = plan.c1;
    const unsigned u = plan.u, tLim = plan.tLim;
    const int step = late_field(chainStep);
    if (__lane_id() == 0) {
        cw->c0 = c0;
        cw->c1 = unsigned(c1);
        cw->tLim = tLim;
        cw->posted = posted + 1u;  // posted before the launch was enqueued
        cw->step = step;
        cw->t = u == own ? own : u - 1u;
        cw->stat = u == own ? own : ~0u;
        if (threadIdx.x == 0) {
            view->last = posted;
            view->flags = chain::view_flags_at_start(step);
            view->stamp = 0;
            view->busy = 0;
        }
    }
    if (u == own) {  // the own batch (group), untaken: first chunks static, as unchained
        if (__lane_id() < group)
            *reinterpret_cast<unsigned long long *>(chain_block(ctl, own + __lane_id(), R) + kChainMarkerWord) =
                chain::marker(own + __lane_id(), e);
        queue_begin(Q, total * group, chunk);
    } else {  // nothing to fetch: the wave's first refill moves it into batch u (chain_next)
        Q.left = 0;
        Q.next = Q.end = 0;
    }
    // this launch's bookkeeping for the next (block 0's first wave): the first batch not combined
    // after this launch (its combines are done by its end), the next epoch's combine counter, and
    // the work counters of the slots combined here (the counters of their next batches)
    if (blockIdx.x == 0 && threadIdx.x < 64u) {
        if (__lane_id() == 0) {
            ctl[kChainCtlWord + 32u * (e & 1u)] = chain::begin_next_c0(c0, c1);
            ctl[kChainCtlWord + 64u + 32u * ((e + 1u) & 1u)] = 0u;
        }
        for (int b = int(c0); b <= c1; ++b)
            if (__lane_id() < kQueues) chain_block(ctl, unsigned(b), R)[__lane_id() * kQueueStride] = 0u;
    }
}

// Is batch nt posted?  (lane 0 of a wave; out: the last batch known posted and the view's flags.)
// The mailbox (one 64-bit word: run << 33 | consecutive frames << 32 | last posted batch) is host
// memory read over PCIe, where reads serialise (~60 ns each: 7168 waves reaching their batch's end
// together waited 0.43-1.1 ms, r5d/r5e), and uncached loads of one device line serialise too (~20 ns:
// every wave asking a device-wide copy cost ~130 us per launch, r5i).  So three levels, each asked
// by one wave for many: the block's view in LDS (one querier per block, the others wait in LDS), a
// per-XCD device copy (one 64-bit word: its refresh stamp, closed, consecutive, last batch) that a
// querier finding it older than kBoxRefresh refreshes from the host after winning a claim, and the
// host word.  A querier that loses the claim sleeps (no memory traffic) for the winner's refresh,
// then reads the copy once more.  Stale answers only ever say "not yet posted": a wave then stops
// taking batches, and a later launch traces them.
__device__ __forceinline__ void chain_ask(unsigned nt, ChainView *view, unsigned &last, unsigned &flags) {
    constexpr unsigned long long kBoxRefresh = 1000;  // 10 us of the 100 MHz clock
    constexpr unsigned kViewRefresh = 500, kWaitBusy = 20000;
    const unsigned t0 = unsigned(__builtin_amdgcn_s_memrealtime());
    for (;;) {
        last = __hip_atomic_load(&view->last, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        flags = __hip_atomic_load(&view->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned st = __hip_atomic_load(&view->stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned now32 = unsigned(__builtin_amdgcn_s_memrealtime());
        if (nt <= last || (flags & chain::kClosed) || (st != 0u && now32 - st < kViewRefresh)) return;
        unsigned idle = 0u;
        if (__hip_atomic_compare_exchange_strong(&view->busy, &idle, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
            break;  // this wave asks for the block
        // another wave of the block is asking: wait for its answer (bounded), then take the view
        while (__hip_atomic_load(&view->busy, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u &&
               unsigned(__builtin_amdgcn_s_memrealtime()) - t0 < kWaitBusy)
            __builtin_amdgcn_s_sleep(2);
        last = __hip_atomic_load(&view->last, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        flags = __hip_atomic_load(&view->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    // the view's only writer now (busy): merge into what it holds at this point, not into the words
    // read before the claim, which another querier may have advanced since
    last = __hip_atomic_load(&view->last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    flags = __hip_atomic_load(&view->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned long long *const box = reinterpret_cast<unsigned long long *>(late_field(chainCtl) + kChainBoxWord +
                                                                          (blockIdx.x % kQueues) * 32u);
    unsigned long long *const copy = box, *const claim = box + 1;
    const unsigned run = late_field(chainRun);
    // the copy and the claim carry the launch (epoch mod 64) that made them: a copy made by an earlier
    // launch says nothing about batches posted since, and chain_batch posts batches without a launch
    // of their own only before the launch that is to take them starts (so its negative must be fresh).
    // (A copy 64 launches old that looks fresh only says "not posted" or "open": view_merge never
    // lowers what the view knows.)
    const unsigned ep = late_field(chainEpoch) & 63u;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    unsigned long long c = __hip_atomic_load(copy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned age = (unsigned(now >> 4) - unsigned(c >> 40)) & 0xffffffu;  // in 16-tick units
    const bool ours = (unsigned(c >> 34) & 63u) == ep;
    if (chain::copy_last(c) < nt && !chain::copy_closed(c) && (!ours || age >= kBoxRefresh / 16u)) {
        const unsigned long long prev = __hip_atomic_load(claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool active = (unsigned(prev) & 63u) == ep && now - (prev & ~63ull) < kBoxRefresh;
        if (!active && atomicCAS(claim, prev, (now & ~63ull) | ep) == prev) {  // this wave refreshes
            const unsigned long long h =
                __hip_atomic_load(late_field(chainBox), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            c = chain::copy_pack(__builtin_amdgcn_s_memrealtime(), h, run, ep);
            __hip_atomic_store(copy, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {  // a refresh is in flight (claimed at most kBoxRefresh ago): give it 4 us, read once more
            while (__builtin_amdgcn_s_memrealtime() - now < 400u) __builtin_amdgcn_s_sleep(8);
            c = __hip_atomic_load(copy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    chain::view_merge(last, flags, c);
    __hip_atomic_store(&view->flags, flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&view->last, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&view->stamp, max(unsigned(__builtin_amdgcn_s_memrealtime()), 1u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&view->busy, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A wave whose batch is drained moves into the next batch of the run, if this launch may take it and
// the mailbox shows it posted (whole wave; at a camera-pool refill, so that the lanes whose paths
// ended take the next batch's items while the others go on with theirs).
__device__ __forceinline__ bool chain_next(WorkQueue &Q, ChainWave *cw, ChainView *view) {
    // (the own group's queue, ChainWave::stat, is followed by the batch after the group)
    const unsigned t = __builtin_amdgcn_readfirstlane(cw->t);
    const unsigned nt = chain::next_batch(t, __builtin_amdgcn_readfirstlane(cw->stat), late_field(chainGroup));
    if (nt > __builtin_amdgcn_readfirstlane(cw->tLim)) return false;
    int step = int(__builtin_amdgcn_readfirstlane(unsigned(cw->step)));
    if (nt >= __builtin_amdgcn_readfirstlane(cw->posted)) {
        unsigned last = 0, flags = 0;
        if (__lane_id() == 0) chain_ask(nt, view, last, flags);
        last = __builtin_amdgcn_readfirstlane(last);
        flags = __builtin_amdgcn_readfirstlane(flags);
        // not (yet) posted, the run closed before it, or its frame pattern not known here
        if (!chain::view_takes(nt, last, flags, late_field(frames), step)) return false;
        if (__lane_id() == 0) {
            cw->posted = last + 1u;
            cw->step = step;
        }
    }
    unsigned *const ctl = late_field(chainCtl);
    const unsigned R = late_field(chainSlots);
    if (__lane_id() == 0) cw->t = nt;
    chain_mark(ctl, nt, R, late_field(chainEpoch));
    chain_select(Q, blockIdx.x % kQueues, late_field(totalItems), late_field(chunk), false);
    Q.left = kQueues;
    Q.next = Q.end = 0;
    return true;
}

// ---- chained-batch audit (MeshParams::chainAudit, HIPPT_OPT_CHAIN_AUDIT) --------------------------
// Order-free summaries the host compares with what the run should have done (tests/chain_audit.py):
// counts and 64-bit sums of a hash of the item / pixel indices, and min/max (as max of ~v) of the
// frames and launches involved.
__device__ __forceinline__ unsigned audit_hash(unsigned i) { return hash32(i ^ 0x5bd1e995u); }
__device__ __forceinline__ unsigned *audit_record(unsigned *audit, unsigned t) {
    return audit + min(t, kAuditBatches) * kAuditWords;
}
// one traced item (per lane, at the refill that generates its camera ray): its batch, index, the
// first frame it was traced with and the launch.  Per-lane atomics: a wave-aggregated version costs
// the chained kernels scratch spills in the refill (the audit is a testing aid; its atomics contend)
__device__ __forceinline__ void audit_trace(unsigned *audit, unsigned t, unsigned item, unsigned frame,
                                            unsigned epoch) {
    unsigned *const r = audit_record(audit, t);
    atomicAdd(r, 1u);
    atomicAdd(reinterpret_cast<unsigned long long *>(r + 2), (unsigned long long)audit_hash(item));
    atomicMax(r + 6, frame + 1u);
    atomicMax(r + 7, ~frame);
    atomicMax(r + 8, epoch + 1u);
    atomicMax(r + 9, ~epoch);
}
// a wave's combine of `n` pixels (hash sum hsum) over batches [c0, c1] (lane 0)
__device__ __forceinline__ void audit_combine(unsigned *audit, int c0, int c1, unsigned n, unsigned long long hsum,
                                              unsigned epoch, int firstFrame, int step) {
    if (__lane_id() != 0 || n == 0u) return;
    for (int b = c0; b <= c1; ++b) {
        unsigned *const r = audit_record(audit, unsigned(b));
        const unsigned f0 = unsigned(firstFrame + b * step);
        atomicAdd(r + 1, n);
        atomicAdd(reinterpret_cast<unsigned long long *>(r + 4), hsum);
        atomicMax(r + 10, epoch + 1u);
        atomicMax(r + 11, ~epoch);
        atomicMax(r + 12, f0 + 1u);
        atomicMax(r + 13, ~f0);
    }
}

// PP: MeshParams or CamArgs.  frameAdd: a chained batch's frame offset from the launch's own frames.
template <typename PP>
__device__ __forceinline__ void camera_sample(const PP &P, unsigned it, Ray &r, uint32_t &rng, unsigned frameAdd = 0u) {
    unsigned fl, p, yb, x;
    divmod(it, P.bandPixels, P.rcpBandPixels, fl, p);
    divmod(p, unsigned(P.width), P.rcpWidth, yb, x);
    const unsigned y = unsigned(P.y0) + yb * unsigned(P.rowStride);
    rng = pixel_seed(x, y, unsigned(P.width), unsigned(P.firstFrame) + fl + frameAdd);
    const float s = (float(x) + rand01(rng)) * P.invW;
    const float t = (float(y) + rand01(rng)) * P.invH;
    float qx, qy;
    for (unsigned tries = 1;; ++tries) {  // random_in_unit_disk, RayTracer.h:163-169
        qx = rand_pm1(rng);
        qy = rand_pm1(rng);
        if (fmaf(qx, qx, qy * qy) < 1.0f) break;
        escape_cycle(rng, tries);
    }
    const CameraF &C = P.cam;
    const float rx = C.lens_radius * qx, ry = C.lens_radius * qy;
    const float fx = fmaf(C.v[0], ry, C.u[0] * rx);
    const float fy = fmaf(C.v[1], ry, C.u[1] * rx);
    const float fz = fmaf(C.v[2], ry, C.u[2] * rx);
    r.ox = C.origin[0] + fx;
    r.oy = C.origin[1] + fy;
    r.oz = C.origin[2] + fz;
    r.dx = (fmaf(t, C.vertical[0], fmaf(s, C.horizontal[0], C.llc[0])) - C.origin[0]) - fx;
    r.dy = (fmaf(t, C.vertical[1], fmaf(s, C.horizontal[1], C.llc[1])) - C.origin[1]) - fy;
    r.dz = (fmaf(t, C.vertical[2], fmaf(s, C.horizontal[2], C.llc[2])) - C.origin[2]) - fz;
}

// A finished sample's radiance: one 12-byte store (one vector-memory instruction; three planes
// cost three, and the store instructions of lanes finishing at different times dominated the
// address unit's load on LDS-resident scenes).
__device__ __forceinline__ void store_radiance(float *scratch, unsigned item, float r, float g, float b) {
    *reinterpret_cast<float3 *>(scratch + 3 * size_t(item)) = make_float3(r, g, b);
}

// Sky gradient on a miss (RayTracer.h:593-595), times throughput; `inv` = 1/sqrtf(|d|^2).
__device__ __forceinline__ void sky_inv(const Ray &r, float inv, float tr, float tg, float tb, float &L0, float &L1,
                                        float &L2) {
    const float uy = inv * r.dy;
    const float al = 0.5f * (uy + 1.0f);
    const float bl = 1.0f - al;
    L0 = tr * fmaf(al, 0.5f, bl);
    L1 = tg * fmaf(al, 0.7f, bl);
    L2 = tb * fmaf(al, 1.0f, bl);
}

__device__ __forceinline__ void sky(const Ray &r, float tr, float tg, float tb, float &L0, float &L1, float &L2) {
    const float uy = rsqrt_rn(fdot(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz)) * r.dy;
    const float al = 0.5f * (uy + 1.0f);
    const float bl = 1.0f - al;
    L0 = tr * fmaf(al, 0.5f, bl);
    L1 = tg * fmaf(al, 0.7f, bl);
    L2 = tb * fmaf(al, 1.0f, bl);
}

// random_in_unit_sphere (RayTracer.h:155-161; x, y, z drawn in that order).  With `table`
// (launch_rng_table) the rejection loop is one lookup: the state the accepted candidate is
// drawn from, then its three draws — the same draws, hence the same bits, without the loop
// whose SIMD tail (a wave loops until its unluckiest lane accepts) runs at 19% lane utilization.
// Measured (r2zd): Cornell -3%, blob70k -18%, random_scene -8%, cornell_mixed +8% — the random
// 4-byte reads over 16 GiB cost more than the loop's tail; loading the entry when the segment's
// ray starts (latency behind the traversal) was worse still (Cornell -15%).  Off by default.
template <bool STATS>
__device__ __forceinline__ float rius(uint32_t &rng, float &rx, float &ry, float &rz, unsigned *pc,
                                      const uint32_t *table = nullptr) {
    if (table) {
        prof<STATS>(pc, 7);
        rng = table[rng];
        rx = rand_pm1(rng);
        ry = rand_pm1(rng);
        rz = rand_pm1(rng);
        return fmaf(rx, rx, fmaf(ry, ry, rz * rz));
    }
    float r2;
    for (unsigned tries = 1;; ++tries) {
        prof<STATS>(pc, 7);
        rx = rand_pm1(rng);
        ry = rand_pm1(rng);
        rz = rand_pm1(rng);
        r2 = fmaf(rx, rx, fmaf(ry, ry, rz * rz));
        if (r2 < 1.0f) break;
        escape_cycle(rng, tries);
    }
    return r2;
}

// The same draw in at most `cap` tries per call: `tries` (persistent, 0 before the first try)
// continues the lane's chain across calls, so the draws and the escape points are rius's.
// Returns |p|^2 once a candidate is accepted, -1 while the draw is still pending.
template <bool STATS>
__device__ __forceinline__ float rius_capped(uint32_t &rng, float &rx, float &ry, float &rz, unsigned &tries,
                                             unsigned cap, unsigned *pc) {
    for (unsigned k = 0; k < cap; ++k) {
        prof<STATS>(pc, 7);
        rx = rand_pm1(rng);
        ry = rand_pm1(rng);
        rz = rand_pm1(rng);
        const float r2 = fmaf(rx, rx, fmaf(ry, ry, rz * rz));
        ++tries;
        if (r2 < 1.0f) return r2;
        escape_cycle(rng, tries);
    }
    return -1.0f;
}

// Scatter at the closest hit (ray_color :585-590 + the material's scatter, :473-540) of
// primitive `prim` at t.  The ray becomes the scattered ray and the throughput takes the
// attenuation; false = absorbed (Metal below the surface), which contributes 0.  FULL=false
// is the Lambertian-triangle specialisation (no sphere normals, no material dispatch).
template <bool FULL, bool STATS>
__device__ __forceinline__ bool scatter(Ray &r, float t, int prim, const float4 *shade, const float4 *prims,
                                        const float4 *mats, uint32_t &rng, float &tr, float &tg, float &tb,
                                        unsigned *pc, const uint32_t *rngTable = nullptr) {
    const float4 sh = shade[prim];
    const int mw = __float_as_int(sh.w);
    const float px = fmaf(t, r.dx, r.ox), py = fmaf(t, r.dy, r.oy), pz = fmaf(t, r.dz, r.oz);  // Ray::at
    float nx = sh.x, ny = sh.y, nz = sh.z;
    if (FULL && (mw & kShadeSphere)) {  // (p - center) / radius, :308
        const float rad = prims[3 * prim].w;
        nx = (px - sh.x) / rad;
        ny = (py - sh.y) / rad;
        nz = (pz - sh.z) / rad;
    }
    const bool front = fdot(r.dx, r.dy, r.dz, nx, ny, nz) < 0.0f;  // set_face_normal, :215-218
    if (!front) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
    const int m = FULL ? (mw & ~kShadeSphere) : mw;
    const float4 m0 = mats[2 * m];
    float sx, sy, sz;
    const int kind = FULL ? __float_as_int(m0.w) : int(kLambertian);
    if (kind == kMetal) {  // Metal::scatter, :496-501
        const float fuzz = mats[2 * m + 1].x;
        const float il = rsqrt_rn(fdot(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz));
        const float ux = r.dx * il, uy = r.dy * il, uz = r.dz * il;
        const float k = 2.0f * fdot(ux, uy, uz, nx, ny, nz);  // reflect, :174-176
        float qx, qy, qz;
        rius<STATS>(rng, qx, qy, qz, pc, rngTable);
        sx = (ux - k * nx) + fuzz * qx;
        sy = (uy - k * ny) + fuzz * qy;
        sz = (uz - k * nz) + fuzz * qz;
        if (!(fdot(sx, sy, sz, nx, ny, nz) > 0.0f)) return false;
        tr *= m0.x;
        tg *= m0.y;
        tb *= m0.z;
    } else if (kind == kDielectric) {  // Dielectric::scatter, :512-530 (attenuation 1)
        const float ir = mats[2 * m + 1].y;
        const float ratio = front ? (1.0f / ir) : ir;
        const float il = rsqrt_rn(fdot(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz));
        const float ux = r.dx * il, uy = r.dy * il, uz = r.dz * il;
        const float cosT = fminf(fdot(-ux, -uy, -uz, nx, ny, nz), 1.0f);
        const float sinT = sqrtf(1.0f - cosT * cosT);
        bool refl = ratio * sinT > 1.0f;
        if (!refl) {  // Schlick (:533-538) > random_double(), drawn only when refraction is possible
            float r0 = (1.0f - ratio) / (1.0f + ratio);
            r0 = r0 * r0;
            const float x = 1.0f - cosT, x2 = x * x;
            refl = r0 + (1.0f - r0) * (x2 * x2 * x) > rand01(rng);
        }
        if (refl) {
            const float k = 2.0f * fdot(ux, uy, uz, nx, ny, nz);
            sx = ux - k * nx;
            sy = uy - k * ny;
            sz = uz - k * nz;
        } else {  // refract, :178-183
            const float qx = (ux + cosT * nx) * ratio, qy = (uy + cosT * ny) * ratio, qz = (uz + cosT * nz) * ratio;
            const float par = -sqrtf(fabsf(1.0f - fdot(qx, qy, qz, qx, qy, qz)));
            sx = qx + par * nx;
            sy = qy + par * ny;
            sz = qz + par * nz;
        }
    } else {  // Lambertian::scatter, :477-484: n + unit(random_in_unit_sphere), 1e-8 fallback
        float qx, qy, qz;
        const float r2 = rius<STATS>(rng, qx, qy, qz, pc, rngTable);
        const float inv = rsqrt_unit_draw(r2);  // unit_vector = (1/len)*v, :137-139,151-153
        sx = nx + qx * inv;
        sy = ny + qy * inv;
        sz = nz + qz * inv;
        if (fdot(sx, sy, sz, sx, sy, sz) < 1e-8f) {
            sx = nx;
            sy = ny;
            sz = nz;
        }
        tr *= m0.x;
        tg *= m0.y;
        tb *= m0.z;
    }
    r.ox = px;
    r.oy = py;
    r.oz = pz;
    r.dx = sx;
    r.dy = sy;
    r.dz = sz;
    return true;
}

// Lambertian scatter at a triangle hit (the FULL=false part of scatter() after its unit-sphere
// draw q, |q|^2 = r2, inv = 1/sqrtf(r2)): the megakernel computes the draw first and shares one
// 1/sqrt sequence between the lanes that scatter and those that take the sky.
__device__ __forceinline__ void lambert_apply(Ray &r, float t, int prim, const float4 *shade, const float4 *mats,
                                              float qx, float qy, float qz, float inv, float &tr, float &tg,
                                              float &tb) {
    const float4 sh = shade[prim];
    const int m = __float_as_int(sh.w);
    const float px = fmaf(t, r.dx, r.ox), py = fmaf(t, r.dy, r.oy), pz = fmaf(t, r.dz, r.oz);  // Ray::at
    float nx = sh.x, ny = sh.y, nz = sh.z;
    if (!(fdot(r.dx, r.dy, r.dz, nx, ny, nz) < 0.0f)) {  // set_face_normal, :215-218
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
    const float4 m0 = mats[2 * m];
    float sx = nx + qx * inv, sy = ny + qy * inv, sz = nz + qz * inv;  // :477-484
    if (fdot(sx, sy, sz, sx, sy, sz) < 1e-8f) {
        sx = nx;
        sy = ny;
        sz = nz;
    }
    tr *= m0.x;
    tg *= m0.y;
    tb *= m0.z;
    r.ox = px;
    r.oy = py;
    r.oz = pz;
    r.dx = sx;
    r.dy = sy;
    r.dz = sz;
}

// Sphere::hit (RayTracer.h:289-314) root selection in the contract's FP32 form
// (pt_oracle.c po_sphere_t: precision-robust roots of the reference's quadratic): the
// smaller root if >= tmin, else the larger.
__device__ __forceinline__ bool sphere_t(float4 A, float r2, const Ray &r, float tmin, float &t) {
    const float ocx = r.ox - A.x, ocy = r.oy - A.y, ocz = r.oz - A.z;
    const float a = fdot(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz);
    const float hb = fdot(ocx, ocy, ocz, r.dx, r.dy, r.dz);
    const float k = hb / a;
    const float lx = fmaf(-k, r.dx, ocx), ly = fmaf(-k, r.dy, ocy), lz = fmaf(-k, r.dz, ocz);
    const float disc = a * (r2 - fdot(lx, ly, lz, lx, ly, lz));
    if (disc < 0.0f) return false;
    const float sq = sqrtf(disc);
    const float q = hb >= 0.0f ? -(hb + sq) : sq - hb;
    const float cc = fdot(ocx, ocy, ocz, ocx, ocy, ocz) - r2;
    const float t0 = q / a, t1 = cc / q;
    float root = fminf(t0, t1);
    if (!(root >= tmin)) {
        root = fmaxf(t0, t1);
        if (!(root >= tmin)) return false;
    }
    t = root;
    return true;
}

struct Trav {
    int cur;    // next node (>= 0), leaf code (< 0), or kDone
    int sp;     // stack depth * kMeshBlock
    int leaf;   // postponed leaf code or 0
    float bestT;
    int bestI, bestO;
    int ovf;    // 4-wide BVH: entries moved to the lane's spill area (bottom of its stack)
};

// Traversal still has work: nodes to visit or a postponed leaf to test.
__device__ __forceinline__ bool busy(const Trav &T) { return T.cur != kDone || T.leaf != 0; }

__device__ __forceinline__ void begin(Trav &T) {
    T.cur = 0;
    T.sp = 0;
    T.ovf = 0;
    T.leaf = 0;
    T.bestT = INFINITY;
    T.bestI = -1;
    T.bestO = 0x7fffffff;
}

// A hit candidate (t >= tmin when `ok`) of primitive i (leaf order, original id `orig`) replaces the
// closest hit when (t, orig) < (bestT, bestO).  Bitwise and selects: no branch per candidate (the
// short-circuit form cost three exec-mask branches per triangle test).
__device__ __forceinline__ void take_hit(Trav &T, float tt, bool ok, int i, int orig) {
    const float tmin = 0.001f;
    const bool win = ok & (tt >= tmin) & ((tt < T.bestT) | ((tt == T.bestT) & (orig < T.bestO)));
    T.bestT = win ? tt : T.bestT;
    T.bestI = win ? i : T.bestI;
    T.bestO = win ? orig : T.bestO;
}

// Primitive i (leaf order) against the ray: closest hit = min (t, primitive id).
template <bool STATS, bool FULL>
__device__ __forceinline__ void test_prim_data(Trav &T, const Ray &r, float4 A, float4 B, float4 Cc, int i,
                                               unsigned long long &ntest, unsigned *pc) {
    const float tmin = 0.001f;
    prof<STATS>(pc, 5);
    if (STATS) ++ntest;
    if (FULL && __float_as_int(Cc.z) != 0) {
        float tt = 0.0f;
        const bool hit = sphere_t(A, B.x, r, tmin, tt);
        take_hit(T, tt, hit, i, __float_as_int(Cc.y));
        return;
    }
    // Möller–Trumbore, division-free edge tests (pt_oracle.c po_tri_hit)
    const float e1x = A.w, e1y = B.x, e1z = B.y;
    const float e2x = B.z, e2y = B.w, e2z = Cc.x;
    const float pvx = fmaf(r.dy, e2z, -(r.dz * e2y));
    const float pvy = fmaf(r.dz, e2x, -(r.dx * e2z));
    const float pvz = fmaf(r.dx, e2y, -(r.dy * e2x));
    const float det = fdot(e1x, e1y, e1z, pvx, pvy, pvz);
    const float tvx = r.ox - A.x, tvy = r.oy - A.y, tvz = r.oz - A.z;
    const float un = fdot(tvx, tvy, tvz, pvx, pvy, pvz);
    const float qvx = fmaf(tvy, e1z, -(tvz * e1y));
    const float qvy = fmaf(tvz, e1x, -(tvx * e1z));
    const float qvz = fmaf(tvx, e1y, -(tvy * e1x));
    const float vn = fdot(r.dx, r.dy, r.dz, qvx, qvy, qvz);
    const bool neg = det < 0.0f;
    const float us = neg ? -un : un, vs = neg ? -vn : vn;
    const bool inside = (det != 0.0f) & (us >= 0.0f) & (vs >= 0.0f) & (us + vs <= fabsf(det));
    // (the division for every lane, without this branch: blob70k -1%, DESIGN_LOG.md §A.0)
    if (inside) take_hit(T, fdot(e2x, e2y, e2z, qvx, qvy, qvz) / det, true, i, __float_as_int(Cc.y));
}

template <bool STATS, bool FULL>
__device__ __forceinline__ void test_prim(Trav &T, const Ray &r, const float4 *tris, int i, unsigned long long &ntest,
                                          unsigned *pc) {
    const float4 *tp = tris + 3 * i;
    test_prim_data<STATS, FULL>(T, r, tp[0], tp[1], tp[2], i, ntest, pc);
}

// One leaf-loop iteration for this lane: the primitives of leaf T.leaf, then the next leaf if it
// is next in line on the stack.  (Measured and rejected: one primitive per lane per iteration,
// so that lanes with short leaves move on: Cornell -9%, blob70k -5%.)
template <bool STATS, bool FULL, typename Pop, bool PAIRS = false>
__device__ __forceinline__ void leaf_step(Trav &T, const Ray &r, const float4 *tris, unsigned long long &ntest,
                                          unsigned *pc, Pop pop) {
    const int code = ~T.leaf;
    const int first = code >> 4, last = first + (code & 15);
    if (PAIRS) {
        // two primitives' loads in flight per iteration (trees in global memory: blob70k +3%;
        // no gain from LDS)
        for (int i = first; i < last; i += 2) {
            const float4 *tp = tris + 3 * i;
            const float4 A0 = tp[0], B0 = tp[1], C0 = tp[2];
            const bool two = i + 1 < last;
            float4 A1 = A0, B1 = B0, C1 = C0;
            if (two) {
                A1 = tp[3];
                B1 = tp[4];
                C1 = tp[5];
            }
            test_prim_data<STATS, FULL>(T, r, A0, B0, C0, i, ntest, pc);
            if (two) test_prim_data<STATS, FULL>(T, r, A1, B1, C1, i + 1, ntest, pc);
        }
    } else {
        for (int i = first; i < last; ++i) test_prim<STATS, FULL>(T, r, tris, i, ntest, pc);
    }
    // a leaf that was next in line is processed in the same loop
    T.leaf = 0;
    if (T.cur < 0 && T.cur != kDone) {
        T.leaf = T.cur;
        T.cur = pop();
    }
}

// One speculative while-while round (Aila & Laine 2009) over the BVH: interior loop until
// every lane still in it holds a postponed leaf, then the leaf loop.  `my` = this lane's
// LDS stack column (entry k at my[k*kMeshBlock]).  Closest hit = min (t, primitive id).
// Interior nodes: the far child is written to the slot above the top unconditionally (one
// spare slot per lane) and kept only when both children are hit; the top is read
// unconditionally and used only when neither is (branch-free child selection).
template <int NODE_F4, bool STATS, bool FULL>
__device__ __forceinline__ void traverse_round(Trav &T, const Ray &r, int *my, const float4 *nodes,
                                               const float4 *tris, unsigned long long &nvis,
                                               unsigned long long &ntest, unsigned *pc, unsigned leafExit = 0,
                                               unsigned nodeExit = 0) {
    const float tmin = 0.001f;
    while (T.cur >= 0) {
        prof<STATS>(pc, 3);
        const float4 *nd = nodes + __umul24(unsigned(T.cur), unsigned(NODE_F4));  // full-rate 24-bit mul
        const float4 a = nd[0], b = nd[1], c = nd[2];
        const int4 e = *reinterpret_cast<const int4 *>(nd + 3);
        if (STATS) ++nvis;
        const float l0x = fmaf(a.x, r.ix, -r.oix), h0x = fmaf(a.w, r.ix, -r.oix);
        const float l0y = fmaf(a.y, r.iy, -r.oiy), h0y = fmaf(b.x, r.iy, -r.oiy);
        const float l0z = fmaf(a.z, r.iz, -r.oiz), h0z = fmaf(b.y, r.iz, -r.oiz);
        const float l1x = fmaf(b.z, r.ix, -r.oix), h1x = fmaf(c.y, r.ix, -r.oix);
        const float l1y = fmaf(b.w, r.iy, -r.oiy), h1y = fmaf(c.z, r.iy, -r.oiy);
        const float l1z = fmaf(c.x, r.iz, -r.oiz), h1z = fmaf(c.w, r.iz, -r.oiz);
        const float n0 = fmaxf(fmaxf(fminf(l0x, h0x), fminf(l0y, h0y)), fmaxf(fminf(l0z, h0z), tmin));
        const float f0 = fminf(fminf(fmaxf(l0x, h0x), fmaxf(l0y, h0y)), fminf(fmaxf(l0z, h0z), T.bestT));
        const float n1 = fmaxf(fmaxf(fminf(l1x, h1x), fminf(l1y, h1y)), fmaxf(fminf(l1z, h1z), tmin));
        const float f1 = fminf(fminf(fmaxf(l1x, h1x), fmaxf(l1y, h1y)), fminf(fmaxf(l1z, h1z), T.bestT));
        const bool hit0 = n0 <= f0, hit1 = n1 <= f1;
        const bool take0 = hit0 & (!hit1 | (n0 <= n1));  // bitwise: no exec-mask branches
        const int nearC = take0 ? e.x : e.y;
        const int farC = take0 ? e.y : e.x;
        my[T.sp] = farC;
        const int top = my[max(T.sp - kMeshBlock, 0)];
        // (logical, not bitwise, operators here: measured 4.5% faster on gfx950)
        const bool none = !(hit0 || hit1);
        T.sp += (hit0 && hit1) ? kMeshBlock : 0;
        T.cur = none ? (T.sp > 0 ? top : kDone) : nearC;
        T.sp -= (none && T.sp > 0) ? kMeshBlock : 0;
        // postpone the first leaf reached and keep descending
        if (T.cur < 0 && T.cur != kDone && T.leaf == 0) {
            T.leaf = T.cur;
            T.cur = T.sp > 0 ? my[T.sp -= kMeshBlock] : kDone;
        }
        // leave for the leaf loop once at most leafExit lanes still search for their first leaf
        if (__popcll(__ballot((T.leaf | T.cur) >= 0)) <= leafExit) break;
    }
    while (T.leaf != 0) {
        prof<STATS>(pc, 4);
        leaf_step<STATS, FULL>(T, r, tris, ntest, pc, [&] { return T.sp > 0 ? my[T.sp -= kMeshBlock] : kDone; });
        // back to the node loop once at most nodeExit lanes still hold a leaf (they keep it)
        if (nodeExit && __popcll(__ballot(T.leaf != 0)) <= nodeExit) break;
    }
}

// ---- 4-wide BVH (bvh_builder.h Bvh4) ------------------------------------------------------
// Stack: entries in LDS (`cap` of them; 3 spare slots above for the unconditional writes), the
// bottom of a deeper stack in the lane's global spill area (spill[base ...], rare: the builder's
// exact bound exceeds `cap` only for deep trees, and real rays stay far below the bound).
struct SpillArea {
    int *buf;
    unsigned base;  // this lane's first entry
    int cap;        // LDS entries in use at most (the stack content capacity)
};

// Moves the bottom entries of the LDS stack to the spill area so that `push` more entries fit
// under the capacity: half the capacity, or more when a small capacity (cap < 6, half < 3)
// would otherwise let a 4-hit visit (3 pushes) grow the stack past it.
__device__ __forceinline__ void spill_bottom(Trav &T, int *my, const SpillArea &S, int push) {
    const int n = T.sp / kMeshBlock;
    const int k = max(S.cap >> 1, n + push - S.cap);
    for (int j = 0; j < k; ++j) S.buf[S.base + unsigned(T.ovf + j)] = my[j * kMeshBlock];
    for (int j = k; j < n; ++j) my[(j - k) * kMeshBlock] = my[j * kMeshBlock];
    T.sp -= k * kMeshBlock;
    T.ovf += k;
}

__device__ __forceinline__ void refill_bottom(Trav &T, int *my, const SpillArea &S) {
    const int n = min(S.cap >> 1, T.ovf);
    T.ovf -= n;
    for (int j = 0; j < n; ++j) my[j * kMeshBlock] = S.buf[S.base + unsigned(T.ovf + j)];
    T.sp = n * kMeshBlock;
}

// The child code in a packed key's low refBits bits (child_key_p), sign-extended.
__device__ __forceinline__ int key_code(unsigned key, unsigned refBits) {
    return __builtin_amdgcn_sbfe(int(key), 0u, refBits);  // v_bfe_i32: sign-extended low bits
}

template <bool SPILL = true, bool PACKED = false>
__device__ __forceinline__ int pop_wide(Trav &T, int *my, const SpillArea &S, unsigned refBits = 0) {
    if (SPILL && T.sp == 0 && T.ovf != 0) refill_bottom(T, my, S);
    if (T.sp == 0) return kDone;
    T.sp -= kMeshBlock;
    return PACKED ? key_code(unsigned(my[T.sp]), refBits) : my[T.sp];
}

// min(a, b) as one v_min_f32: fminf() of the loop-carried bestT makes the compiler quieten a
// possible signaling NaN first (a v_max_f32 b, b per node visit); the box test has no NaN
// (finite padded boxes, clamped reciprocals), and v_min_f32 of non-NaN inputs is fminf.
__device__ __forceinline__ float fmin_raw(float a, float b) {
    float d;
    asm("v_min_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}

// Sort key of a child box from its near and far planes on each axis (the ray's direction signs
// choose them, see traverse_round_wide): entry distance bits (>= tmin > 0, so ordered as
// unsigned); a miss sorts last.  Two min/max per bound instead of five: the planes need no
// min/max ordering.
__device__ __forceinline__ unsigned child_key(float nx, float fx, float ny, float fy, float nz, float fz,
                                              const Ray &r, float tmin, float bestT) {
    const float ax = fmaf(nx, r.ix, -r.oix), bx = fmaf(fx, r.ix, -r.oix);
    const float ay = fmaf(ny, r.iy, -r.oiy), by = fmaf(fy, r.iy, -r.oiy);
    const float az = fmaf(nz, r.iz, -r.oiz), bz = fmaf(fz, r.iz, -r.oiz);
    const float n = fmaxf(fmaxf(ax, ay), fmaxf(az, tmin));
    const float f = fminf(fminf(bx, by), fmin_raw(bz, bestT));
    return n <= f ? __float_as_uint(n) : 0xffffffffu;
}

// child_key over a quantized node: byte I of each plane word (v_cvt_f32_ubyteI), scaled
// and offset per axis (t = q*B + A).
template <int I>
__device__ __forceinline__ unsigned child_key_q(unsigned nxw, unsigned fxw, unsigned nyw, unsigned fyw, unsigned nzw,
                                                unsigned fzw, float ax, float bx, float ay, float by, float az,
                                                float bz, float tmin, float bestT) {
    const float tnx = fmaf(float((nxw >> (8 * I)) & 0xffu), bx, ax), tfx = fmaf(float((fxw >> (8 * I)) & 0xffu), bx, ax);
    const float tny = fmaf(float((nyw >> (8 * I)) & 0xffu), by, ay), tfy = fmaf(float((fyw >> (8 * I)) & 0xffu), by, ay);
    const float tnz = fmaf(float((nzw >> (8 * I)) & 0xffu), bz, az), tfz = fmaf(float((fzw >> (8 * I)) & 0xffu), bz, az);
    const float n = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, tmin));
    const float f = fminf(fminf(tfx, tfy), fmin_raw(tfz, bestT));
    return n <= f ? __float_as_uint(n) : 0xffffffffu;
}

// Byte offset of the near-plane row within a (lo, hi) row pair: 16 when the axis's reciprocal
// direction is negative (its hi plane is entered first), else 0.
__device__ __forceinline__ unsigned near_row(float inv) { return (__float_as_uint(inv) >> 27) & 16u; }

__device__ __forceinline__ float4 ld4(const float4 *base, unsigned byteOffset) {
    return *reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(base) + byteOffset);
}

// A 16-byte read at LDS byte address `a` (the kernels' dynamic LDS starts at address 0 and an
// LDS-resident scene's nodes sit at its start): the address is the node row's offset itself.  The
// compiler does not fold the dynamic LDS symbol's address (0) into the instruction, so a read
// through the array costs an add (v_xad for the far row) per row.
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_ld4(unsigned a) {
    const f32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) f32x4 *>(size_t(a));
    return make_float4(v.x, v.y, v.z, v.w);
}

// The four children's planes of a half_bvh4 (near, far) read: halves 0-3 near, 4-7 far.  The
// conversions fold into the slab test's FMAs (v_fma_mix_f32 with op_sel).
__device__ __forceinline__ float hlo(unsigned w) { return float(__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu))); }
__device__ __forceinline__ float hhi(unsigned w) { return float(__builtin_bit_cast(_Float16, (unsigned short)(w >> 16))); }
__device__ __forceinline__ float4 half_near(uint4 w) { return make_float4(hlo(w.x), hhi(w.x), hlo(w.y), hhi(w.y)); }
__device__ __forceinline__ float4 half_far(uint4 w) { return make_float4(hlo(w.z), hhi(w.z), hlo(w.w), hhi(w.w)); }

// Compare-exchange of (key, child code) pairs: afterwards ka <= kb.
__device__ __forceinline__ void cas(unsigned &ka, int &ca, unsigned &kb, int &cb) {
    const bool sw = kb < ka;
    const unsigned k = ka;
    const int c = ca;
    ka = sw ? kb : ka;
    kb = sw ? k : kb;
    ca = sw ? cb : ca;
    cb = sw ? c : cb;
}

// Packed child keys (PACKED, LDS-resident scenes; child_key_p): the entry distance's bits with the
// child's code in the low `refBits` bits, (bits & ~mask) | (code & mask); a miss is all ones.  The
// LDS copy of the nodes holds the codes already masked (mesh_kernel's scene copy).  An interior code (a
// node byte offset) and a leaf code (~(first<<4 | count)) of a scene that fits the LDS copy are
// small enough in magnitude that their low refBits bits, sign-extended, give them back
// (hippt_api.cpp packed_ref_bits): the sorted keys ARE the sorted codes, so the sorting network
// is 5 unsigned min/max pairs (no compare + 4 selects per exchange moving the codes along), and the
// stack holds keys.  Truncating the distance to its high bits only reorders near-equal children,
// and the closest hit is argmin (t, primitive id): no result bit depends on the visiting order.
template <bool PACKED>
__device__ __forceinline__ unsigned child_key_p(float nx, float fx, float ny, float fy, float nz, float fz,
                                                const Ray &r, float tmin, float bestT, int code, unsigned mask) {
    if (!PACKED) return child_key(nx, fx, ny, fy, nz, fz, r, tmin, bestT);
    const float ax = fmaf(nx, r.ix, -r.oix), bx = fmaf(fx, r.ix, -r.oix);
    const float ay = fmaf(ny, r.iy, -r.oiy), by = fmaf(fy, r.iy, -r.oiy);
    const float az = fmaf(nz, r.iz, -r.oiz), bz = fmaf(fz, r.iz, -r.oiz);
    const float n = fmaxf(fmaxf(ax, ay), fmaxf(az, tmin));
    const float f = fminf(fminf(bx, by), fmin_raw(bz, bestT));
    return n <= f ? (__float_as_uint(n) & ~mask) | unsigned(code) : 0xffffffffu;  // code: pre-masked
}

__device__ __forceinline__ void cas_key(unsigned &ka, unsigned &kb) {
    const unsigned lo = min(ka, kb), hi = max(ka, kb);
    ka = lo;
    kb = hi;
}

// traverse_round over the 4-wide tree: a node visit tests its four child boxes, descends into
// the nearest hit child and pushes the other hit children far to near.  SPILL=false: the tree's
// stack bound fits the LDS capacity (no spill/refill code in the loop).
// TOP (trees in global memory): the first topBytes of the node array (the top of the tree,
// breadth-first) also sit at LDS address 0; a visit to one of them reads LDS, which spares the
// texture addresser (TA) — the unit that bounds the traversal of global-memory trees — the loads
// every ray makes at the top of the tree.
// HYBRID (with QUANT and TOP; bvh_builder.h hybrid_bvh4): the top is 128-byte float nodes (read
// from LDS, no decode) and every node below it a 64-byte 8-bit node in global memory (4 loads
// instead of 7 where the TA binds); a node byte offset below topBytes is a top node.  Measured and
// kept off (DESIGN_LOG.md §A.1): the wave's lanes straddle the top/bottom boundary on most iterations,
// which then run both paths (blob70k 17.5 vs 20.9 G); visiting the top first, the lanes below it
// waiting, was worse still (11.7 G).
// PACKED (LDS-resident scenes): packed child keys (pack_key), refBits low bits carrying the code.
// HALF (with TOP, trees in global memory; bvh_builder.h half_bvh4): the same 128-byte nodes with
// half-precision planes, each axis's near and far planes one aligned 16-byte read (4 reads per
// visit instead of 7 where the TA binds), the slab FMAs taking the halves directly (v_fma_mix_f32).
template <int NODE_F4, bool STATS, bool FULL, bool QUANT = false, bool SPILL = true, bool LDS0 = false,
          bool TOP = false, bool HYBRID = false, bool PACKED = false, bool HALF = false>
__device__ __forceinline__ void traverse_round_wide(Trav &T, const Ray &r, int *my, const float4 *nodes,
                                                    const float4 *tris, unsigned long long &nvis,
                                                    unsigned long long &ntest, unsigned *pc, unsigned leafExit,
                                                    unsigned nodeExit, const SpillArea &S,
                                                    unsigned topBytes = 0, unsigned refBits = 0) {
    static_assert(!HYBRID || (QUANT && TOP), "hybrid trees: 8-bit nodes below an LDS top");
    static_assert(!PACKED || (LDS0 && !QUANT), "packed keys: LDS-resident float trees");
    static_assert(!HALF || (TOP && !QUANT && !LDS0), "half planes: 4-wide trees in global memory");
    const unsigned refMask = PACKED ? (1u << refBits) - 1u : 0u;
    const float tmin = 0.001f;
    // near-row byte offsets of this ray's octant within a node (x at 0/16, y at 32/48, z at 64/80)
    const unsigned sx = near_row(r.ix), sy = near_row(r.iy) | 32u, sz = near_row(r.iz) | 64u;
    while (T.cur >= 0) {
        prof<STATS>(pc, 3);
        // rows lo.x hi.x lo.y hi.y lo.z hi.z: read as near/far rows of this ray's octant (32-bit
        // byte offsets from the uniform base: base-register + offset-register loads).  NODE_F4
        // (the node stride) is implied by the codes: the device trees store byte offsets.
        const unsigned nb = unsigned(T.cur);  // interior codes are node byte offsets
        const bool topVisit = TOP && nb < topBytes;
        unsigned k0, k1, k2, k3;
        int4 ch;
        if (!QUANT || (HYBRID && topVisit)) {
            // 128-byte float nodes (LDS and global): nb's low 7 bits are zero, so the octant's
            // near row is nb | s and the far row its ^ 16
            const unsigned ax = nb | sx, ay = nb | sy, az = nb | sz;
            // LDS0: the nodes are the LDS scene copy at LDS address 0
            float4 nx, fx, ny, fy, nz, fz, cw;
            if (HALF) {
                // the octant's (near, far) row of each axis: the float node's near-row address
                float4 vx, vy, vz;
                if (topVisit) {
                    vx = lds_ld4(ax);
                    vy = lds_ld4(ay);
                    vz = lds_ld4(az);
                    cw = lds_ld4(nb + 96u);
                } else {
                    vx = ld4(nodes, ax);
                    vy = ld4(nodes, ay);
                    vz = ld4(nodes, az);
                    cw = ld4(nodes, nb + 96u);
                }
                const uint4 wx = *reinterpret_cast<const uint4 *>(&vx), wy = *reinterpret_cast<const uint4 *>(&vy),
                            wz = *reinterpret_cast<const uint4 *>(&vz);
                nx = half_near(wx);
                fx = half_far(wx);
                ny = half_near(wy);
                fy = half_far(wy);
                nz = half_near(wz);
                fz = half_far(wz);
            } else if (LDS0 || HYBRID || topVisit) {
                nx = lds_ld4(ax);
                fx = lds_ld4(ax ^ 16u);
                ny = lds_ld4(ay);
                fy = lds_ld4(ay ^ 16u);
                nz = lds_ld4(az);
                fz = lds_ld4(az ^ 16u);
                cw = lds_ld4(nb + 96u);
            } else {
                nx = ld4(nodes, ax);
                fx = ld4(nodes, ax ^ 16u);
                ny = ld4(nodes, ay);
                fy = ld4(nodes, ay ^ 16u);
                nz = ld4(nodes, az);
                fz = ld4(nodes, az ^ 16u);
                cw = ld4(nodes, nb + 96u);
            }
            ch = *reinterpret_cast<const int4 *>(&cw);
            k0 = child_key_p<PACKED>(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x, r, tmin, T.bestT, ch.x, refMask);
            k1 = child_key_p<PACKED>(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y, r, tmin, T.bestT, ch.y, refMask);
            k2 = child_key_p<PACKED>(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z, r, tmin, T.bestT, ch.z, refMask);
            k3 = child_key_p<PACKED>(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w, r, tmin, T.bestT, ch.w, refMask);
            if (STATS && (k0 & k1 & k2 & k3) == 0xffffffffu) {
                const unsigned u = child_key(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x, r, tmin, INFINITY) &
                                   child_key(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y, r, tmin, INFINITY) &
                                   child_key(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z, r, tmin, INFINITY) &
                                   child_key(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w, r, tmin, INFINITY);
                if (u != 0xffffffffu) ++pc[kNhHist + 5];
            }
        } else {
            // 64-byte node (bvh_builder.h quantize_bvh4): 4 loads instead of 7.  Plane q of axis
            // a enters the slab test as t = q*(s*inv) + (o*inv - o_ray*inv).
            float4 o, qf, q2, cw;
            if (!HYBRID && topVisit) {
                o = lds_ld4(nb);
                qf = lds_ld4(nb + 16u);
                q2 = lds_ld4(nb + 32u);
                cw = lds_ld4(nb + 48u);
            } else {
                o = ld4(nodes, nb);
                qf = ld4(nodes, nb + 16u);
                q2 = ld4(nodes, nb + 32u);
                cw = ld4(nodes, nb + 48u);
            }
            const uint4 q = *reinterpret_cast<const uint4 *>(&qf);
            ch = *reinterpret_cast<const int4 *>(&cw);
            const float bx = o.w * r.ix, ax = fmaf(o.x, r.ix, -r.oix);
            const float by = q2.z * r.iy, ay = fmaf(o.y, r.iy, -r.oiy);
            const float bz = q2.w * r.iz, az = fmaf(o.z, r.iz, -r.oiz);
            const unsigned qlz = __float_as_uint(q2.x), qhz = __float_as_uint(q2.y);
            const bool mx = sx & 16u, my_ = sy & 16u, mz = sz & 16u;
            const unsigned nxw = mx ? q.y : q.x, fxw = mx ? q.x : q.y;
            const unsigned nyw = my_ ? q.w : q.z, fyw = my_ ? q.z : q.w;
            const unsigned nzw = mz ? qhz : qlz, fzw = mz ? qlz : qhz;
            k0 = child_key_q<0>(nxw, fxw, nyw, fyw, nzw, fzw, ax, bx, ay, by, az, bz, tmin, T.bestT);
            k1 = child_key_q<1>(nxw, fxw, nyw, fyw, nzw, fzw, ax, bx, ay, by, az, bz, tmin, T.bestT);
            k2 = child_key_q<2>(nxw, fxw, nyw, fyw, nzw, fzw, ax, bx, ay, by, az, bz, tmin, T.bestT);
            k3 = child_key_q<3>(nxw, fxw, nyw, fyw, nzw, fzw, ax, bx, ay, by, az, bz, tmin, T.bestT);
        }
        if (STATS) ++nvis;
        if (STATS && TOP && nb < topBytes) ++pc[kTopVisits];
        // hit children: a miss key is all ones (bit 31), a hit key a positive float's bits
        const int nh = 4 - int((k0 >> 31) + (k1 >> 31) + (k2 >> 31) + (k3 >> 31));
        if (STATS) ++pc[kNhHist + nh];
        // sorting network (0,1)(2,3)(0,2)(1,3)(1,2), codes carried along (or inside the keys):
        // c0 nearest
        int c0, c1, c2, c3;
        if (PACKED) {
            cas_key(k0, k1);
            cas_key(k2, k3);
            cas_key(k0, k2);
            cas_key(k1, k3);
            cas_key(k1, k2);
            c0 = key_code(k0, refBits);  // the stack holds the keys themselves
            c1 = int(k1);
            c2 = int(k2);
            c3 = int(k3);
        } else {
            c0 = ch.x;
            c1 = ch.y;
            c2 = ch.z;
            c3 = ch.w;
            cas(k0, c0, k1, c1);
            cas(k2, c2, k3, c3);
            cas(k0, c0, k2, c2);
            cas(k1, c1, k3, c3);
            cas(k1, c1, k2, c2);
        }
        if (SPILL && T.sp + (nh - 1) * kMeshBlock > S.cap * kMeshBlock) spill_bottom(T, my, S, nh - 1);
        // push c[nh-1] .. c1 (c1 on top); unused writes land in the spare slots above
        my[T.sp] = nh == 4 ? c3 : (nh == 3 ? c2 : c1);
        my[T.sp + kMeshBlock] = nh == 4 ? c2 : c1;
        my[T.sp + 2 * kMeshBlock] = c1;
        T.sp += nh > 1 ? (nh - 1) * kMeshBlock : 0;
        T.cur = nh > 0 ? c0 : pop_wide<SPILL, PACKED>(T, my, S, refBits);
        // postpone the first leaf reached and keep descending
        if (T.cur < 0 && T.cur != kDone && T.leaf == 0) {
            T.leaf = T.cur;
            T.cur = pop_wide<SPILL, PACKED>(T, my, S, refBits);
        }
        if (__popcll(__ballot((T.leaf | T.cur) >= 0)) <= leafExit) break;
    }
    auto popw = [&] { return pop_wide<SPILL, PACKED>(T, my, S, refBits); };
    while (T.leaf != 0) {
        prof<STATS>(pc, 4);
        leaf_step<STATS, FULL, decltype(popw), !LDS0>(T, r, tris, ntest, pc, popw);
        if (nodeExit && __popcll(__ballot(T.leaf != 0)) <= nodeExit) break;
    }
}

}  // namespace trace
}  // namespace hippt
