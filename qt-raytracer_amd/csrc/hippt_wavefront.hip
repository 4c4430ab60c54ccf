// hippt_wavefront.hip — wavefront variant of the triangle path tracer (BASELINE config 5 A/B;
// Laine, Karras & Aila 2013), bit-identical to mesh_kernel.
//
// Path state lives in HBM as a pool of S slots (structure of arrays).  Per iteration:
//   wf_extend    persistent grid; lanes pull ray-queue entries (wave-pooled counter), traverse
//                the BVH (the megakernel's speculative while-while round, threshold refill)
//                and write (t, triangle) per slot;
//   wf_shade     one lane per queued slot: sky on a miss, depth cut-off, or material scatter;
//                scattered slots go to the next ray queue, finished samples write their radiance
//                to the sample scratch and go to the regenerate queue;
//   wf_generate  one lane per regenerate-queue entry: work item = base + queue position (no
//                atomics), camera ray, append to the next ray queue.
// Queue appends are aggregated per 1024-thread block (one atomic per block) into 8 sharded
// segments; counters also give the exact segment and sample counts without per-wave atomics.
#include "hippt_trace.h"
#include "hippt_wavefront.h"

namespace hippt {
namespace {
using namespace trace;

// A path's state as it sits in a ray queue (WfParams::ra/rb/rc, three float4 arrays per queue).
struct Path {
    Ray r;
    float tr, tg, tb;
    uint32_t rng, item;
    int depth;
};

__device__ __forceinline__ void load_ray(const WfParams &W, int q, unsigned i, Ray &r) {
    const float4 a = W.ra[q][i], b = W.rb[q][i];
    r.ox = a.x;
    r.oy = a.y;
    r.oz = a.z;
    r.dx = a.w;
    r.dy = b.x;
    r.dz = b.y;
}

__device__ __forceinline__ void store_path(const WfParams &W, int q, unsigned i, const Path &p) {
    W.ra[q][i] = make_float4(p.r.ox, p.r.oy, p.r.oz, p.r.dx);
    W.rb[q][i] = make_float4(p.r.dy, p.r.dz, p.tr, p.tg);
    W.rc[q][i] = make_float4(p.tb, __uint_as_float(p.rng), __int_as_float(p.depth), __uint_as_float(p.item));
}

// Entries of queue q's shard k: appended by wf_shade plus added by wf_generate.
__device__ __forceinline__ unsigned shard_size(const unsigned *ctr, int q, int k) {
    return ctr[ctr_word(ctr_queue(q) + k)] + ctr[ctr_word(ctr_gen(q) + k)];
}

// Block-aggregated append (one atomic per block) to shard blockIdx % kWfShards of queue q:
// returns this thread's entry index (kNone for a thread that does not append).  Every thread of
// the block must call it (it synchronises); `lds` holds kWfBlock/64 + 1 words.
__device__ __forceinline__ unsigned block_append(bool req, unsigned cap, unsigned *ctr, int q, unsigned *lds) {
    const unsigned long long m = __ballot(req);
    const unsigned wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
    if (__lane_id() == 0) lds[wave] = unsigned(__popcll(m));
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
        for (unsigned w = 0; w < nw; ++w) {
            const unsigned c = lds[w];
            lds[w] = tot;
            tot += c;
        }
        const unsigned shard = blockIdx.x % kWfShards;
        lds[nw] = tot ? shard * cap + atomicAdd(&ctr[ctr_word(ctr_queue(q) + int(shard))], tot) : 0u;
    }
    __syncthreads();
    const unsigned at = req ? lds[nw] + lds[wave] + rank : kNone;
    __syncthreads();
    return at;
}

// block_append with the block's appends ordered by key (< 64; WfParams::sortBits): an LDS counting
// sort, one atomic per block as before.  A path's entry within its key's bin follows the LDS atomics'
// order: the queue's order changes which lane traces a path, never what it computes.
__device__ __forceinline__ unsigned block_append_sorted(bool req, unsigned key, unsigned bins, unsigned cap,
                                                        unsigned *ctr, int q, unsigned *lds) {
    if (threadIdx.x < 64) lds[threadIdx.x] = 0;
    __syncthreads();
    const unsigned rank = req ? atomicAdd(&lds[key], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {
        // exclusive scan of the bin counts (wave 0)
        const unsigned v = threadIdx.x < bins ? lds[threadIdx.x] : 0u;
        unsigned inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned t = __shfl_up(inc, o);
            if (int(threadIdx.x) >= o) inc += t;
        }
        lds[threadIdx.x] = inc - v;
        if (threadIdx.x == 63) {
            const unsigned shard = blockIdx.x % kWfShards;
            lds[64] = inc ? shard * cap + atomicAdd(&ctr[ctr_word(ctr_queue(q) + int(shard))], inc) : 0u;
        }
    }
    __syncthreads();
    const unsigned at = req ? lds[64] + lds[key] + rank : kNone;
    __syncthreads();
    return at;
}

// Counters of both queues and the work base start at 0.
static_assert(kCtrCount <= 64, "wf_init clears the counters with one wave");
__global__ void wf_init(WfParams W) {
    const unsigned i = threadIdx.x;
    if (i < unsigned(kCtrCount)) W.ctr[ctr_word(int(i))] = 0;
}

// WIDE: the megakernel's 4-wide traversal (QUANT: over 8-bit child boxes, HALF: over half-precision
// planes; global memory only).
template <bool STATS, bool LDS_SCENE, bool FULL, bool WIDE, bool QUANT, bool HALF = false>
__global__ __launch_bounds__(kMeshBlock) void wf_extend(WfParams W, int cur) {
    extern __shared__ int lds[];  // LDS scene: nodes at address 0, then stack, primitives
    constexpr int ldsNodeF4 = WIDE ? kLdsNode4F4 : kLdsNodeF4;  // mesh_lds_bytes layout
    const MeshParams &P = W.mp;
    // trees in global memory: the top of the tree (P.topBytes) at LDS address 0, then the stack
    constexpr bool TOP = WIDE && !LDS_SCENE;
    int *const stk = LDS_SCENE ? lds + P.numNodes * ldsNodeF4 * 4 : lds + (TOP ? (P.topBytes >> 2) : 0u);
    int *const my = stk + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // this iteration's rays = its segments; the paths wf_generate started into this queue
        // = samples (every path of a batch ends within it) and advance the work base; this
        // iteration's shade and generate fill the other queue (emptied here)
        unsigned rays = 0, gen = 0;
#pragma unroll
        for (int k = 0; k < kWfShards; ++k) {
            rays += shard_size(W.ctr, cur, k);
            gen += W.ctr[ctr_word(ctr_gen(cur) + k)];
            W.ctr[ctr_word(ctr_queue(cur ^ 1) + k)] = 0;
            W.ctr[ctr_word(ctr_gen(cur ^ 1) + k)] = 0;
        }
        atomicAdd(&P.stats[0], (unsigned long long)rays);
        if (gen) atomicAdd(&P.stats[1], (unsigned long long)gen);
        W.ctr[ctr_word(kCtrWork)] += gen;
    }
    const float4 *nodes = P.nodes, *tris = P.tris;
    if (LDS_SCENE) {
        float4 *sNodes = reinterpret_cast<float4 *>(lds);
        float4 *sTris = reinterpret_cast<float4 *>(stk + (P.stackDepth + 1) * kMeshBlock);
        if (WIDE) {
            for (int i = threadIdx.x; i < P.numNodes * kLdsNode4F4; i += kMeshBlock) sNodes[i] = P.nodes[i];
        } else {
            for (int i = threadIdx.x; i < P.numNodes * 4; i += kMeshBlock)
                sNodes[(i >> 2) * kLdsNodeF4 + (i & 3)] = P.nodes[i];
        }
        for (int i = threadIdx.x; i < P.numTris * 3; i += kMeshBlock) sTris[i] = P.tris[i];
        __syncthreads();
        nodes = sNodes;
        tris = sTris;
    }
    if (TOP && P.topBytes) {
        float4 *sTop = reinterpret_cast<float4 *>(lds);
        for (unsigned i = threadIdx.x; i < (P.topBytes >> 4); i += kMeshBlock) sTop[i] = P.nodes[i];
        __syncthreads();
    }
    constexpr int nodeF4 = WIDE ? (QUANT ? 4 : (LDS_SCENE ? kLdsNode4F4 : 8)) : (LDS_SCENE ? kLdsNodeF4 : 4);
    const SpillArea S{P.spill, (blockIdx.x * unsigned(kMeshBlock) + threadIdx.x) * unsigned(P.spillCap), P.stackCap};
    // each wave drains its block's home shard first, then the others in turn (one fetch
    // counter per shard spreads the atomics over kWfShards lines); consecutive lanes take
    // consecutive entries, so the ray and hit arrays are read and written in whole lines
    unsigned fs = blockIdx.x % kWfShards, left = kWfShards;
    unsigned fsCount = shard_size(W.ctr, cur, int(fs));
    unsigned poolNext = 0, poolEnd = 0;
    unsigned slot = kNone;  // this lane's queue entry
    bool need = true;
    Ray r{};
    Trav T;
    T.cur = kDone;
    T.sp = 0;
    T.leaf = 0;
    T.bestT = INFINITY;
    T.bestI = -1;
    T.bestO = 0x7fffffff;
    unsigned long long nvis = 0, ntest = 0;
    unsigned pc[kProfSlots] = {};  // phase profile slots (not reported by the wavefront path)
    for (;;) {
        while (left && __ballot(need)) {
            const unsigned qi =
                wave_fetch(need, poolNext, poolEnd, &W.ctr[ctr_word(kCtrFetch + int(fs))], unsigned(P.chunk), fsCount);
            if (need && qi != kNone) {
                need = false;
                slot = fs * W.shardCap + qi;
                load_ray(W, cur, slot, r);
                prepare(r);
                begin(T);
            }
            if (__ballot(need)) {  // this shard is drained
                fs = fs + 1 == kWfShards ? 0u : fs + 1;
                fsCount = shard_size(W.ctr, cur, int(fs));
                poolNext = poolEnd = 0;
                --left;
            }
        }
        need = false;
        if (!__any(busy(T))) break;
        do {
            if (WIDE)
                traverse_round_wide<nodeF4, STATS, FULL, QUANT, true, LDS_SCENE, TOP, false, false, HALF>(
                    T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit, S, P.topBytes);
            else
                traverse_round<nodeF4, STATS, FULL>(T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit);
        } while (__popcll(__ballot(busy(T))) > unsigned(P.waveThreshold));
        if (slot != kNone && !busy(T)) {
            W.hit[slot] = make_float2(T.bestT, __int_as_float(T.bestI));
            slot = kNone;
            need = true;
        }
    }
    if (STATS) {
        const unsigned long long a = wave_sum(nvis), b = wave_sum(ntest);
        if (__lane_id() == 0) {
            atomicAdd(&stat_slot(P.stats)[2], a);
            atomicAdd(&stat_slot(P.stats)[3], b);
        }
    }
}

// Shade and generate keep every shard an independent pipeline: block b works on shard
// b % kWfShards of queue cur and appends to the same shard of the other queue, so a shard never
// holds more than its ceil(slots / kWfShards) entries.
template <bool FULL>
__global__ __launch_bounds__(kWfBlock) void wf_shade(WfParams W, int cur) {
    static_assert(kWfBlock / 64 + 1 <= 65, "one LDS array serves both appends");
    __shared__ unsigned lds[65];
    const MeshParams &P = W.mp;
    if (blockIdx.x == 0 && threadIdx.x < kWfShards) W.ctr[ctr_word(kCtrFetch + int(threadIdx.x))] = 0;
    const unsigned shard = blockIdx.x % kWfShards;
    const unsigned first = (blockIdx.x / kWfShards) * kWfBlock;
    const unsigned count = shard_size(W.ctr, cur, int(shard));
    // the grid covers a full shard; blocks past this iteration's queue leave before the appends
    // (block-uniform: no thread of such a block appends, so none needs the barriers)
    if (first >= count) return;
    const unsigned local = first + threadIdx.x;
    bool again = false, finished = false;
    Path q{};
    if (local < count) {
        const unsigned i = shard * W.shardCap + local;
        const float4 a = W.ra[cur][i], b = W.rb[cur][i], c = W.rc[cur][i];
        const float2 h = W.hit[i];
        q.r.ox = a.x;
        q.r.oy = a.y;
        q.r.oz = a.z;
        q.r.dx = a.w;
        q.r.dy = b.x;
        q.r.dz = b.y;
        q.tr = b.z;
        q.tg = b.w;
        q.tb = c.x;
        q.rng = __float_as_uint(c.y);
        q.depth = __float_as_int(c.z);
        q.item = __float_as_uint(c.w);
        const int tri = __float_as_int(h.y);
        float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
        if (tri < 0) {
            sky(q.r, q.tr, q.tg, q.tb, L0, L1, L2);
            finished = true;
        } else if (++q.depth >= P.maxDepth) {
            finished = true;
        } else if (scatter<FULL, false>(q.r, h.x, tri, P.shade, P.tris, P.mats, q.rng, q.tr, q.tg, q.tb, nullptr,
                                        P.rngTable)) {
            again = true;
        } else {
            finished = true;  // absorbed: contributes 0
        }
        if (finished) store_radiance(P.scratch, q.item, L0, L1, L2);
    }
    unsigned at;
    if (W.sortBits) {
        // direction octant, then the origin's cell of a 2x2x2 grid over the scene box
        unsigned key = (q.r.dx < 0.0f ? 1u : 0u) | (q.r.dy < 0.0f ? 2u : 0u) | (q.r.dz < 0.0f ? 4u : 0u);
        if (W.sortBits > 3) {
            const unsigned cx = (q.r.ox - W.sortLo[0]) * W.sortScale[0] >= 1.0f ? 1u : 0u;
            const unsigned cy = (q.r.oy - W.sortLo[1]) * W.sortScale[1] >= 1.0f ? 1u : 0u;
            const unsigned cz = (q.r.oz - W.sortLo[2]) * W.sortScale[2] >= 1.0f ? 1u : 0u;
            key = key << 3 | cx | cy << 1 | cz << 2;
        }
        at = block_append_sorted(again, again ? key : 0u, 1u << W.sortBits, W.shardCap, W.ctr, cur ^ 1, lds);
    } else {
        at = block_append(again, W.shardCap, W.ctr, cur ^ 1, lds);
    }
    if (again) store_path(W, cur ^ 1, at, q);
}

// New paths into the free capacity of queue nxt (after this iteration's shade), work items in
// order: shard k's share starts after the lower shards' (no atomics); W.ctr[kCtrWork] = items
// generated so far (advanced by the next wf_extend, which reads the shards' counts).
__global__ __launch_bounds__(kWfBlock) void wf_generate(WfParams W, int nxt) {
    const MeshParams &P = W.mp;
    const unsigned base = W.ctr[ctr_word(kCtrWork)];
    const unsigned left = P.totalItems - min(base, P.totalItems);
    unsigned lower = 0, here = 0, used = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k) {
        const unsigned n = W.ctr[ctr_word(ctr_queue(nxt) + k)];
        const unsigned gen = min(W.shardCap - min(n, W.shardCap), left - min(lower, left));
        if (unsigned(k) == blockIdx.x % kWfShards) {
            here = gen;
            used = n;
            break;
        }
        lower += gen;
    }
    const unsigned local = (blockIdx.x / kWfShards) * kWfBlock + threadIdx.x;
    if (local < here) {
        const unsigned shard = blockIdx.x % kWfShards;
        Path q;
        q.item = base + lower + local;
        camera_sample(P, q.item, q.r, q.rng);
        q.tr = q.tg = q.tb = 1.0f;
        q.depth = 0;
        store_path(W, nxt, shard * W.shardCap + used + local, q);
    }
    // the shard's count, computed alike by every block of the shard from values no block of
    // this launch changes
    if (local == 0) W.ctr[ctr_word(ctr_gen(nxt) + int(blockIdx.x % kWfShards))] = here;
}

using ExtFn = void (*)(WfParams, int);
template <bool STATS, bool FULL>
ExtFn ext_fn_fmt(bool lds, bool wide, bool quant, bool half) {
    if (lds) return wide ? wf_extend<STATS, true, FULL, true, false> : wf_extend<STATS, true, FULL, false, false>;
    if (!wide) return wf_extend<STATS, false, FULL, false, false>;
    if (half) return wf_extend<STATS, false, FULL, true, false, true>;
    return quant ? wf_extend<STATS, false, FULL, true, true> : wf_extend<STATS, false, FULL, true, false>;
}
ExtFn ext_fn(bool count, bool lds, bool full, bool wide, bool quant, bool half = false) {
    if (count)
        return full ? ext_fn_fmt<true, true>(lds, wide, quant, half) : ext_fn_fmt<true, false>(lds, wide, quant, half);
    return full ? ext_fn_fmt<false, true>(lds, wide, quant, half) : ext_fn_fmt<false, false>(lds, wide, quant, half);
}

}  // namespace

size_t wf_pool_words(unsigned slots, unsigned *shardCap) {
    // shards are closed pipelines (wf_shade/wf_generate): shard k never holds more than cap
    // entries
    const unsigned cap = (slots + kWfShards - 1) / kWfShards;
    *shardCap = cap;
    return size_t(kWfShards) * cap * kWfWordsPerSlot;
}

// kWfShards blocks per 1024 entries of one shard segment
static unsigned shard_grid(const WfParams &W) { return kWfShards * ((W.shardCap + kWfBlock - 1) / kWfBlock); }

hipError_t wf_launch_init(const WfParams &W, hipStream_t s) {
    hipLaunchKernelGGL(wf_init, dim3(1), dim3(64), 0, s, W);
    return hipGetLastError();
}

hipError_t wf_launch_generate(const WfParams &W, int nxt, hipStream_t s) {
    hipLaunchKernelGGL(wf_generate, dim3(shard_grid(W)), dim3(kWfBlock), 0, s, W, nxt);
    return hipGetLastError();
}

hipError_t wf_launch_extend(const WfParams &W, int cur, int blocks, bool countTraversal, hipStream_t s) {
    const MeshParams &P = W.mp;
    const bool lds = P.ldsScene != 0;
    if (P.topBytes && (lds || !P.wide || P.topBytes % (P.wide == 2 ? 64u : 128u) ||
                       P.topBytes > (unsigned(P.numNodes) << (P.wide == 2 ? 6 : 7))))
        return hipErrorInvalidValue;
    const size_t bytes = mesh_lds_bytes(P.stackDepth, lds ? P.numNodes : 0, lds ? P.numTris : 0, P.wide != 0, P.topBytes);
    const auto fn = ext_fn(countTraversal, lds, P.full != 0, P.wide != 0, P.wide == kWideQuant && !lds,
                           P.wide == kWideHalf && !lds);
    if (P.wide && (lds || P.topBytes)) {  // the variant launched (8-bit nodes included) reads LDS at 0
        const hipError_t e = check_lds_at_zero(reinterpret_cast<const void *>(fn));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(kMeshBlock), bytes, s, W, cur);
    return hipGetLastError();
}

hipError_t wf_launch_shade(const WfParams &W, int cur, hipStream_t s) {
    hipLaunchKernelGGL(W.mp.full ? wf_shade<true> : wf_shade<false>, dim3(shard_grid(W)), dim3(kWfBlock), 0, s, W, cur);
    return hipGetLastError();
}

int wf_extend_blocks_per_cu(bool countTraversal, bool full, bool wide, bool quant, int stackDepth, int ldsNodes,
                            int ldsTris, unsigned topBytes) {
    int n = 0;
    const size_t bytes = mesh_lds_bytes(stackDepth, ldsNodes, ldsTris, wide, topBytes);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &n, ext_fn(countTraversal, ldsNodes > 0, full, wide, quant && wide && ldsNodes == 0), kMeshBlock, bytes) !=
            hipSuccess ||
        n <= 0)
        n = 1;
    return n;
}

}  // namespace hippt
