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

// Slot record fields (see WfParams::st).
struct Slot {
    Ray r;
    float tr, tg, tb;
    uint32_t rng, item;
    int depth;
};

__device__ __forceinline__ void load_ray(const WfParams &W, unsigned s, Ray &r) {
    const float4 a = W.st[4 * size_t(s)], b = W.st[4 * size_t(s) + 1];
    r.ox = a.x;
    r.oy = a.y;
    r.oz = a.z;
    r.dx = a.w;
    r.dy = b.x;
    r.dz = b.y;
}

// whole: also the hit row (zeros), so that the record's 64 bytes are written at once.  wf_generate's
// fresh records: 3.9 -> 2.8 ms for 132.7 M camera rays (r3ac; a partly written line is merged by the
// memory side); wf_shade: no gain (+0.7%), its records' lines were read just before.
__device__ __forceinline__ void store_slot(const WfParams &W, unsigned s, const Slot &q, bool whole = false) {
    float4 *p = W.st + 4 * size_t(s);
    p[0] = make_float4(q.r.ox, q.r.oy, q.r.oz, q.r.dx);
    p[1] = make_float4(q.r.dy, q.r.dz, q.tr, q.tg);
    p[2] = make_float4(q.tb, __uint_as_float(q.rng), __int_as_float(q.depth), __uint_as_float(q.item));
    if (whole) p[3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// Shard sizes of one sharded queue (counters first .. first + kWfShards - 1) and their prefix.
struct Shards {
    unsigned pre[kWfShards + 1];
};

__device__ __forceinline__ Shards load_shards(const unsigned *ctr, int first) {
    Shards s;
    s.pre[0] = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k) s.pre[k + 1] = s.pre[k] + ctr[ctr_word(first + k)];
    return s;
}

// Block-aggregated append (one atomic per block) to shard blockIdx % kWfShards of the queue
// whose counters start at `first`.  Every thread of the block must call it (it synchronises);
// `lds` holds kWfBlock/64 + 1 words.
__device__ __forceinline__ void block_append(bool req, unsigned value, unsigned *q, unsigned cap, unsigned *ctr,
                                             int first, unsigned *lds) {
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
        lds[nw] = tot ? shard * cap + atomicAdd(&ctr[ctr_word(first + int(shard))], tot) : 0u;
    }
    __syncthreads();
    if (req) q[lds[nw] + lds[wave] + rank] = value;
    __syncthreads();
}

// Initial regenerate queue: every slot, spread over the shards.
__global__ void wf_init(WfParams W) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    const unsigned per = W.shardCap;
    if (i < W.slots) W.genQ[(i / per) * W.shardCap + i % per] = i;
    if (i < kWfShards) {
        const unsigned lo = i * per, hi = min(W.slots, (i + 1) * per);
        W.ctr[ctr_word(kCtrGen + i)] = hi > lo ? hi - lo : 0u;
        W.ctr[ctr_word(kCtrExt0 + i)] = 0;
        W.ctr[ctr_word(kCtrExt1 + i)] = 0;
        W.ctr[ctr_word(kCtrFetch + i)] = 0;
    }
    if (i == 0) W.ctr[ctr_word(kCtrWork)] = 0;
}

// WIDE: the megakernel's 4-wide traversal (QUANT: over 8-bit child boxes, global memory only).
template <bool STATS, bool LDS_SCENE, bool FULL, bool WIDE, bool QUANT>
__global__ __launch_bounds__(kMeshBlock) void wf_extend(WfParams W, int cur) {
    extern __shared__ int lds[];  // LDS scene: nodes at address 0, then stack, primitives
    constexpr int ldsNodeF4 = WIDE ? kLdsNode4F4 : kLdsNodeF4;  // mesh_lds_bytes layout
    const MeshParams &P = W.mp;
    // trees in global memory: the top of the tree (P.topBytes) at LDS address 0, then the stack
    constexpr bool TOP = WIDE && !LDS_SCENE;
    int *const stk = LDS_SCENE ? lds + P.numNodes * ldsNodeF4 * 4 : lds + (TOP ? (P.topBytes >> 2) : 0u);
    int *const my = stk + threadIdx.x;
    const int qFirst = kCtrExt0 + cur * kWfShards;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // this iteration's rays = its segments; consume the generated work; shade/generate
        // of this iteration append to the other ray queue and the regenerate queue
        const Shards rays = load_shards(W.ctr, qFirst), gen = load_shards(W.ctr, kCtrGen);
        atomicAdd(&P.stats[0], (unsigned long long)rays.pre[kWfShards]);
        W.ctr[ctr_word(kCtrWork)] += gen.pre[kWfShards];
#pragma unroll
        for (int k = 0; k < kWfShards; ++k) {
            W.ctr[ctr_word(kCtrExt0 + (cur ^ 1) * kWfShards + k)] = 0;
            W.ctr[ctr_word(kCtrGen + k)] = 0;
        }
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
    const unsigned *queue = cur ? W.extQ1 : W.extQ0;
    // each wave drains its block's home shard first, then the others in turn (one fetch
    // counter per shard spreads the atomics over kWfShards lines)
    unsigned fs = blockIdx.x % kWfShards, left = kWfShards;
    unsigned fsCount = W.ctr[ctr_word(qFirst + int(fs))];
    unsigned poolNext = 0, poolEnd = 0;
    unsigned slot = kNone;
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
                slot = queue[fs * W.shardCap + qi];
                load_ray(W, slot, r);
                prepare(r);
                begin(T);
            }
            if (__ballot(need)) {  // this shard is drained
                fs = fs + 1 == kWfShards ? 0u : fs + 1;
                fsCount = W.ctr[ctr_word(qFirst + int(fs))];
                poolNext = poolEnd = 0;
                --left;
            }
        }
        need = false;
        if (!__any(busy(T))) break;
        do {
            if (WIDE)
                traverse_round_wide<nodeF4, STATS, FULL, QUANT, true, LDS_SCENE, TOP>(
                    T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit, S, P.topBytes);
            else
                traverse_round<nodeF4, STATS, FULL>(T, r, my, nodes, tris, nvis, ntest, pc, P.leafExit, P.nodeExit);
        } while (__popcll(__ballot(busy(T))) > unsigned(P.waveThreshold));
        if (slot != kNone && !busy(T)) {
            *reinterpret_cast<float2 *>(W.st + 4 * size_t(slot) + 3) = make_float2(T.bestT, __int_as_float(T.bestI));
            slot = kNone;
            need = true;
        }
    }
    if (STATS) {
        const unsigned long long a = wave_sum(nvis), b = wave_sum(ntest);
        if (__lane_id() == 0) {
            atomicAdd(&P.stats[2], a);
            atomicAdd(&P.stats[3], b);
        }
    }
}

// Shade and generate keep every shard an independent pipeline: block b works on shard
// b % kWfShards and appends back to the same shard, so a shard never holds more than its
// initial ceil(slots / kWfShards) entries.
template <bool FULL>
__global__ __launch_bounds__(kWfBlock) void wf_shade(WfParams W, int cur) {
    __shared__ unsigned lds[kWfBlock / 64 + 1];
    const MeshParams &P = W.mp;
    if (blockIdx.x == 0 && threadIdx.x < kWfShards) W.ctr[ctr_word(kCtrFetch + int(threadIdx.x))] = 0;
    const unsigned shard = blockIdx.x % kWfShards;
    const unsigned first = (blockIdx.x / kWfShards) * kWfBlock;
    const unsigned count = W.ctr[ctr_word(kCtrExt0 + cur * kWfShards + int(shard))];
    // the grid covers a full shard; blocks past this iteration's queue leave before the appends
    // (block-uniform: no thread of such a block appends, so none needs the barriers)
    if (first >= count) return;
    const unsigned local = first + threadIdx.x;
    bool again = false, finished = false;
    unsigned slot = kNone;
    if (local < count) {
        slot = (cur ? W.extQ1 : W.extQ0)[shard * W.shardCap + local];
        const float4 *p = W.st + 4 * size_t(slot);
        const float4 a = p[0], b = p[1], c = p[2], h = p[3];
        Slot q;
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
            store_slot(W, slot, q);
            again = true;
        } else {
            finished = true;  // absorbed: contributes 0
        }
        if (finished) {
            store_radiance(P.scratch, q.item, L0, L1, L2);
        }
    }
    block_append(again, slot, cur ? W.extQ0 : W.extQ1, W.shardCap, W.ctr, kCtrExt0 + (cur ^ 1) * kWfShards, lds);
    block_append(finished, slot, W.genQ, W.shardCap, W.ctr, kCtrGen, lds);
}

__global__ __launch_bounds__(kWfBlock) void wf_generate(WfParams W, int nxt, int countSamples) {
    __shared__ unsigned lds[kWfBlock / 64 + 1];
    const MeshParams &P = W.mp;
    const Shards sh = load_shards(W.ctr, kCtrGen);
    const unsigned count = sh.pre[kWfShards];
    if (countSamples && blockIdx.x == 0 && threadIdx.x == 0 && count)
        atomicAdd(&P.stats[1], (unsigned long long)count);  // the regenerate queue = finished samples
    const unsigned shard = blockIdx.x % kWfShards;
    const unsigned local = (blockIdx.x / kWfShards) * kWfBlock + threadIdx.x;
    // work items in queue order: base + (entries of lower shards) + position in this shard
    unsigned lower = 0, here = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k) {
        if (unsigned(k) == shard) {
            lower = sh.pre[k];
            here = sh.pre[k + 1] - sh.pre[k];
        }
    }
    const unsigned base = W.ctr[ctr_word(kCtrWork)];  // advanced by the next wf_extend
    // blocks with nothing to generate leave before the appends (block-uniform, see wf_shade)
    const unsigned first = local - threadIdx.x;
    if (first >= here || base + lower + first >= P.totalItems) return;
    const bool ok = local < here && base + lower + local < P.totalItems;
    unsigned slot = kNone;
    if (ok) {
        const unsigned item = base + lower + local;
        slot = W.genQ[shard * W.shardCap + local];
        Slot q;
        camera_sample(P, item, q.r, q.rng);
        q.tr = q.tg = q.tb = 1.0f;
        q.depth = 0;
        q.item = item;
        store_slot(W, slot, q, true);
    }
    block_append(ok, slot, nxt ? W.extQ1 : W.extQ0, W.shardCap, W.ctr, kCtrExt0 + nxt * kWfShards, lds);
}

using ExtFn = void (*)(WfParams, int);
template <bool STATS, bool FULL>
ExtFn ext_fn_fmt(bool lds, bool wide, bool quant) {
    if (lds) return wide ? wf_extend<STATS, true, FULL, true, false> : wf_extend<STATS, true, FULL, false, false>;
    if (!wide) return wf_extend<STATS, false, FULL, false, false>;
    return quant ? wf_extend<STATS, false, FULL, true, true> : wf_extend<STATS, false, FULL, true, false>;
}
ExtFn ext_fn(bool count, bool lds, bool full, bool wide, bool quant) {
    if (count) return full ? ext_fn_fmt<true, true>(lds, wide, quant) : ext_fn_fmt<true, false>(lds, wide, quant);
    return full ? ext_fn_fmt<false, true>(lds, wide, quant) : ext_fn_fmt<false, false>(lds, wide, quant);
}

}  // namespace

size_t wf_pool_words(unsigned slots, unsigned *shardCap) {
    // shards are closed pipelines (wf_shade/wf_generate): shard k never holds more than the
    // slots wf_init gave it
    const unsigned cap = (slots + kWfShards - 1) / kWfShards;
    *shardCap = cap;
    return size_t(slots) * kWfStateWords + size_t(3) * kWfShards * cap;
}

// kWfShards blocks per 1024 entries of one shard segment
static unsigned shard_grid(const WfParams &W) { return kWfShards * ((W.shardCap + kWfBlock - 1) / kWfBlock); }

hipError_t wf_launch_init(const WfParams &W, hipStream_t s) {
    hipLaunchKernelGGL(wf_init, dim3((W.slots + 255) / 256), dim3(256), 0, s, W);
    return hipGetLastError();
}

hipError_t wf_launch_generate(const WfParams &W, int nxt, bool countSamples, hipStream_t s, bool countOnly) {
    hipLaunchKernelGGL(wf_generate, dim3(countOnly ? unsigned(kWfShards) : shard_grid(W)), dim3(kWfBlock), 0, s, W, nxt,
                       countSamples ? 1 : 0);
    return hipGetLastError();
}

hipError_t wf_launch_extend(const WfParams &W, int cur, int blocks, bool countTraversal, hipStream_t s) {
    const MeshParams &P = W.mp;
    const bool lds = P.ldsScene != 0;
    if (P.topBytes && (lds || !P.wide || P.topBytes % (P.wide == 2 ? 64u : 128u) ||
                       P.topBytes > (unsigned(P.numNodes) << (P.wide == 2 ? 6 : 7))))
        return hipErrorInvalidValue;
    const size_t bytes = mesh_lds_bytes(P.stackDepth, lds ? P.numNodes : 0, lds ? P.numTris : 0, P.wide != 0, P.topBytes);
    const auto fn = ext_fn(countTraversal, lds, P.full != 0, P.wide != 0, P.wide == 2 && !lds);
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
