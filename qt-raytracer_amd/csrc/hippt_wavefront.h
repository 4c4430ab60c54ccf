// hippt_wavefront.h — host-side launch interface of the wavefront variant (hippt_wavefront.hip).
#pragma once

#include "hippt_device.h"

namespace hippt {

// Ray queues with their payload: queue q's entry i is a path's state in three float4 arrays,
//   ra[q][i] = ox oy oz dx   rb[q][i] = dy dz tr tg   rc[q][i] = tb rng depth item,
// and hit[i] = (t, primitive) of queue cur's entry i after wf_extend.  wf_shade appends a
// scattered path to the other queue in block order, so every kernel reads and writes these
// arrays in whole cache lines (no slot indirection: a scrambled slot order cost a line per lane).
constexpr int kWfWordsPerSlot = 2 * 3 * 4 + 2;

// Queues are split into kWfShards segments, each with its own counter; a 1024-thread block
// appends to segment blockIdx % kWfShards with one atomic (contention on one counter word
// caps at ~88 atomics/us, MI355X_MICROARCH.md "dequeue").
constexpr int kWfShards = 8;
constexpr int kWfBlock = 1024;

// Device counters (W.ctr): per queue, its shards' appended entries then the entries wf_generate
// added after them; the extend kernel's per-shard fetch counters; the work items generated so
// far.  Counter c lives at word c * kCtrStride: one 128-byte line each, so atomics on different
// counters do not serialise on a shared line.
enum {
    kCtrFetch = 4 * kWfShards,
    kCtrWork = 5 * kWfShards,
    kCtrCount = 5 * kWfShards + 1
};
__host__ __device__ constexpr int ctr_queue(int q) { return 2 * kWfShards * q; }
__host__ __device__ constexpr int ctr_gen(int q) { return 2 * kWfShards * q + kWfShards; }
constexpr int kCtrStride = 32;
constexpr int kCtrWords = kCtrCount * kCtrStride;
__host__ __device__ constexpr int ctr_word(int c) { return c * kCtrStride; }

struct WfParams {
    MeshParams mp;  // scene, camera, image band, batch, scratch, stats
    float4 *ra[2], *rb[2], *rc[2];  // the two ray queues' payload (kWfShards segments of shardCap)
    float2 *hit;
    unsigned *ctr;
    unsigned slots, shardCap;
    // Coherence sort of the scattered paths (HIPPT_OPT_WAVEFRONT_SORT): wf_shade appends each
    // block's paths in the order of a key, so that a wave of wf_extend takes rays of one direction
    // octant (sortBits 3) and, with sortBits 6, one cell of a 2x2x2 grid over the scene's box
    // (cell c on axis a: (o_a - sortLo[a]) * sortScale[a] in [c, c+1)); 0: append in thread order.
    unsigned sortBits;
    float sortLo[3], sortScale[3];
};

// Words of the queues: 2 x 3 float4 + the hit float2 per entry, kWfShards segments of
// ceil(slots/kWfShards) entries.
size_t wf_pool_words(unsigned slots, unsigned *shardCap);
hipError_t wf_launch_init(const WfParams &W, hipStream_t s);
// New paths into queue nxt's free capacity while work items remain.
hipError_t wf_launch_generate(const WfParams &W, int nxt, hipStream_t s);
hipError_t wf_launch_extend(const WfParams &W, int cur, int blocks, bool countTraversal, hipStream_t s);
hipError_t wf_launch_shade(const WfParams &W, int cur, hipStream_t s);
int wf_extend_blocks_per_cu(bool countTraversal, bool full, bool wide, bool quant, int stackDepth, int ldsNodes,
                            int ldsTris, unsigned topBytes = 0);

}  // namespace hippt
