// hippt_wavefront.h — host-side launch interface of the wavefront variant (hippt_wavefront.hip).
#pragma once

#include "hippt_device.h"

namespace hippt {

// Path-state pool: one 64-byte record (four float4) per slot.  Queue entries point at slots
// in an order that scrambles as paths end and compact, so a record costs one cache line per
// lane where separate arrays would cost one line per field.
//   [0] ox oy oz dx   [1] dy dz tr tg   [2] tb rng depth item   [3] hitT hitI - -
constexpr int kWfStateWords = 16;

// Queues are split into kWfShards segments, each with its own counter; a 1024-thread block
// appends to segment blockIdx % kWfShards with one atomic (contention on one counter word
// caps at ~88 atomics/us, MI355X_MICROARCH.md "dequeue").
constexpr int kWfShards = 8;
constexpr int kWfBlock = 1024;

// Device counters (W.ctr): ray-queue shard sizes (double-buffered), regenerate-queue shard
// sizes, the extend kernel's per-shard fetch counters, and the work-item base.  Counter c
// lives at word c * kCtrStride: one 128-byte line each, so atomics on different counters do
// not serialise on a shared line.
enum {
    kCtrExt0 = 0,
    kCtrExt1 = kWfShards,
    kCtrGen = 2 * kWfShards,
    kCtrFetch = 3 * kWfShards,
    kCtrWork = 4 * kWfShards,
    kCtrCount = 4 * kWfShards + 1
};
constexpr int kCtrStride = 32;
constexpr int kCtrWords = kCtrCount * kCtrStride;
__host__ __device__ constexpr int ctr_word(int c) { return c * kCtrStride; }

struct WfParams {
    MeshParams mp;  // scene, camera, image band, batch, scratch, stats
    float4 *st;  // slots records
    unsigned *extQ0, *extQ1, *genQ;  // kWfShards segments of shardCap entries each
    unsigned *ctr;
    unsigned slots, shardCap;
};

// Words of the pool: state + three queues of kWfShards segments of ceil(slots/kWfShards).
size_t wf_pool_words(unsigned slots, unsigned *shardCap);
hipError_t wf_launch_init(const WfParams &W, hipStream_t s);
// countSamples: the regenerate queue holds finished samples (false for the initial fill).
// countOnly: nothing is left to generate (every work item of the batch was generated up front);
// one block per shard only counts the finished samples
hipError_t wf_launch_generate(const WfParams &W, int nxt, bool countSamples, hipStream_t s, bool countOnly = false);
hipError_t wf_launch_extend(const WfParams &W, int cur, int blocks, bool countTraversal, hipStream_t s);
hipError_t wf_launch_shade(const WfParams &W, int cur, hipStream_t s);
int wf_extend_blocks_per_cu(bool countTraversal, bool full, bool wide, bool quant, int stackDepth, int ldsNodes,
                            int ldsTris, unsigned topBytes = 0);

}  // namespace hippt
