// hippt_device.h — launch parameter blocks shared by the host API (hippt_api.cpp) and the
// gfx950 kernels (hippt_kernels.hip).  Plain structs passed by value as kernel arguments.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hippt {

struct CameraF {  // layout == hipptCamera (include/hippt.h)
    float origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
    float lens_radius;
    float reserved;
};

// Legacy 4-sphere scene (CudaPathTracerKernel.cu:136-179).
struct Sphere4Params {
    float4 *accum;      // rows*width RGBA
    uint32_t *out;      // rows*width ARGB
    unsigned long long *stats;
    int width, height, y0, rows, rowStride;  // image rows y0 + k*rowStride, k < rows
    int firstFrame, frames, maxDepth;
    int format;  // kPixelArgb / kPixelRgba8
    uint32_t *hostOut;  // null, or the W*H full frame in pinned host memory (device-mapped)
};

// Pixel word formats of the output frame (HIPPT_OPT_PIXEL_FORMAT)
enum { kPixelArgb = 0, kPixelRgba8 = 1 };

// Running average + tonemap over a batch of per-sample radiances
// (CudaPathTracerKernel.cu:157-178).
struct CombineParams {
    float4 *accum;
    uint32_t *out;
    const float *scratch;
    unsigned bandPixels, totalItems;
    int firstFrame, frames;
    int format;  // kPixelArgb / kPixelRgba8
};

// combine_kernel's output words also into the pinned full W*H host frame (device-mapped; a
// blocking frame), band pixel p at row y0 + (p / width) * stride; host null: device words only
struct HostFrame {
    uint32_t *host;
    int width, y0, stride;
};

// Mesh megakernel: one persistent grid drains `totalItems` (pixel, frame) samples of the band's
// rows and frames [firstFrame, firstFrame+frames).
struct MeshParams {
    const float4 *nodes;   // 4 float4 per interior node (bvh_builder.h layout)
    // 3 float4 per primitive, BVH leaf order, tag = third .z (int bits):
    //   triangle (tag 0): (v0, e1.x) (e1.yz, e2.xy) (e2.z, prim id, 0, -)
    //   sphere   (tag 1): (center, radius) (radius^2, -, -, -) (-, prim id, 1, -)
    const float4 *tris;
    // 1 float4 per primitive: triangle (unit normal, material), sphere (center, material |
    // kShadeSphere); material index as int bits
    const float4 *shade;
    const float4 *mats;    // 2 float4 per material: (albedo rgb, kind) (fuzz, ir, -, -)
    float *scratch;        // per-sample radiance, RGB float triples (12 B) in item order
    unsigned *queue;       // kQueues work counters, 128 B apart (zeroed before launch)
    unsigned long long *stats;  // [0] segments, [1] pixel samples, [2] node visits, [3] tri tests
    CameraF cam;
    float invW, invH;      // 1/max(1,W-1), 1/max(1,H-1) (RayTracerFboItem.cpp:61-64)
    int width, height, y0, bandRows, rowStride;  // band row k is image row y0 + k*rowStride
    int firstFrame, frames, maxDepth;
    unsigned bandPixels, totalItems;
    float rcpBandPixels, rcpWidth;  // 1/bandPixels, 1/width for the item -> (frame, x, y) split
    int stackDepth;        // LDS stack entries per lane (>= BVH interior levels)
    int numNodes, numTris, numMats;
    int ldsScene;          // 1: copy nodes/triangles/shading into LDS (small scenes)
    int full;              // 1: spheres or non-Lambertian materials present (general kernel)
    int waveThreshold;     // shade once fewer than this many lanes still traverse
    unsigned chunk;        // items per queue grab (multiple of 64)
    unsigned leafExit;     // node loop exits once <= leafExit lanes still search for a leaf
    unsigned nodeExit;     // leaf loop exits once <= nodeExit lanes still hold a leaf (0: never)
    // Node format (kWide*): 0 the 2-wide tree; 1 the 4-wide tree (Bvh4 layout, 8 float4 per node);
    // 2 quantize_bvh4 layout (4 float4 per node; global-memory scenes only); 3 hybrid_bvh4 (the
    // top's topBytes as float nodes, read from LDS, then 8-bit nodes; global-memory scenes only);
    // 4 half_bvh4 (128-byte nodes of half-precision planes, the Bvh4 codes; global-memory scenes).
    // LDS stack content capacity and the per-lane spill area (spillCap entries per lane of the
    // persistent grid; null if never used)
    int wide;
    int stackCap;
    int spillCap;
    int *spill;
    // 4-wide trees in global memory: bytes of the node array's prefix (the top of the tree,
    // breadth-first, bvh_builder.h order_bvh4_top) copied to LDS address 0 and read from there
    unsigned topBytes;
    // LDS-resident 4-wide trees: low bits of a packed child key that carry the child's code
    // (trace::child_key_p; hippt_api.cpp packed_ref_bits)
    unsigned refBits;
    // The queues' order of the batch's items (item_order.h build_item_table): queue position
    // fl*bandPixels + 64*j + k is item k of the run at runOrder[fl*runCount + j] for j < runCount
    // (runs of 64 band pixels per frame: consecutive pixels, or a tile when flagged, item_order.h);
    // null: image order.
    const unsigned *runOrder;
    unsigned runCount;
    // log2 of a tile run's columns (item_order.h RunLayout; entries flagged kRunTile are tiles)
    unsigned runTileShift;
    // random_in_unit_sphere memoized (null: the rejection loop): entry 2^32-word table, see
    // launch_rng_table
    const uint32_t *rngTable;
    // camera-ray pool (HIPPT_OPT_CAMERA_POOL): each wave's 64 pre-generated camera rays at LDS byte
    // poolOffset + wave * poolWords * 256, poolWords fields of 64 words each: item, rng, d.xyz and,
    // unless the camera is a pinhole at a nonzero origin (every ray starts at cam.origin), o.xyz
    unsigned poolOffset;
    int poolWords;
    // the previous batch's running average + tonemap, done by this launch's waves between their
    // paths (its scratch is the other buffer): comb.bandPixels == 0 for none; chunks of 64 pixels
    // claimed from *combCtr (zeroed with the work queue)
    CombineParams comb;
    unsigned *combCtr;
    // Chained batches (chainCtl non-null; hippt_trace.h "chained batches").  A run is a
    // sequence of asynchronous batches with the same scene, camera, rows and frames per batch, each
    // rendering the same frames again or the next ones; batch t of the run (t = 0, 1, ...) has ring
    // slot t % chainSlots: its work counters are the slot's block of chainCtl, its radiances start
    // at sample slot << chainShift of `scratch`, and its items carry the slot above bit chainShift
    // (so store_radiance is unchanged).  This launch is the run's launch number chainEpoch and was
    // enqueued for batch chainSeq; it combines every batch that earlier launches finished and did not
    // combine, then traces from the first batch no launch has taken, going on with the later batches
    // the host has posted (*chainBox = run << 33 | consecutive frames << 32 | last posted batch) up to
    // chainCap batches and the ring's free slots.  comb.* (frames, bandPixels, format, accum, out)
    // describe every batch of the run; comb.firstFrame is batch 0's first frame and chainStep the
    // frames from one batch to the next (-1: not known when enqueued; read from the mailbox).
    unsigned *chainCtl;
    const unsigned long long *chainBox;
    unsigned chainSeq, chainEpoch, chainRun;
    unsigned chainSlots, chainShift, chainCap;
    int chainStep;
    unsigned chainPosted;  // the run's last batch posted when the launch was enqueued (>= chainSeq)
    // batches chainSeq .. chainSeq + chainGroup - 1 are this launch's own group, traced as one job: one
    // set of queues over their items, each queue's cost order walked once for the whole group (64-item
    // runs of the group's batches interleaved); 1: the own batch alone
    unsigned chainGroup;
    // HIPPT_OPT_CHAIN_AUDIT: the run's audit records (kAuditBatches + 1 records of kAuditWords words:
    // per batch what was traced and combined, hipptChainAudit), or null
    unsigned *chainAudit;
};

// Chained batches: the control block (unsigned words).  Ring slot k's block at k * kChainBlockWords:
// the kQueues work counters 128 B apart, then (own line) a 64-bit marker (batch << 32 | launch + 1) of
// the last launch that took a batch in this slot.  After the kChainSlotsMax blocks, at kChainCtlWord:
// the first batch not yet combined after the launches of epoch parity 0 / 1 (+0 / +32), the combine
// chunk counters of epoch parity 0 / 1 (+64 / +96).
constexpr unsigned kChainSlotsMax = 32, kChainBlockWords = 8 * 32 + 32, kChainMarkerWord = 8 * 32;
constexpr unsigned kChainCtlWord = kChainSlotsMax * kChainBlockWords;
// (+128: kQueues device copies of the host mailbox, one 128-byte line each, for the blocks of one
// XCD: the copy (64-bit), the realtime stamp of its last completed refresh, the stamp of the last
// claimed refresh)
constexpr unsigned kChainBoxWord = kChainCtlWord + 128, kChainCtlWords = kChainBoxWord + 8 * 32;
// batches of at most 2^kChainMaxShift items chain (the slot bits above them, kNone above all)
constexpr unsigned kChainMaxShift = 27;
// camera-pool kernels: per-wave state words in LDS before each wave's pool (trace::WaveWords)
constexpr unsigned kWaveWords = 22;

// The chain's final combine (launch_chain_flush): every batch of the run that no launch combined,
// [first uncombined (from the control block, launch epoch `epoch`), lastSeq], in order per pixel.
struct ChainFlushParams {
    CombineParams comb;  // as MeshParams::comb (comb.firstFrame: batch 0's first frame)
    const float *scratch;
    const unsigned *ctl;
    unsigned epoch, lastSeq, slots, shift;
    int step;
    unsigned *audit;  // MeshParams::chainAudit
};

// Chained-batch audit records (HIPPT_OPT_CHAIN_AUDIT, include/hippt.h hipptChainAudit): per run, one
// record of kAuditWords words per batch below kAuditBatches and one pooled record for the rest;
// kAuditRuns runs' records per context on the device.
constexpr unsigned kAuditBatches = 256, kAuditWords = 16, kAuditRuns = 64;
constexpr unsigned kAuditRunWords = (kAuditBatches + 1) * kAuditWords;


// MeshParams::wide
enum { kWide2 = 0, kWideFloat = 1, kWideQuant = 2, kWideHybrid = 3, kWideHalf = 4 };

// Material kinds (RayTracer.h:473-540) and the sphere flag of a shading record.
enum { kLambertian = 0, kMetal = 1, kDielectric = 2 };
constexpr int kShadeSphere = 1 << 30;

// The LDS-scene kernels read the node copy at LDS address 0 (trace::lds_ld4): true when the
// kernel has no static LDS, so that its dynamic LDS starts at address 0.
inline hipError_t check_lds_at_zero(const void *kernel) {
    hipFuncAttributes a{};
    const hipError_t e = hipFuncGetAttributes(&a, kernel);
    if (e != hipSuccess) return e;
    return a.sharedSizeBytes == 0 ? hipSuccess : hipErrorInvalidDeviceFunction;
}

hipError_t launch_sphere4(const Sphere4Params &p, hipStream_t s);
hipError_t launch_mesh(const MeshParams &p, int blocks, bool countTraversal, hipStream_t s);
hipError_t launch_combine(const CombineParams &p, hipStream_t s, const HostFrame &h = HostFrame{});
hipError_t launch_chain_flush(const ChainFlushParams &p, hipStream_t s);
// random_in_unit_sphere's rejection loop (RayTracer.h:155-161 with the hash RNG and the short-cycle
// escape) is a pure function of the RNG state it starts from: table[s] = the state from which the
// accepted candidate's three draws are made.  One 32-bit word per state: 16 GiB.
constexpr size_t kRngTableBytes = size_t(4) << 32;
hipError_t launch_rng_table(uint32_t *table, hipStream_t s);
// Resident mesh-kernel blocks per CU for a given LDS stack depth and LDS scene size.
int mesh_blocks_per_cu(bool countTraversal, bool full, int fmt, int stackDepth, int ldsNodes, int ldsTris, bool spill,
                       unsigned topBytes = 0, int ldsMats = 0, int poolWords = 0, bool chain = false);
// (poolWords != 0: each wave's pool block also holds its kWaveWords state words)
size_t mesh_lds_bytes(int stackDepth, int ldsNodes, int ldsTris, bool wide, unsigned topBytes = 0, int ldsMats = 0,
                      int poolWords = 0);
// camera-ray pool words per ray: item, rng, direction (+ origin unless every ray starts at the
// camera origin)
constexpr int kPoolWordsPinhole = 5, kPoolWordsFull = 8;
// LDS bytes per block that keep the persistent grid's resident blocks within a CU's LDS
size_t mesh_lds_block_budget();
size_t mesh_lds_scene_limit();
constexpr int kMeshBlock = 256;
// Launch counters (MeshParams::stats, Sphere4Params::stats): kStatSlots copies of kStatWords
// words ([0..3] hipptStats counters, [4..19] phase profile, [20..24] hit-children histogram),
// block b adding into copy b % kStatSlots; the host sums the copies.  One shared copy took every
// wave's end-of-launch atomics on one cache line: ~50 us of each megakernel launch's tail
// (7168 waves x 2), and ~0.3 ms of a 1080p legacy frame (32k waves).
constexpr int kStatWords = 32, kStatSlots = 64;
// megakernel work queues (one per XCD; hippt_trace.h queue_start splits the items evenly)
constexpr unsigned kMeshQueues = 8;
// LDS-resident scene copies: 2-wide nodes at an 80-byte stride, 4-wide nodes in the 128-byte
// global layout (the octant row addressing by or/xor needs 128-byte alignment; a 144- or
// 160-byte stride cut the LDS bank conflicts of node rows by 40% but not the kernel time, and
// the add-based addressing it needs costs registers: spills in the general kernels).
constexpr int kLdsNodeF4 = 5;
constexpr int kLdsNode4F4 = 8;

}  // namespace hippt
