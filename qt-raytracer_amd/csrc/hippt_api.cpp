// hippt_api.cpp — C ABI of libhippt.so (include/hippt.h).
//
// Owns all device state, like the reference's single global CudaState
// (CudaPathTracerKernel.cu:12-21), but:
//   * one context per device, each rendering a contiguous row band of the image
//     (multi-GPU; no collective — bands are gathered on the host);
//   * every entry point is serialised by a mutex (the reference is called from the GUI
//     thread and the QSG render thread without a lock, RayTracerFboItem.cpp:261,521,529);
//   * triangle-mesh scenes with a host-built SAH BVH in addition to the reference's
//     built-in 4-sphere scene.
#include "../../include/hippt.h"
#include "item_order.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <utility>
#include <vector>

#include "bvh_builder.h"
#include "mesh_io.h"
#include "hippt_device.h"
#include "hippt_wavefront.h"

struct hipptBvh {
    hippt::Bvh bvh;
    hippt::Bvh4 bvh4;
    std::vector<uint32_t> bvh4q;
};

namespace {

using hippt::CameraF;

using hippt::kStatSlots;
using hippt::kStatWords;
constexpr size_t kStatBytes = size_t(kStatSlots) * kStatWords * sizeof(unsigned long long);


// 4-wide traversal: LDS stack content capacity for scenes outside LDS (19 + 3 spare entries =
// 22 KB per 256-lane block: 7 blocks per CU in 160 KB).
constexpr int kWideStackCap = 19;
// a tree that spills anyway keeps 10 entries and gives the rest to the top of the tree (r3al,
// alternating on leaf-2 trees: blob70k 1080p +0.5%, 4K +0.6% over 13; r3q before: +0.6%)
constexpr int kSpillStackCap = 10;
// 4-wide trees are numbered breadth-first for their first kTopOrderNodes nodes, so that a prefix
// of the node array is the top of the tree; trees read from global memory keep such a prefix in
// LDS (HIPPT_OPT_LDS_TOP_NODES)
constexpr int kTopOrderNodes = 1365;  // 6 complete levels
// hippt_trace.h kQueues x kQueueStride work counters, then (its own line) the fused combine's
// chunk counter (MeshParams::combCtr)
constexpr size_t kCombCtrWord = 8 * 32;
constexpr size_t kQueueBytes = (kCombCtrWord + 32) * sizeof(unsigned);

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};

#ifndef HIPPT_LEGACY_ZERO_COPY
#define HIPPT_LEGACY_ZERO_COPY 1
#endif
constexpr bool kLegacyZeroCopy = HIPPT_LEGACY_ZERO_COPY != 0;

// The key of a context's run-cost estimates (item order): what the estimate depends on.
struct OrderKey {
    int version = -1, width = 0, height = 0, y0 = 0, rows = 0, stride = 0, maxDepth = 0;
    unsigned tileShift = 6;  // the runs' shape (item_order.h RunLayout)
    CameraF cam{};
};

bool same_key(const OrderKey &a, const OrderKey &b) {
    if (a.version != b.version || a.width != b.width || a.height != b.height || a.y0 != b.y0 || a.rows != b.rows ||
        a.stride != b.stride || a.maxDepth != b.maxDepth || a.tileShift != b.tileShift ||
        a.cam.lens_radius != b.cam.lens_radius)
        return false;
    for (int k = 0; k < 3; ++k)
        if (a.cam.origin[k] != b.cam.origin[k] || a.cam.llc[k] != b.cam.llc[k] ||
            a.cam.horizontal[k] != b.cam.horizontal[k] || a.cam.vertical[k] != b.cam.vertical[k] ||
            a.cam.u[k] != b.cam.u[k] || a.cam.v[k] != b.cam.v[k])
            return false;
    return true;
}

// Run costs computed on a detached host thread (HIPPT_OPT_ITEM_ORDER automatic).  The thread owns a
// reference to its job and reads only the job's copies of the tree and primitives, so scene uploads,
// renders and process exit never wait for it: a context that no longer wants the result drops its
// reference (abandon_cost_job), and no joinable std::thread is ever destroyed (a
// function-local static State destroyed at exit with a joinable thread called std::terminate).
struct CostJob {
    OrderKey key;
    hippt::Bvh4 bvh;
    std::vector<float4> tris;
    std::vector<float> cost;
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    bool finished() {
        std::lock_guard<std::mutex> g(mu);
        return done;
    }
    void wait() {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [this] { return done; });
    }
};

struct Ctx {
    int device = 0;
    int y0 = 0, rows = 0, stride = 1;  // image rows y0, y0+stride, ... (rows of them)
    hipStream_t stream = nullptr;
    float4 *accum = nullptr;
    uint32_t *out = nullptr;
    float *scratch = nullptr;
    size_t scratchBytes = 0;
    // Megakernel batches defer their combine (running average + tonemap) into the next batch's
    // launch on this context, which does it between its paths (MeshParams::comb); the two batches'
    // per-sample radiances then live in two buffers.  Flushed (a combine launch of its own) before
    // anything reads or resets the image: sync, present, copies, reset, a non-megakernel batch.
    float *scratchAlt = nullptr;
    size_t scratchAltBytes = 0;
    hippt::CombineParams deferred{};
    hippt::HostFrame deferredHost{};  // a blocking frame's flush: the words into the host frame too
    bool hasDeferred = false;
    unsigned *queue = nullptr;
    unsigned long long *stats = nullptr;
    int sceneVersion = -1;
    float4 *nodes = nullptr, *tris = nullptr, *shade = nullptr, *mats = nullptr;
    float4 *nodes4 = nullptr;  // 4-wide BVH (same primitive order as nodes)
    float4 *nodes4q = nullptr; // the 4-wide BVH with 8-bit child boxes
    float4 *nodes4h = nullptr; // hybrid layout (float top + 8-bit nodes) for hybridTop top nodes
    float4 *nodes4f = nullptr; // the 4-wide BVH with half-precision planes (half_bvh4; on use)
    int halfVersion = -1;      // scene version of nodes4f
    int hybridTop = -1;
    // the queues' pixel-run order of this context's rows (HIPPT_OPT_ITEM_ORDER): run costs per key,
    // device item tables per batch size for those costs
    OrderKey orderKey;            // of runCosts
    std::vector<float> runCosts;  // per run of 64 band pixels (item_order.h run_costs)
    bool runCostsValid = false;
    struct OrderTable {
        int frames;
        unsigned *dev;
    };
    std::vector<OrderTable> orderTables;  // most recently used first, at most kOrderTables
    struct RetiredTable {
        unsigned *dev;
        hipEvent_t done;  // recorded on the stream after the last launch that may read it
    };
    std::vector<RetiredTable> retiredTables;
    std::shared_ptr<CostJob> costJob;  // automatic mode: the costs of a new key, off the render path
    int *spill = nullptr;      // 4-wide traversal: per-lane stack spill area
    size_t spillBytes = 0;
    // wavefront path-state pool (allocated on first use)
    void *wfPool = nullptr;
    unsigned wfSlots = 0;  // slots allocated
    unsigned wfWant = 0;   // slots asked for when the pool was allocated (>= wfSlots)
    unsigned *wfCtr = nullptr;
    unsigned *wfHost = nullptr;  // pinned: two snapshots of the ray-queue shard counters
    hipEvent_t wfPoll[2] = {nullptr, nullptr};
    long long wfOccKey = -1;  // occupancy cached per (scene version, depth, lds, full)
    int wfBlocksPerCu[2] = {0, 0};
    int cus = 0;
    long long occKey = -1;  // occupancy cached per (scene version, depth, lds, full)
    int meshBlocksPerCu[2] = {0, 0};
    int meshBlocksPerCuChain = 0;  // the chained-batch kernel's
    // Chained batches (HIPPT_OPT_CHAIN; MeshParams::chain*, hippt_trace.h): the open run.  Its launches
    // share a ring of `slots` scratch slots and work-counter blocks (chainCtl, zeroed when a run
    // starts); the host posts each batch in the mailbox (run << 33 | consecutive << 32 | batch) before
    // its launch is enqueued, and the run's last combines are a flush before anything reads or
    // resets the image (flush_deferred).
    struct Chain {
        bool live = false;   // a run is open
        unsigned run = 0;    // its id
        unsigned seq = 0;    // the next batch's number in the run
        unsigned epoch = 0;  // the next launch's number in the run
        int firstFrame = 0;  // batch 0's first frame
        int step = -1;       // frames from one batch to the next (-1: one batch so far)
        unsigned slots = 0, shift = 0, cap = 0;
        hippt::MeshParams key{};  // what every batch of the run shares (chain_same)
        long long blocks = 0;
        unsigned lastOwn = 0;     // the batch of the run's last enqueued launch
        // batches held for one group launch while the run's last launch has not started (chain_batch):
        // the first one's parameters and their count; flush_chain launches them if the run ends first
        unsigned pendN = 0;
        hippt::MeshParams pendP{};
        unsigned *audit = nullptr;  // the run's audit records (HIPPT_OPT_CHAIN_AUDIT), or null
    } chain;
    // HIPPT_OPT_CHAIN_AUDIT: kAuditRuns runs' records on the device (run k in slab k % kAuditRuns) and
    // the headers of the runs not yet copied to the host (State::auditWords), oldest first
    unsigned *auditDev = nullptr;
    unsigned auditNext = 0;
    struct AuditRun {
        unsigned hdr[hippt::kAuditWords];
        unsigned slab;
        bool closed;
    };
    std::vector<AuditRun> auditRuns;
    hipEvent_t chainStartEv = nullptr;  // recorded before each chained launch (chain_batch's hold test)
    hipEvent_t chainEndEv = nullptr;    // recorded after each chained launch (chain_batch's hold test)
    unsigned *chainCtl = nullptr;
    float *chainScratch = nullptr;
    size_t chainScratchBytes = 0;
    unsigned long long *chainBox = nullptr;     // pinned, coherent mailbox word
    unsigned long long *chainBoxDev = nullptr;  // its device address
    // pixel samples of chained batches (their kernels do not count them: every item is one sample)
    unsigned long long hostSamples = 0;
    std::vector<EventPair> pool;                         // every timing event pair created
    std::vector<EventPair> freeEv;                       // pairs not in flight
    std::vector<std::pair<int, EventPair>> pending;      // (0 trace / 1 combine, events)
    hipEvent_t presentEv[2] = {nullptr, nullptr};        // band copy into State::present[b] done
};

struct SceneHost {
    int kind = HIPPT_SCENE_SPHERE4;
    int version = 0;
    std::vector<float4> nodes, tris, shade, mats;  // device layouts (hippt_device.h MeshParams)
    int numTris = 0, numNodes = 0, levels = 0;  // numTris: primitive records (triangles + spheres)
    std::vector<float4> nodes4;                 // 4-wide BVH (bvh_builder.h Bvh4)
    std::vector<float4> nodes4q;                // quantize_bvh4 of it
    std::vector<float4> nodes4f;                // half_bvh4 of it (device codes; built on use)
    int halfState = 0;                          // nodes4f: 0 not built, 1 built, -1 out of half range
    hippt::Bvh4 bvh4;                           // the 4-wide tree with node-index codes ...
    std::vector<uint32_t> q4;                   // ... and its 8-bit nodes (hybrid_bvh4 inputs)
    std::vector<float4> hybrid;                 // hybrid_bvh4 for hybridTop top nodes (built on use)
    int hybridTop = -1;
    int numNodes4 = 0, levels4 = 0, stackBound4 = 0;
    bool full = false;                          // spheres or non-Lambertian materials
    double lookfrom[3] = {0, 0, 0}, lookat[3] = {0, 0, -1}, vup[3] = {0, 1, 0};
    double vfov = 90, aperture = 0, focus = 1;
    bool rawCamera = false;
    CameraF cam{};
};

struct State {
    std::mutex mu;
    bool ready = false;
    int width = 0, height = 0;
    int rowY0 = 0, rowY1 = 0;              // process rows: range [rowY0, rowY1) ...
    int rowPhase = 0, rowStride = 1;       // ... or every rowStride-th row from rowPhase
    bool deviceInterleave = true;          // devices of this process: interleaved rows (else bands)
    std::vector<int> devices;
    std::vector<Ctx> ctxs;
    unsigned *host = nullptr;  // pinned W*H ARGB frame (library-owned, as gState.hostOutput)
    size_t hostCount = 0;
    // asynchronous hand-off (hipptRenderFramesPresent / hipptLatestFrame): two pinned frames
    unsigned *present[2] = {nullptr, nullptr};
    int presentNext = 0;                 // buffer the next present call writes
    bool presentPending[2] = {false, false};
    long long presentSeq[2] = {-1, -1};  // present call number of the buffer's contents
    int presentFrames[2] = {0, 0};       // frames accumulated in that image
    long long presentCalls = 0;
    int latest = -1;                     // newest completed buffer
    SceneHost scene;
    char error[256] = {0};
    // options
    bool countTraversal = false;
    int waveThreshold = -1;  // -1: automatic (24 for LDS scenes and the general kernel, 40 for Lambertian scenes over trees in global memory)
    // one batch (and one end-of-batch tail) per call up to 4K/256 spp: 2.12G samples x 12 B
    long long scratchMB = 32768;
    unsigned chunk = 0;  // work items per claim (0: automatic, see enqueue_locked)
    int leafExit = -1;  // -1: automatic from the tree depth and LDS residency
    int nodeExit = -1;  // -1: automatic
    int bvhWidth = 0;   // megakernel traversal over the 2- or 4-wide BVH; 0: 4-wide if it fits in LDS
    int stackCap = 0;   // 4-wide LDS stack entries (0: automatic)
    int bvhQuant = -1;  // 4-wide global-memory traversal over 8-bit child boxes (-1: automatic)
    int ldsTopNodes = -1;  // top-of-tree nodes copied into LDS for global-memory trees (-1: automatic)
    bool rngTable = false;  // memoized random_in_unit_sphere (HIPPT_OPT_RNG_TABLE)
    int pixelFormat = HIPPT_PIXEL_ARGB;  // output frame words (HIPPT_OPT_PIXEL_FORMAT)
    int cameraPool = -1;  // megakernel camera-ray pool (HIPPT_OPT_CAMERA_POOL; -1: automatic)
    int fuseCombine = -1;  // combine inside the next megakernel launch (HIPPT_OPT_FUSE_COMBINE)
    int itemOrder = -1;    // scene-hitting pixel runs first (HIPPT_OPT_ITEM_ORDER; -1: automatic)
    int pixelTile = -1;    // the item order's runs: tile columns (HIPPT_OPT_PIXEL_TILE; 0 rows, -1 automatic)
    int chainBatches = -1; // batches a chained launch may trace (HIPPT_OPT_CHAIN; 0 off, -1 automatic)
    bool chainAudit = false;            // HIPPT_OPT_CHAIN_AUDIT
    std::vector<unsigned> auditWords;   // closed runs' audit words not yet read (hipptChainAudit)
    std::vector<std::pair<int, uint32_t *>> rngTables;  // per device, built on first use
    // The big work buffers (sample scratch, chain ring, spill area) of the contexts a re-initialization
    // destroyed, kept for the new contexts of the same device: a fresh hipMalloc of a 13 GB ring took
    // up to 5.9 s and its hipFree ~0.29 s (r6ae/r6af), a stall on the first render after every resize.
    // Held for one initialization; cudaPathTracerShutdown frees them.
    struct SpareBuf {
        int device;
        void *ptr;
        size_t bytes;
    };
    std::vector<SpareBuf> spare;
    unsigned activeTopBytes = 0;  // of the last mesh render (hipptGetOption HIPPT_INFO_*)
    int activeBlocksPerCu = 0;
    int activeChunk = 0;     // the last megakernel batch's claim size
    int activeChainCap = 0;  // its run's chain cap (0: not chained)
    int activeWidth = 0;  // BVH width of the last mesh render (hipptActiveBvhWidth)
    int blocksPerCu = 0;
    bool ldsScene = true;
    int pathMode = 0;             // 0 megakernel, 1 wavefront
    // wavefront path-state slots per device: 2^27 holds a whole 1080p/64-spp step in flight (one
    // generation, no regenerate rounds; 8.6 GB of 64-byte records): blob70k 6.8 -> 7.4+ G vs 2^24
    unsigned wfSlots = 1u << 27;
    int wfSort = -1;  // wavefront coherence sort key bits (HIPPT_OPT_WAVEFRONT_SORT: 0, 3, 6; -1 automatic)
    hippt::BvhParams bvh;         // applied at the next scene upload
    // host-side timing accumulators
    double traceMs = 0, combineMs = 0;
    int traceLaunches = 0, combineLaunches = 0;
};

State &S() {
    static State s;
    return s;
}

// A kept buffer of `device` of at least `need` bytes (the smallest such), or null.
void *spare_take(int device, size_t need, size_t *bytes) {
    auto &v = S().spare;
    size_t best = v.size();
    for (size_t k = 0; k < v.size(); ++k)
        if (v[k].device == device && v[k].bytes >= need && (best == v.size() || v[k].bytes < v[best].bytes)) best = k;
    if (best == v.size()) return nullptr;
    void *p = v[best].ptr;
    *bytes = v[best].bytes;
    v.erase(v.begin() + long(best));
    return p;
}

void spare_free_all() {
    for (auto &b : S().spare) {
        (void)hipSetDevice(b.device);
        (void)hipFree(b.ptr);
    }
    S().spare.clear();
}

// hipMalloc of a big work buffer, or a kept one of the same device (spare_take); *bytes = its size,
// set only on success (a failed allocation leaves the caller's buffer empty, size 0).
hipError_t work_malloc(int device, void **p, size_t need, size_t *bytes) {
    if ((*p = spare_take(device, need, bytes)) != nullptr) return hipSuccess;
    const hipError_t e = hipMalloc(p, need);
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    *bytes = need;
    return hipSuccess;
}

bool fail(const char **errorMessage, const std::string &msg) {
    State &s = S();
    std::strncpy(s.error, msg.c_str(), sizeof(s.error) - 1);
    s.error[sizeof(s.error) - 1] = '\0';
    if (errorMessage) *errorMessage = s.error;
    return false;
}

// fail() for the C ABI's exception handlers (no lock held there: the entry point's lock_guard is gone
// by the time its function-try-block's handler runs).  An exception (std::bad_alloc from a scene
// buffer sized by caller input, ...) becomes the reference's false + message
// (CudaPathTracerKernel.cu:181-184) instead of crossing extern "C" into std::terminate.
bool fail_free(const char **errorMessage, const char *what) {
    std::lock_guard<std::mutex> g(S().mu);
    return fail(errorMessage, std::string("HIP path tracer: ") + (what ? what : "exception"));
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return fail(err, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// ---- fp32 helpers with the oracle's contract (explicit fma only) ---------------------------
inline float fdot(const float *a, const float *b) { return std::fmaf(a[0], b[0], std::fmaf(a[1], b[1], a[2] * b[2])); }
inline void fcross(const float *a, const float *b, float *o) {
    o[0] = std::fmaf(a[1], b[2], -(a[2] * b[1]));
    o[1] = std::fmaf(a[2], b[0], -(a[0] * b[2]));
    o[2] = std::fmaf(a[0], b[1], -(a[1] * b[0]));
}
inline float as_float(int v) {
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}

// RayTracer.h Camera::Camera (:545-561), FP64, stored FP32.
void build_camera(const double lookfrom[3], const double lookat[3], const double vup[3], double vfov,
                  double aspect, double aperture, double focus, CameraF &out) {
    const double pi = 3.1415926535897932385;
    const double theta = vfov * pi / 180.0;
    const double h = std::tan(theta / 2);
    const double vh = 2.0 * h, vw = aspect * vh;
    auto unit = [](const double a[3], double o[3]) {
        const double len = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        const double inv = 1.0 / len;
        o[0] = inv * a[0];
        o[1] = inv * a[1];
        o[2] = inv * a[2];
    };
    auto cross = [](const double a[3], const double b[3], double o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    double wv[3] = {lookfrom[0] - lookat[0], lookfrom[1] - lookat[1], lookfrom[2] - lookat[2]};
    double w[3], u[3], v[3], c[3];
    unit(wv, w);
    cross(vup, w, c);
    unit(c, u);
    cross(w, u, v);
    for (int i = 0; i < 3; ++i) {
        const double hor = (focus * vw) * u[i];
        const double ver = (focus * vh) * v[i];
        const double llc = ((lookfrom[i] - 0.5 * hor) - 0.5 * ver) - focus * w[i];
        out.origin[i] = float(lookfrom[i]);
        out.llc[i] = float(llc);
        out.horizontal[i] = float(hor);
        out.vertical[i] = float(ver);
        out.u[i] = float(u[i]);
        out.v[i] = float(v[i]);
    }
    out.lens_radius = float(aperture / 2);
    out.reserved = 0.0f;
}

// The held batches of the open chain run (Ctx::chain.pendN) launched now as one group: before
// anything frees or replaces a buffer their parameters (Ctx::chain.pendP) point at — scene buffers,
// node layouts, item tables, the spill area (a held group launched after the free read
// freed memory).  The run stays open.
bool launch_held(Ctx &c, const char **err);

// Item tables no launch reads any more are freed; with `all`, after waiting for the stream.
void free_retired_tables(Ctx &c, bool all) {
    size_t k = 0;
    for (auto &t : c.retiredTables) {
        if (all || hipEventQuery(t.done) == hipSuccess) {
            if (all) (void)hipEventSynchronize(t.done);
            (void)hipFree(t.dev);
            (void)hipEventDestroy(t.done);
        } else {
            c.retiredTables[k++] = t;
        }
    }
    c.retiredTables.resize(k);
}

// A table the queued launches may still read: freed once the stream has passed this point.
void retire_table(Ctx &c, unsigned *dev) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(e, c.stream) != hipSuccess) {
        if (e) (void)hipEventDestroy(e);
        (void)hipStreamSynchronize(c.stream);
        (void)hipFree(dev);
        return;
    }
    c.retiredTables.push_back({dev, e});
}

// The context stops waiting for its cost job; the detached thread finishes on its own reference.
void abandon_cost_job(Ctx &c) { c.costJob.reset(); }

// Forgets the run costs and every item table (scene buffers freed, context destroyed).
void drop_order(Ctx &c) {
    abandon_cost_job(c);
    for (auto &t : c.orderTables) retire_table(c, t.dev);
    c.orderTables.clear();
    c.orderKey = OrderKey{};
    c.runCostsValid = false;
}

void free_scene_buffers(Ctx &c) {
    (void)hipFree(c.nodes);
    (void)hipFree(c.tris);
    (void)hipFree(c.shade);
    (void)hipFree(c.mats);
    (void)hipFree(c.nodes4);
    (void)hipFree(c.nodes4q);
    (void)hipFree(c.nodes4h);
    (void)hipFree(c.nodes4f);
    c.nodes = c.tris = c.shade = c.mats = c.nodes4 = c.nodes4q = c.nodes4h = c.nodes4f = nullptr;
    c.halfVersion = -1;
    c.hybridTop = -1;
    drop_order(c);
    c.sceneVersion = -1;
}

void harvest_audit(Ctx &c);

// keep: the big work buffers go to State::spare (a re-initialization) instead of hipFree.
void destroy_ctx(Ctx &c, bool keep) {
    (void)hipSetDevice(c.device);
    if (c.stream) (void)hipStreamSynchronize(c.stream);  // (so no queued launch reads a kept buffer)
    auto drop = [&](void *p, size_t bytes) {
        if (!p) return;
        if (keep && bytes) S().spare.push_back({c.device, p, bytes});
        else (void)hipFree(p);
    };
    harvest_audit(c);  // closed runs' records; an open run's (its image discarded) are dropped
    (void)hipFree(c.auditDev);
    (void)hipFree(c.accum);
    (void)hipFree(c.out);
    drop(c.scratch, c.scratchBytes);
    drop(c.scratchAlt, c.scratchAltBytes);
    c.scratchAlt = nullptr;
    c.scratchAltBytes = 0;
    c.hasDeferred = false;
    (void)hipFree(c.queue);
    (void)hipFree(c.chainCtl);
    drop(c.chainScratch, c.chainScratchBytes);
    if (c.chainBox) (void)hipHostFree(c.chainBox);
    if (c.chainStartEv) (void)hipEventDestroy(c.chainStartEv);
    if (c.chainEndEv) (void)hipEventDestroy(c.chainEndEv);
    (void)hipFree(c.stats);
    (void)hipFree(c.wfPool);
    (void)hipFree(c.wfCtr);
    drop(c.spill, c.spillBytes);
    c.spill = nullptr;
    c.spillBytes = 0;
    (void)hipHostFree(c.wfHost);
    for (hipEvent_t e : c.wfPoll)
        if (e) (void)hipEventDestroy(e);
    free_scene_buffers(c);
    free_retired_tables(c, true);
    for (auto &e : c.pool) {
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    for (hipEvent_t e : c.presentEv)
        if (e) (void)hipEventDestroy(e);
    if (c.stream) (void)hipStreamDestroy(c.stream);
    c = Ctx();
}

// keep: a re-initialization (init_inner) keeps the contexts' big work buffers for the new ones.
void destroy_all(bool keep = false) {
    State &s = S();
    if (!keep) spare_free_all();
    for (auto &c : s.ctxs) destroy_ctx(c, keep);
    s.ctxs.clear();
    for (auto &t : s.rngTables) {
        (void)hipSetDevice(t.first);
        (void)hipFree(t.second);
    }
    s.rngTables.clear();
    if (s.host) (void)hipHostFree(s.host);
    s.host = nullptr;
    s.hostCount = 0;
    for (int b = 0; b < 2; ++b) {
        if (s.present[b]) (void)hipHostFree(s.present[b]);
        s.present[b] = nullptr;
        s.presentPending[b] = false;
        s.presentSeq[b] = -1;
    }
    s.presentNext = 0;
    s.latest = -1;
    s.ready = false;
}

bool next_events(Ctx &c, EventPair &ev, const char **err) {
    if (c.freeEv.empty()) {
        EventPair e;
        HIP_TRY(hipEventCreate(&e.a));
        HIP_TRY(hipEventCreate(&e.b));
        c.pool.push_back(e);
        c.freeEv.push_back(e);
    }
    ev = c.freeEv.back();
    c.freeEv.pop_back();
    return true;
}

// Adds a finished launch's event time to the stats and recycles its events.
bool account(const std::pair<int, EventPair> &pe, Ctx &c, const char **err) {
    State &s = S();
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, pe.second.a, pe.second.b));
    if (pe.first == 0) {
        s.traceMs += ms;
        ++s.traceLaunches;
    } else {
        s.combineMs += ms;
        ++s.combineLaunches;
    }
    c.freeEv.push_back(pe.second);
    return true;
}

// Non-blocking: accounts the launches (in stream order) that have already finished.
bool harvest_locked(Ctx &c, const char **err) {
    size_t done = 0;
    while (done < c.pending.size() && hipEventQuery(c.pending[done].second.b) == hipSuccess) {
        if (!account(c.pending[done], c, err)) return false;
        ++done;
    }
    c.pending.erase(c.pending.begin(), c.pending.begin() + long(done));
    return true;
}

bool ensure_scene(Ctx &c, const char **err) {
    State &s = S();
    if (s.scene.kind != HIPPT_SCENE_MESH || c.sceneVersion == s.scene.version) return true;
    if (!launch_held(c, err)) return false;
    HIP_TRY(hipSetDevice(c.device));
    HIP_TRY(hipStreamSynchronize(c.stream));  // queued launches read the old buffers
    free_scene_buffers(c);
    auto up = [&](float4 *&dst, const std::vector<float4> &src) -> bool {
        HIP_TRY(hipMalloc(&dst, std::max<size_t>(16, src.size() * sizeof(float4))));
        if (!src.empty()) HIP_TRY(hipMemcpy(dst, src.data(), src.size() * sizeof(float4), hipMemcpyHostToDevice));
        return true;
    };
    if (!up(c.nodes, s.scene.nodes) || !up(c.tris, s.scene.tris) || !up(c.shade, s.scene.shade) ||
        !up(c.mats, s.scene.mats) || !up(c.nodes4, s.scene.nodes4) || !up(c.nodes4q, s.scene.nodes4q))
        return false;
    c.sceneVersion = s.scene.version;
    return true;
}

// Low bits of a packed child key (trace::child_key_p) that give an LDS-resident 4-wide tree's child
// codes back when sign-extended: interior codes are node byte offsets < numNodes*128, leaf codes
// ~(first<<4 | count) with first + count <= numPrims; one more bit for the sign.  At most 16 for a
// scene that fits the LDS copy (24 KB: < 192 nodes, < 384 primitives), which leaves the entry
// distance 7 or more mantissa bits (Cornell-34: 12 bits, 11 mantissa bits) to order children by.
unsigned packed_ref_bits(int numNodes, int numPrims) {
    const unsigned long long maxMag =
        std::max<unsigned long long>((unsigned long long)std::max(numNodes, 1) * 128ull,
                                     ((unsigned long long)numPrims << 4) + 16ull);
    unsigned bits = 1;
    while ((1ull << (bits - 1)) < maxMag) ++bits;  // magnitude < 2^(bits-1)
    return std::max(bits, 8u);
}

// The queues' item table of a context's rows (item_order.h) for a batch of `frames` frames: run cost
// estimates per key (scene, camera, image, rows, depth), tables per batch size (kOrderTables of
// them, so a call's full batches and its remainder batch both stay cached).  With `forced`
// (HIPPT_OPT_ITEM_ORDER 1) new costs are computed here, on all host threads.  In automatic mode they
// are computed on a host thread of their own, and the batches queued meanwhile run in image order
// (*table = nullptr: the same results), so moving the camera never stalls a frame on
// the estimate (0.34 s single-threaded at 1080p).  A replaced table is freed once the launches
// that read it are done (an event, not a stream synchronisation).
constexpr size_t kOrderTables = 4;

int cost_threads() { return int(std::max(1u, std::min(16u, std::thread::hardware_concurrency()))); }

bool ensure_order(Ctx &c, const CameraF &cam, int frames, int maxDepth, bool forced, unsigned tileShift,
                  const unsigned **table, const char **err) {
    State &s = S();
    *table = nullptr;
    OrderKey key;
    key.tileShift = hippt::tile_shift_for(unsigned(s.width), tileShift);
    key.version = s.scene.version;
    key.width = s.width;
    key.height = s.height;
    key.y0 = c.y0;
    key.rows = c.rows;
    key.stride = c.stride;
    key.maxDepth = maxDepth;
    key.cam = cam;
    HIP_TRY(hipSetDevice(c.device));
    free_retired_tables(c, false);
    if (!c.runCostsValid || !same_key(key, c.orderKey)) {
        std::vector<float> cost;
        const bool jobForKey = c.costJob && same_key(c.costJob->key, key);
        if (jobForKey && (forced || c.costJob->finished())) {
            // forced mode takes the in-flight job's estimate for this key rather than computing it
            // again
            c.costJob->wait();
            cost = std::move(c.costJob->cost);
            c.costJob.reset();
        } else if (forced) {
            abandon_cost_job(c);  // a stale key's job: not joined on the render path
            hippt::run_costs(s.scene.bvh4, reinterpret_cast<const float *>(s.scene.tris.data()), cam,
                             hippt::RunLayout{unsigned(s.width), unsigned(c.rows), key.tileShift}, s.height, c.y0,
                             c.stride, maxDepth, cost, cost_threads());
        } else {
            if (c.costJob && !jobForKey) abandon_cost_job(c);
            if (!c.costJob) {
                auto job = std::make_shared<CostJob>();
                job->key = key;
                job->bvh = s.scene.bvh4;
                job->tris = s.scene.tris;
                const int nt = std::max(1, cost_threads() / 2);
                try {
                    std::thread([job, nt] {
                        // an exception must not leave the thread (std::terminate): no estimate then,
                        // and this key's batches stay in image order
                        try {
                            hippt::run_costs(job->bvh, reinterpret_cast<const float *>(job->tris.data()),
                                             job->key.cam,
                                             hippt::RunLayout{unsigned(job->key.width), unsigned(job->key.rows),
                                                              job->key.tileShift},
                                             job->key.height, job->key.y0, job->key.stride, job->key.maxDepth,
                                             job->cost, nt);
                        } catch (...) {
                            job->cost.clear();
                        }
                        {
                            std::lock_guard<std::mutex> g(job->mu);
                            job->done = true;
                        }
                        job->cv.notify_all();
                    }).detach();
                    c.costJob = std::move(job);
                } catch (const std::system_error &) {
                    // no thread to be had: this batch in image order, the next one tries again
                }
            }
            return true;  // this batch in image order
        }
        if (!launch_held(c, err)) return false;
        for (auto &t : c.orderTables) retire_table(c, t.dev);
        c.orderTables.clear();
        c.runCosts = std::move(cost);
        c.orderKey = key;
        c.runCostsValid = true;
    }
    if (c.runCosts.empty()) return true;  // no estimate for this key (its job failed): image order
    for (size_t k = 0; k < c.orderTables.size(); ++k)
        if (c.orderTables[k].frames == frames) {
            std::rotate(c.orderTables.begin(), c.orderTables.begin() + k, c.orderTables.begin() + k + 1);
            *table = c.orderTables.front().dev;
            return true;
        }
    std::vector<uint32_t> order;
    hippt::build_item_table(c.runCosts, hippt::RunLayout{unsigned(s.width), unsigned(c.rows), c.orderKey.tileShift},
                            unsigned(frames), hippt::kMeshQueues, order);
    unsigned *dev = nullptr;
    HIP_TRY(hipMalloc(&dev, std::max<size_t>(1, order.size()) * sizeof(unsigned)));
    // a fresh buffer: the copy need not wait for the launches queued on the context's stream
    if (!order.empty() && hipMemcpy(dev, order.data(), order.size() * sizeof(unsigned), hipMemcpyHostToDevice) !=
                              hipSuccess) {
        (void)hipFree(dev);
        return fail(err, "HIP path tracer: item table upload failed");
    }
    if (c.orderTables.size() >= kOrderTables) {
        if (!launch_held(c, err)) return false;
        retire_table(c, c.orderTables.back().dev);
        c.orderTables.pop_back();
    }
    c.orderTables.insert(c.orderTables.begin(), Ctx::OrderTable{frames, dev});
    *table = dev;
    return true;
}

// The half-precision node layout (bvh_builder.h half_bvh4, HIPPT_OPT_BVH_QUANT 3): built on the host
// once per scene (half_tree_ok) and uploaded to a context's device the first time a render there
// uses it.
bool half_tree_ok(SceneHost &sc) {
    if (sc.halfState == 0) {
        std::vector<uint32_t> h;
        if (hippt::half_bvh4(reinterpret_cast<const uint32_t *>(sc.nodes4.data()), size_t(sc.numNodes4), h)) {
            sc.nodes4f.assign(h.size() / 4, float4{});
            std::memcpy(sc.nodes4f.data(), h.data(), h.size() * sizeof(uint32_t));
            sc.halfState = 1;
        } else {
            sc.halfState = -1;  // planes beyond the half range: float nodes
        }
    }
    return sc.halfState > 0;
}

bool ensure_half(Ctx &c, const char **err) {
    SceneHost &sc = S().scene;
    if (!half_tree_ok(sc)) return fail(err, "HIP path tracer: no half-precision tree for this scene");
    if (c.halfVersion == sc.version && c.nodes4f) return true;
    if (!launch_held(c, err)) return false;
    HIP_TRY(hipSetDevice(c.device));
    HIP_TRY(hipStreamSynchronize(c.stream));
    (void)hipFree(c.nodes4f);
    c.nodes4f = nullptr;
    HIP_TRY(hipMalloc(&c.nodes4f, sc.nodes4f.size() * sizeof(float4)));
    HIP_TRY(hipMemcpy(c.nodes4f, sc.nodes4f.data(), sc.nodes4f.size() * sizeof(float4), hipMemcpyHostToDevice));
    c.halfVersion = sc.version;
    return true;
}

// The hybrid node layout (bvh_builder.h hybrid_bvh4) for `top` top-of-tree nodes: built on the
// host once per (scene, top) and uploaded to the context's device.
bool ensure_hybrid(Ctx &c, int top, const char **err) {
    State &s = S();
    SceneHost &sc = s.scene;
    if (sc.hybridTop != top) {
        std::vector<uint32_t> w;
        if (!hippt::hybrid_bvh4(sc.bvh4, sc.q4, top, w)) return fail(err, "hybrid BVH layout failed");
        sc.hybrid.assign(w.size() / 4, float4{});
        std::memcpy(sc.hybrid.data(), w.data(), w.size() * sizeof(uint32_t));
        sc.hybridTop = top;
    }
    if (c.hybridTop == top && c.nodes4h) return true;
    if (!launch_held(c, err)) return false;
    HIP_TRY(hipSetDevice(c.device));
    HIP_TRY(hipStreamSynchronize(c.stream));
    (void)hipFree(c.nodes4h);
    c.nodes4h = nullptr;
    c.hybridTop = -1;
    HIP_TRY(hipMalloc(&c.nodes4h, sc.hybrid.size() * sizeof(float4)));
    HIP_TRY(hipMemcpy(c.nodes4h, sc.hybrid.data(), sc.hybrid.size() * sizeof(float4), hipMemcpyHostToDevice));
    c.hybridTop = top;
    return true;
}

bool init_inner(int width, int height, const char **err) {
    State &s = S();
    spare_free_all();   // the previous initialization's, none of which its contexts took again
    destroy_all(true);  // this one's, for the new contexts
    if (width <= 0 || height <= 0) return fail(err, "invalid image size");
    s.width = width;
    s.height = height;
    std::vector<int> devs = s.devices;
    if (devs.empty()) {
        int d = 0;
        HIP_TRY(hipGetDevice(&d));
        devs.push_back(d);
    }
    // this process's rows: first p0, count pn, stride ps
    int p0, pn, ps;
    if (s.rowStride > 1) {
        p0 = std::min(s.rowPhase, height);
        ps = s.rowStride;
        pn = p0 < height ? (height - p0 + ps - 1) / ps : 0;
    } else {
        p0 = std::clamp(s.rowY0, 0, height);
        pn = (s.rowY1 <= 0 ? height : std::clamp(s.rowY1, p0, height)) - p0;
        ps = 1;
    }
    const int n = int(devs.size());
    s.ctxs.resize(size_t(n));
    for (int k = 0; k < n; ++k) {
        Ctx &c = s.ctxs[size_t(k)];
        c.device = devs[size_t(k)];
        if (s.deviceInterleave && n > 1) {  // device k: every n-th of the process's rows
            c.y0 = p0 + ps * k;
            c.rows = pn > k ? (pn - k + n - 1) / n : 0;
            c.stride = ps * n;
        } else {  // device k: a contiguous run of the process's rows
            const int a = int((long long)pn * k / n), b = int((long long)pn * (k + 1) / n);
            c.y0 = p0 + ps * a;
            c.rows = b - a;
            c.stride = ps;
        }
        HIP_TRY(hipSetDevice(c.device));
        HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        const size_t px = size_t(c.rows) * size_t(width);
        HIP_TRY(hipMalloc(&c.accum, std::max<size_t>(16, px * sizeof(float4))));
        HIP_TRY(hipMalloc(&c.out, std::max<size_t>(16, px * sizeof(uint32_t))));
        HIP_TRY(hipMalloc(&c.queue, kQueueBytes));
        HIP_TRY(hipMalloc(&c.stats, kStatBytes));
        HIP_TRY(hipMemsetAsync(c.accum, 0, px * sizeof(float4), c.stream));
        HIP_TRY(hipMemsetAsync(c.out, 0, px * sizeof(uint32_t), c.stream));
        HIP_TRY(hipMemsetAsync(c.stats, 0, kStatBytes, c.stream));
        HIP_TRY(hipDeviceGetAttribute(&c.cus, hipDeviceAttributeMultiprocessorCount, c.device));
        HIP_TRY(hipStreamSynchronize(c.stream));
    }
    s.hostCount = size_t(width) * size_t(height);
    // portable, mapped, coherent (fine-grained: the GPU writes go straight to host memory): every
    // context's device may write it (legacy zero-copy frames)
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.host), s.hostCount * sizeof(unsigned),
                          hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(s.host, 0, s.hostCount * sizeof(unsigned));
    s.ready = true;
    return true;
}

// Cleans up on failure, as cudaPathTracerInit does (CudaPathTracerKernel.cu:202-234).
bool init_locked(int width, int height, const char **err) {
    if (init_inner(width, height, err)) return true;
    destroy_all();
    return false;
}

long long occupancy_key(int version, int stackDepth, bool lds, bool full, bool wide = false, bool quant = false,
                        bool spills = true) {
    return ((long long)version << 11) | ((long long)stackDepth << 5) | (spills ? 16 : 0) | (quant ? 8 : 0) |
           (wide ? 4 : 0) | (lds ? 2 : 0) | (full ? 1 : 0);
}

// 4-wide traversal of a tree whose stack bound exceeds the LDS capacity: a per-lane spill
// area of spillCap entries for every lane of a `blocks`-block persistent grid.
bool ensure_spill(Ctx &c, hippt::MeshParams &p, long long blocks, bool spills, int spillCap, const char **err) {
    if (!spills) return true;
    p.spillCap = spillCap;
    const size_t bytes = size_t(blocks) * hippt::kMeshBlock * size_t(spillCap) * sizeof(int);
    if (c.spillBytes < bytes) {
        if (!launch_held(c, err)) return false;
        HIP_TRY(hipStreamSynchronize(c.stream));
        (void)hipFree(c.spill);
        c.spill = nullptr;
        c.spillBytes = 0;
        void *p = nullptr;
        HIP_TRY(work_malloc(c.device, &p, bytes, &c.spillBytes));
        c.spill = static_cast<int *>(p);
    }
    p.spill = c.spill;
    return true;
}

// The memoized random_in_unit_sphere table of c's device (hippt_device.h launch_rng_table),
// built once per device on first use (16 GiB, a few ms) and shared by the device's contexts.
bool rng_table(Ctx &c, const uint32_t **out, const char **err) {
    State &s = S();
    for (auto &t : s.rngTables)
        if (t.first == c.device) {
            *out = t.second;
            return true;
        }
    uint32_t *t = nullptr;
    HIP_TRY(hipMalloc(&t, hippt::kRngTableBytes));
    const hipError_t e = hippt::launch_rng_table(t, c.stream);
    if (e != hipSuccess || hipStreamSynchronize(c.stream) != hipSuccess) {
        (void)hipFree(t);
        return fail(err, std::string("rng table: ") + hipGetErrorString(e));
    }
    s.rngTables.emplace_back(c.device, t);
    *out = t;
    return true;
}

// Wavefront variant (hippt_wavefront.hip): init + generate, then extend/shade/generate
// iterations until the ray queue stays empty.  The host reads the queue size with one batch of
// lag (pinned snapshot + event), so the call returns within ~16 iterations of the end.
bool run_wavefront(Ctx &c, hippt::MeshParams p, bool cnt, bool spills, int spillCap, const char **err) {
    State &s = S();
    unsigned slots = std::max(64u, std::min(s.wfSlots, std::max(64u, p.totalItems)));
    unsigned shardCap = 0;
    if (c.wfWant != slots || !c.wfPool) {
        HIP_TRY(hipStreamSynchronize(c.stream));
        (void)hipFree(c.wfPool);
        c.wfPool = nullptr;
        c.wfSlots = c.wfWant = 0;
        const unsigned want = slots;
        // Every context owns a pool, and several contexts may share a device (hipptSetDevices
        // with a repeated id): each takes at most half the device's free memory divided by the
        // contexts on it, and a failed allocation retries with half the slots.  A smaller pool
        // only adds regenerate rounds; the image is the same.
        size_t freeB = 0, totalB = 0;
        HIP_TRY(hipMemGetInfo(&freeB, &totalB));
        int sharing = 0;
        for (const Ctx &o : s.ctxs) sharing += o.device == c.device && !o.wfPool ? 1 : 0;
        const size_t budget = freeB / 2 / size_t(std::max(1, sharing));
        while (slots > 64u && hippt::wf_pool_words(slots, &shardCap) * sizeof(uint32_t) > budget) slots >>= 1;
        for (;;) {
            const hipError_t e = hipMalloc(&c.wfPool, hippt::wf_pool_words(slots, &shardCap) * sizeof(uint32_t));
            if (e == hipSuccess) break;
            (void)hipGetLastError();  // clear the sticky allocation error
            c.wfPool = nullptr;
            if (slots <= (1u << 16)) return fail(err, std::string("wavefront pool: ") + hipGetErrorString(e));
            slots >>= 1;
        }
        c.wfSlots = slots;
        c.wfWant = want;
    }
    slots = c.wfSlots;
    (void)hippt::wf_pool_words(slots, &shardCap);
    if (!c.wfCtr) HIP_TRY(hipMalloc(&c.wfCtr, hippt::kCtrWords * sizeof(unsigned)));
    hippt::WfParams W{};
    W.mp = p;
    W.slots = slots;
    W.shardCap = shardCap;
    W.ctr = c.wfCtr;
    // the two ray queues' payload arrays (float4 each), then the hit array
    auto *base = static_cast<float4 *>(c.wfPool);
    const size_t entries = size_t(hippt::kWfShards) * shardCap;
    for (int q = 0; q < 2; ++q) {
        W.ra[q] = base + (3 * q + 0) * entries;
        W.rb[q] = base + (3 * q + 1) * entries;
        W.rc[q] = base + (3 * q + 2) * entries;
    }
    W.hit = reinterpret_cast<float2 *>(base + 6 * entries);
    // coherence sort of the scattered paths (HIPPT_OPT_WAVEFRONT_SORT; automatic: off)
    W.sortBits = unsigned(s.wfSort > 0 ? s.wfSort : 0);
    if (W.sortBits > 3) {
        // the scene box: the union of the 4-wide root's child boxes (Bvh4 words lo.x[4] hi.x[4] ...)
        const std::vector<uint32_t> &n = s.scene.bvh4.nodes;
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int i = 0; i < 4 && n.size() >= size_t(hippt::kNode4Words); ++i) {
                float l, h;
                std::memcpy(&l, &n[size_t(8 * a + i)], 4);
                std::memcpy(&h, &n[size_t(8 * a + 4 + i)], 4);
                if (l <= h) {
                    lo = std::min(lo, l);
                    hi = std::max(hi, h);
                }
            }
            const bool ok = std::isfinite(lo) && std::isfinite(hi) && hi > lo;
            W.sortLo[a] = ok ? lo : 0.0f;
            W.sortScale[a] = ok ? 2.0f / (hi - lo) : 0.0f;
        }
    }
    const bool wide = p.wide != 0, quant = p.wide == 2;
    const long long occKey = occupancy_key(s.scene.version, p.stackDepth, p.ldsScene != 0, p.full != 0, wide, quant) ^
                             ((long long)p.topBytes << 40) ^ ((long long)(p.wide == hippt::kWideHalf) << 34);
    if (c.wfOccKey != occKey) {
        const int ln = p.ldsScene ? p.numNodes : 0, lt = p.ldsScene ? p.numTris : 0;
        c.wfBlocksPerCu[0] =
            hippt::wf_extend_blocks_per_cu(false, p.full != 0, wide, quant, p.stackDepth, ln, lt, p.topBytes);
        c.wfBlocksPerCu[1] =
            hippt::wf_extend_blocks_per_cu(true, p.full != 0, wide, quant, p.stackDepth, ln, lt, p.topBytes);
        c.wfOccKey = occKey;
    }
    s.activeBlocksPerCu = c.wfBlocksPerCu[cnt ? 1 : 0];
    const int bpc = s.blocksPerCu > 0 ? s.blocksPerCu : c.wfBlocksPerCu[cnt ? 1 : 0];
    const int blocks = int(std::max(1LL, std::min<long long>((long long)c.cus * bpc, (slots + 255) / 256)));
    if (!ensure_spill(c, p, blocks, spills, spillCap, err)) return false;
    W.mp = p;
    EventPair ev;
    if (!next_events(c, ev, err)) return false;
    HIP_TRY(hipEventRecord(ev.a, c.stream));
    HIP_TRY(hippt::wf_launch_init(W, c.stream));
    HIP_TRY(hippt::wf_launch_generate(W, 0, c.stream));
    // every path needs <= maxDepth extend rounds; slots regenerate as paths end
    const long long maxIter = (long long)p.maxDepth * ((p.totalItems + slots - 1) / slots + 1) + 64;
    // Every kPollEvery iterations the ray-queue sizes (appended + generated entries) are copied to
    // pinned memory; the host reads the snapshot one batch later, so the stream always holds a
    // batch of queued work.  Iterations after the queue drained are no-ops (empty queues).
    constexpr int kPollEvery = 8, kSnap = 2 * hippt::kWfShards * hippt::kCtrStride;
    if (!c.wfHost) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c.wfHost), 2 * kSnap * sizeof(unsigned)));
    for (hipEvent_t &e : c.wfPoll)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int cur = 0;
    // A pool that holds every work item of the batch generates them all up front and never
    // regenerates, and every path ends within maxDepth extend rounds: at most maxDepth iterations
    // (a polled loop alone runs up to 2*kPollEvery - 1 empty iterations past the end; the poll
    // still ends a deep maxDepth early once every path has ended).
    const bool allInFlight = slots >= p.totalItems;
    for (long long it = 0;; ++it) {
        if (allInFlight && it == p.maxDepth) break;
        if (it > maxIter) return fail(err, "wavefront path tracer did not drain its ray queue");
        HIP_TRY(hippt::wf_launch_extend(W, cur, blocks, cnt, c.stream));
        HIP_TRY(hippt::wf_launch_shade(W, cur, c.stream));
        if (!allInFlight) HIP_TRY(hippt::wf_launch_generate(W, cur ^ 1, c.stream));
        cur ^= 1;
        if (it % kPollEvery != kPollEvery - 1) continue;
        const int b = int(it / kPollEvery) & 1;
        HIP_TRY(hipMemcpyAsync(c.wfHost + b * kSnap, c.wfCtr + hippt::ctr_word(hippt::ctr_queue(cur)),
                               kSnap * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
        HIP_TRY(hipEventRecord(c.wfPoll[b], c.stream));
        if (it < 2 * kPollEvery - 1) continue;
        HIP_TRY(hipEventSynchronize(c.wfPoll[b ^ 1]));
        unsigned left = 0;
        for (int k = 0; k < 2 * hippt::kWfShards; ++k) left += c.wfHost[(b ^ 1) * kSnap + k * hippt::kCtrStride];
        if (left == 0) break;
    }
    HIP_TRY(hipEventRecord(ev.b, c.stream));
    c.pending.push_back({0, ev});
    return true;
}

CameraF current_camera() {
    State &s = S();
    if (s.scene.rawCamera) return s.scene.cam;
    CameraF cam;
    build_camera(s.scene.lookfrom, s.scene.lookat, s.scene.vup, s.scene.vfov, double(s.width) / double(s.height),
                 s.scene.aperture, s.scene.focus, cam);
    return cam;
}

// Enqueues `count` frames on every context (no host wait).
// Copies a context's compact rows (c.rows rows of W pixels of `bytes` each) to their image rows
// c.y0, c.y0 + c.stride, ... of a full-frame host buffer, on the context's stream.
bool copy_rows_async(Ctx &c, void *dstFrame, const void *src, size_t bytes, const char **err) {
    State &s = S();
    if (c.rows <= 0) return true;
    const size_t row = size_t(s.width) * bytes;
    char *dst = static_cast<char *>(dstFrame) + size_t(c.y0) * row;
    HIP_TRY(hipMemcpy2DAsync(dst, row * size_t(c.stride), src, row, row, size_t(c.rows), hipMemcpyDeviceToHost, c.stream));
    return true;
}

// The open chain run's last combines (Ctx::chain): every batch no launch combined, in order; the run
// ends (the next chained batch starts a new one).
bool launch_chained(Ctx &c, hippt::MeshParams &p, const char **err);

bool flush_chain(Ctx &c, const char **err) {
    Ctx::Chain &ch = c.chain;
    if (!ch.live) return true;
    HIP_TRY(hipSetDevice(c.device));
    if (!launch_held(c, err)) return false;  // the held batches' group launch, before the run closes
    ch.live = false;
    hippt::ChainFlushParams f{};
    f.comb = ch.key.comb;
    f.scratch = c.chainScratch;
    f.ctl = c.chainCtl;
    f.epoch = ch.epoch;  // the run's launches were epochs 0 .. epoch - 1
    f.lastSeq = ch.seq - 1u;
    f.slots = ch.slots;
    f.shift = ch.shift;
    f.step = std::max(ch.step, 0);
    f.audit = ch.audit;
    if (ch.audit && !c.auditRuns.empty()) {  // the run's header: what it asked for
        Ctx::AuditRun &a = c.auditRuns.back();
        a.hdr[4] = unsigned(ch.step);
        a.hdr[8] = ch.seq;
        a.hdr[9] = ch.epoch;
        a.hdr[11] = ch.seq > hippt::kAuditBatches ? ch.seq - hippt::kAuditBatches : 0u;
        a.closed = true;
    }
    EventPair ev;
    if (!next_events(c, ev, err)) return false;
    HIP_TRY(hipEventRecord(ev.a, c.stream));
    HIP_TRY(hippt::launch_chain_flush(f, c.stream));
    HIP_TRY(hipEventRecord(ev.b, c.stream));
    c.pending.push_back({1, ev});
    return true;
}

// The deferred combine of a context as a launch of its own (see Ctx::deferred), or the open chain
// run's flush.
bool flush_deferred(Ctx &c, const char **err) {
    if (!flush_chain(c, err)) return false;
    if (!c.hasDeferred) return true;
    c.hasDeferred = false;
    HIP_TRY(hipSetDevice(c.device));
    EventPair ev;
    if (!next_events(c, ev, err)) return false;
    HIP_TRY(hipEventRecord(ev.a, c.stream));
    HIP_TRY(hippt::launch_combine(c.deferred, c.stream, c.deferredHost));
    HIP_TRY(hipEventRecord(ev.b, c.stream));
    c.pending.push_back({1, ev});
    c.deferredHost = hippt::HostFrame{};
    return true;
}

// A per-sample radiance buffer of at least `need` bytes that the deferred combine does not read.
bool batch_scratch(Ctx &c, size_t need, float **out, const char **err) {
    const bool alt = c.hasDeferred && c.deferred.scratch == c.scratch;
    float *&buf = alt ? c.scratchAlt : c.scratch;
    size_t &bytes = alt ? c.scratchAltBytes : c.scratchBytes;
    if (bytes < need) {
        HIP_TRY(hipStreamSynchronize(c.stream));
        (void)hipFree(buf);
        buf = nullptr;
        bytes = 0;
        void *p = nullptr;
        HIP_TRY(work_malloc(c.device, &p, need, &bytes));
        buf = static_cast<float *>(p);
    }
    *out = buf;
    return true;
}

// Chained batches (Ctx::chain).  Automatic (HIPPT_OPT_CHAIN -1): every batch (whose items fit the ring's
// slot bits) is chained; a launch traces up to cap batches (chain_cap) and the ring holds twice that, so
// that a launch traces one group of batches while it combines the previous one.  Measured (r5s/r5x, 20
// steps, cap by chain_cap): 1/8 shares Cornell 1.112 -> 1.047 ms, blob70k 3.003 -> 2.518, cornell_mixed
// 1.831 -> 1.573; 1/2 shares blob70k 9.79 -> 9.49, cornell_mixed 6.20 -> 5.92, Cornell 3.757 -> 3.765;
// whole images blob70k 18.94 -> 18.69, cornell_mixed 12.06 -> 11.70, but Cornell 7.255 -> 7.321, so
// round 5 ran a whole image of an LDS-resident Lambertian scene one launch per batch.  Round 6 (r6aw/r6ax,
// alternating passes, with the held groups and the clock warm-up): a whole Cornell image chained at cap 8
// 55,875 -> 56,111 M/s, so it is chained too.
// chain_batch's held groups (an A/B build knob)
#ifndef HIPPT_CHAIN_GROUPS
#define HIPPT_CHAIN_GROUPS 1
#endif
constexpr bool kChainGroups = HIPPT_CHAIN_GROUPS != 0;
// chain_batch holds the batches that arrive while the run's first launch runs (an A/B build knob)
#ifndef HIPPT_CHAIN_HOLD_RUNNING
#define HIPPT_CHAIN_HOLD_RUNNING 1
#endif
constexpr bool kChainHoldRunning = HIPPT_CHAIN_HOLD_RUNNING != 0;

// The automatic cap's ceiling: 16 for trees in global memory, 8 for LDS-resident scenes.  A bigger
// cap makes a burst's groups bigger (a 1/8 row share's 20 steps: 3 launches instead of 4), and the
// launch after a group combines the whole group: hidden behind a global tree's slower batches
// (blob70k 1/8 share 2.538/2.539 -> 2.497/2.493 ms, 1/4 share 4.799/4.778 -> 4.754/4.754), exposed
// beside Cornell's (1/8 share 0.991/0.989 -> 1.025/1.015: the last launch's 16-batch combine adds
// ~0.9 ms), r6n.
// Batches of more than 2^26 samples (whole 1080p/64 spp images) take cap 8 (r6aw/r6ax: blob70k 22,302 ->
// 22,391 M/s against cap 3, cornell_mixed 35,314 -> 35,422, Cornell chained at 8 as above; cap 2 and 6
// lower or equal); the ring (16 slots) stays within the scratch budget (ring_plan) or the cap shrinks.
unsigned chain_cap(long long option, unsigned total, bool ldsScene) {
    if (option > 0) return unsigned(std::min<long long>(option, 16));
    const double c = total > (1u << 26) ? 8.0 : std::round(4e8 / double(std::max(1u, total)));
    return unsigned(std::clamp(c, 2.0, ldsScene ? 8.0 : 16.0));
}

// The ring of a run of `total`-item batches: 2^shift samples per slot (the slot bits above them in
// an item), at least 2 x cap slots (a launch traces up to cap batches while up to cap batches before
// its own wait for its combine), 12 bytes per sample.  The ring stays within the sample-scratch
// budget (HIPPT_OPT_SCRATCH_MB): the cap shrinks until it fits, and a batch whose smallest ring
// (2 slots) does not fit runs unchained (bytes = 0).  (blob70k at 1080p/64 spp and cap 8
// asked for 25.8 GB whatever the budget.)
struct RingPlan {
    unsigned cap = 0, slots = 0, shift = 0;
    size_t bytes = 0;
};
RingPlan ring_plan(unsigned total, long long option, bool ldsScene, size_t budget) {
    RingPlan r;
    r.shift = 6;
    while ((1u << r.shift) < total) ++r.shift;
    const size_t slotBytes = (size_t(1) << r.shift) * 3 * sizeof(float);
    for (unsigned cap = chain_cap(option, total, ldsScene); cap >= 1; --cap) {
        unsigned slots = 2;
        while (slots < 2 * cap) slots <<= 1;
        slots = std::min(slots, hippt::kChainSlotsMax);
        if (size_t(slots) * slotBytes <= budget) {
            r.cap = cap;
            r.slots = slots;
            r.bytes = size_t(slots) * slotBytes;
            return r;
        }
    }
    return r;
}

// The ring's buffers for plan `r` (allocated, or grown after the open run's last combines); *ok =
// false when the device has no memory for them (the batch then runs unchained).
bool ensure_ring(Ctx &c, const RingPlan &r, bool *ok, const char **err) {
    *ok = true;
    if (!c.chainCtl) HIP_TRY(hipMalloc(&c.chainCtl, hippt::kChainCtlWords * sizeof(unsigned)));
    if (!c.chainBox) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c.chainBox), sizeof(unsigned long long),
                              hipHostMallocMapped | hipHostMallocCoherent));
        *c.chainBox = 0;
        void *d = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&d, c.chainBox, 0));
        c.chainBoxDev = static_cast<unsigned long long *>(d);
    }
    if (c.chainScratchBytes >= r.bytes) return true;
    if (!flush_deferred(c, err)) return false;  // the open run's last combines read the old ring
    HIP_TRY(hipStreamSynchronize(c.stream));
    (void)hipFree(c.chainScratch);
    c.chainScratch = nullptr;
    c.chainScratchBytes = 0;
    void *p = nullptr;
    size_t got = 0;
    if (work_malloc(c.device, &p, r.bytes, &got) != hipSuccess) {
        (void)hipGetLastError();
        c.chainScratch = nullptr;
        *ok = false;
        return true;
    }
    c.chainScratch = static_cast<float *>(p);
    c.chainScratchBytes = got;
    return true;
}

bool same_cam(const CameraF &a, const CameraF &b) {
    if (a.lens_radius != b.lens_radius) return false;
    for (int k = 0; k < 3; ++k)
        if (a.origin[k] != b.origin[k] || a.llc[k] != b.llc[k] || a.horizontal[k] != b.horizontal[k] ||
            a.vertical[k] != b.vertical[k] || a.u[k] != b.u[k] || a.v[k] != b.v[k])
            return false;
    return true;
}

// Two batches' launch parameters agree on everything the run's launches take from their own
// parameters for every batch of the run (all but the frames, scratch, counters and chain fields).
bool chain_same(const hippt::MeshParams &a, const hippt::MeshParams &b) {
    return a.nodes == b.nodes && a.tris == b.tris && a.shade == b.shade && a.mats == b.mats && a.stats == b.stats &&
           same_cam(a.cam, b.cam) && a.invW == b.invW && a.invH == b.invH && a.width == b.width &&
           a.height == b.height && a.y0 == b.y0 && a.bandRows == b.bandRows && a.rowStride == b.rowStride &&
           a.frames == b.frames && a.maxDepth == b.maxDepth && a.bandPixels == b.bandPixels &&
           a.totalItems == b.totalItems && a.stackDepth == b.stackDepth && a.numNodes == b.numNodes &&
           a.numTris == b.numTris && a.numMats == b.numMats && a.ldsScene == b.ldsScene && a.full == b.full &&
           a.waveThreshold == b.waveThreshold && a.chunk == b.chunk && a.leafExit == b.leafExit &&
           a.nodeExit == b.nodeExit && a.wide == b.wide && a.stackCap == b.stackCap && a.spillCap == b.spillCap &&
           a.spill == b.spill && a.topBytes == b.topBytes && a.refBits == b.refBits && a.runOrder == b.runOrder &&
           a.runCount == b.runCount && a.runTileShift == b.runTileShift && a.rngTable == b.rngTable && a.poolOffset == b.poolOffset &&
           a.poolWords == b.poolWords && a.comb.format == b.comb.format;
}

// Enqueues the launch of chained batch p (its chain fields set by chain_batch but the epoch): the run's
// next launch number, and the start event chain_batch's skip test queries.
bool launch_chained(Ctx &c, hippt::MeshParams &p, const char **err) {
    Ctx::Chain &ch = c.chain;
    p.chainEpoch = ch.epoch++;
    ch.lastOwn = p.chainSeq;
    ch.pendN = 0;
    if (!c.chainStartEv) HIP_TRY(hipEventCreateWithFlags(&c.chainStartEv, hipEventDisableTiming));
    if (!c.chainEndEv) HIP_TRY(hipEventCreateWithFlags(&c.chainEndEv, hipEventDisableTiming));
    EventPair ev;
    if (!next_events(c, ev, err)) return false;
    HIP_TRY(hipEventRecord(c.chainStartEv, c.stream));
    HIP_TRY(hipEventRecord(ev.a, c.stream));
    HIP_TRY(hippt::launch_mesh(p, int(ch.blocks), false, c.stream));
    HIP_TRY(hipEventRecord(ev.b, c.stream));
    HIP_TRY(hipEventRecord(c.chainEndEv, c.stream));
    c.pending.push_back({0, ev});
    return true;
}

bool launch_held(Ctx &c, const char **err) {
    Ctx::Chain &ch = c.chain;
    if (!ch.live || !ch.pendN) return true;
    HIP_TRY(hipSetDevice(c.device));
    ch.pendP.chainGroup = ch.pendN;
    ch.pendP.chainPosted = ch.seq - 1u;
#ifdef HIPPT_CHAIN_TRACE
    std::fprintf(stderr, "chain run %u group launched early: own %u batches %u epoch %u\n", ch.run, ch.pendP.chainSeq,
                 ch.pendN, ch.epoch);
#endif
    return launch_chained(c, ch.pendP, err);
}

// The closed runs' audit records to State::auditWords (the context's stream finished past their
// final flush: after a synchronisation).  A run still open stays.
void harvest_audit(Ctx &c) {
    if (!c.auditDev) return;
    State &s = S();
    size_t k = 0;
    for (auto &a : c.auditRuns) {
        if (!a.closed) {
            c.auditRuns[k++] = a;
            continue;
        }
        const unsigned recs = std::min(a.hdr[8], hippt::kAuditBatches) + 1u;
        std::vector<unsigned> w(size_t(recs) * hippt::kAuditWords);
        if (hipMemcpy(w.data(), c.auditDev + size_t(a.slab) * hippt::kAuditRunWords, w.size() * sizeof(unsigned),
                      hipMemcpyDeviceToHost) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        s.auditWords.insert(s.auditWords.end(), a.hdr, a.hdr + hippt::kAuditWords);
        s.auditWords.insert(s.auditWords.end(), w.begin(), w.end());
    }
    c.auditRuns.resize(k);
}

// Makes batch `p` (its parameters otherwise complete, `blocks` its grid) the next batch of the open
// run, or of a new run (the old one flushed first): the chain fields, the ring slot's scratch, and
// the launch.  While the run's last enqueued launch has not started, batches are held (not posted)
// and then launched together as one group (MeshParams::chainGroup, up to chainCap): the group is one
// job whose queues walk the item order once for all its batches, as one batch of that many frames
// would (a chain of small batches walks it once per batch: -3.6% for a 1/8 share, r5ad), and a burst
// of async batches gets one launch per group instead of one per batch (each a ~21 us launch that
// finds its batch taken, plus the gap between launches; r5j).  A batch launched on its own is posted
// in the mailbox, so that a running launch may go on with it (chained batches); held batches are
// not, so no launch but their group's takes them.
bool chain_batch(Ctx &c, hippt::MeshParams &p, long long blocks, const RingPlan &ring, const char **err) {
    Ctx::Chain &ch = c.chain;
    p.comb = hippt::CombineParams{c.accum, c.out, nullptr, p.bandPixels, p.totalItems, 0, p.frames, p.comb.format};
    bool same = ch.live && blocks == ch.blocks && chain_same(p, ch.key);
    if (same && ch.seq == 1) {  // the run's frame pattern: every batch the same frames, or the next ones
        const int d = p.firstFrame - ch.firstFrame;
        if (d == 0 || d == p.frames)
            ch.step = d;
        else
            same = false;
    } else if (same && p.firstFrame != ch.firstFrame + int(ch.seq) * ch.step) {
        same = false;
    }
    if (!same) {
        if (!flush_deferred(c, err)) return false;  // the old run's (or an unchained batch's) combines
        // (the ring's buffers: ensure_ring, before the batch was chained)
        const unsigned shift = ring.shift, cap = ring.cap, slots = ring.slots;
        HIP_TRY(hipMemsetAsync(c.chainCtl, 0, hippt::kChainCtlWords * sizeof(unsigned), c.stream));
        ch.live = true;
        ch.run = (ch.run + 1u) & 0x7fffffffu;
        ch.seq = 0;
        ch.epoch = 0;
        ch.lastOwn = 0;
        ch.pendN = 0;
        ch.firstFrame = p.firstFrame;
        ch.step = -1;
        ch.slots = slots;
        ch.shift = shift;
        ch.cap = cap;
        ch.blocks = blocks;
        p.comb.scratch = c.chainScratch;
        p.comb.firstFrame = p.firstFrame;
        ch.key = p;
        ch.audit = nullptr;
        if (S().chainAudit) {
            if (!c.auditDev) {
                HIP_TRY(hipMalloc(&c.auditDev, size_t(hippt::kAuditRuns) * hippt::kAuditRunWords * sizeof(unsigned)));
            }
            if (c.auditRuns.size() >= hippt::kAuditRuns) {  // every slab holds a closed run: to the host first
                HIP_TRY(hipStreamSynchronize(c.stream));
                harvest_audit(c);
            }
            const unsigned slab = c.auditNext++ % hippt::kAuditRuns;
            ch.audit = c.auditDev + size_t(slab) * hippt::kAuditRunWords;
            HIP_TRY(hipMemsetAsync(ch.audit, 0, hippt::kAuditRunWords * sizeof(unsigned), c.stream));
            Ctx::AuditRun a{};
            a.hdr[0] = 0xC4A1D17u;
            a.hdr[1] = ch.run;
            a.hdr[2] = unsigned(c.device);
            a.hdr[3] = unsigned(p.firstFrame);
            a.hdr[4] = ~0u;
            a.hdr[5] = unsigned(p.frames);
            a.hdr[6] = p.bandPixels;
            a.hdr[7] = p.totalItems;
            a.hdr[10] = ch.slots;
            a.slab = slab;
            a.closed = false;
            c.auditRuns.push_back(a);
        }
    }
    p.chainAudit = ch.audit;
    p.scratch = c.chainScratch;
    p.queue = c.chainCtl;
    p.combCtr = nullptr;
    p.comb.scratch = c.chainScratch;
    p.comb.firstFrame = ch.firstFrame;
    p.chainCtl = c.chainCtl;
    p.chainBox = c.chainBoxDev;
    p.chainSeq = ch.seq;
    p.chainRun = ch.run;
    p.chainSlots = ch.slots;
    p.chainShift = ch.shift;
    p.chainCap = ch.cap;
    p.chainStep = ch.step;
    p.chainPosted = ch.seq;
    p.chainGroup = 1;
    c.hostSamples += p.totalItems;
    const unsigned seq = ch.seq++;
    // held while the last launch has not started and the group is not full (64-item runs only: the
    // group interleaves its batches' runs)
    // (kChainHoldRunning: also while the run's only launch so far is still running — the burst's
    // second batch then opens the first group instead of being taken by that launch on its own walk
    // of the item order and leaving its own launch nothing but the combine)
    const bool hold = kChainGroups && ch.epoch > 0 && ch.pendN + 1u < ch.cap && p.totalItems % 64u == 0 &&
                      (hipEventQuery(c.chainStartEv) == hipErrorNotReady ||
                       (kChainHoldRunning && ch.epoch == 1 && hipEventQuery(c.chainEndEv) == hipErrorNotReady));
#ifdef HIPPT_CHAIN_TRACE
    std::fprintf(stderr, "chain run %u seq %u %s (held %u epoch %u cap %u slots %u)\n", ch.run, seq,
                 hold ? "held" : ch.pendN ? "launched with the held ones" : "launched", ch.pendN, ch.epoch,
                 ch.cap, ch.slots);
#endif
    if (hold) {
        if (!ch.pendN) ch.pendP = p;
        ++ch.pendN;
        return true;
    }
    if (ch.pendN) {  // the held batches and this one: one group launch
        hippt::MeshParams q = ch.pendP;
        q.chainGroup = ch.pendN + 1u;
        q.chainPosted = seq;
        return launch_chained(c, q, err);
    }
    // post: one word, so that a launch reads the run, its frame pattern and the last batch together
    const unsigned long long consecutive = ch.step > 0 ? 1u : 0u;
    __atomic_store_n(c.chainBox, ((unsigned long long)ch.run << 33) | (consecutive << 32) | seq, __ATOMIC_RELEASE);
    return launch_chained(c, p, err);
}

// The device address of a mapped pinned host frame on the current device, or null where the
// runtime cannot map it (the caller then copies after the kernel).
uint32_t *host_frame_on_device(unsigned *frame) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, frame, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint32_t *>(d);
}

// copy: the frame's words end in the full-frame pinned host buffer `dst` (State::host when null),
// written by the kernel that makes them (legacy kernel or combine) or copied after it.
bool enqueue_locked(int firstFrame, int count, int maxDepth, bool copy, const char **err, unsigned *dst = nullptr) {
    State &s = S();
    if (!dst) dst = s.host;
    if (!s.ready) return fail(err, "HIP path tracer not initialized");
    if (count < 0) return fail(err, "negative frame count");
    const bool mesh = s.scene.kind == HIPPT_SCENE_MESH;
    const CameraF cam = mesh ? current_camera() : CameraF{};
    for (Ctx &c : s.ctxs) {
        HIP_TRY(hipSetDevice(c.device));
        const int rows = c.rows;
        const unsigned bandPixels = unsigned(rows) * unsigned(s.width);
        bool copied = false;  // the kernel wrote the frame's rows into s.host (legacy zero copy)
        if (rows > 0 && count > 0) {
            if (!mesh) {
                // the legacy kernel writes accum/out itself: a mesh batch's pending combine goes first
                if (!flush_deferred(c, err)) return false;
                hippt::Sphere4Params p{c.accum, c.out, c.stats, s.width, s.height, c.y0, rows, c.stride, firstFrame, count,
                                       maxDepth, s.pixelFormat, nullptr};
                // A blocking frame (the app's cudaPathTracerRender): the kernel writes the words into
                // the pinned host frame itself, overlapping the PCIe transfer with the trace, instead
                // of a D2H copy after it (1080p: 0.17 ms of copy behind 0.13 ms of kernel)
                if (copy && kLegacyZeroCopy) {
                    p.hostOut = host_frame_on_device(dst);
                    copied = p.hostOut != nullptr;  // else the copy after the kernel
                }
                EventPair ev;
                if (!next_events(c, ev, err)) return false;
                HIP_TRY(hipEventRecord(ev.a, c.stream));
                HIP_TRY(hippt::launch_sphere4(p, c.stream));
                HIP_TRY(hipEventRecord(ev.b, c.stream));
                c.pending.push_back({0, ev});
            } else {
                if (!ensure_scene(c, err)) return false;
                const size_t perFrame = size_t(bandPixels) * 3 * sizeof(float);
                const size_t cap = size_t(std::max<long long>(1, s.scratchMB)) << 20;
                int fpb = int(std::max<size_t>(1, cap / perFrame));
                fpb = std::min(fpb, count);
                fpb = int(std::min<long long>(fpb, (1LL << 31) / std::max<unsigned>(1, bandPixels)));
                fpb = std::max(fpb, 1);
                const size_t need = perFrame * size_t(fpb);
                const bool cnt = s.countTraversal;
                // Traversal over the 4-wide tree (HIPPT_OPT_BVH_WIDTH), megakernel and wavefront.
                // Automatic: 4-wide.  With near/far rows read by the ray's octant, 4-wide beats
                // 2-wide on LDS scenes (Cornell 31.7 -> 35.3 G) and on global-memory trees (blob70k
                // 14.2 -> 15.4 G: half the dependent node fetches, 18% fewer load instructions);
                // random_scene (spheres, general kernel) 20.6 vs 20.5 G.
                const bool wide = s.scene.numNodes4 > 0 && s.bvhWidth != 2;
                s.activeWidth = wide ? 4 : 2;
                const int numNodes = wide ? s.scene.numNodes4 : s.scene.numNodes, numTris = s.scene.numTris;
                // small scenes live in LDS (scene bytes beyond the stack under the limit)
                const int numMats = int(s.scene.mats.size() / 2);
                const bool ldsScene = s.ldsScene && hippt::mesh_lds_bytes(0, numNodes, numTris, wide, 0, numMats) <=
                                                        hippt::mesh_lds_scene_limit();
                // LDS stack entries per lane: 2-wide = interior levels (+1 spare); 4-wide = the
                // builder's exact bound up to kWideStackCap (+3 spare; deeper stacks spill their
                // bottom half to global memory), so that 7 blocks of a big scene fit in LDS.  A
                // traversal of a tree in global memory whose bound exceeds kWideStackCap (it
                // spills anyway) keeps kSpillStackCap entries and gives the rest of its LDS to the
                // top of the tree (blob70k, float nodes: cap 19 + 4 top nodes 17.8 G, cap 13 + 52
                // top nodes 20.4 G; caps 9-15 within 1%, 7: -3%; r2w; cap 10 + 76 nodes +0.5%, r3al)
                const bool topTree = wide && !ldsScene;
                const int capLimit = s.stackCap > 0 ? s.stackCap
                                     : ldsScene     ? 30
                                     : topTree && s.scene.stackBound4 > kWideStackCap ? kSpillStackCap
                                                                                       : kWideStackCap;
                const int stackCap = wide ? std::max(1, std::min(s.scene.stackBound4, capLimit)) : 0;
                const int stackDepth = wide ? stackCap + 2 : std::max(1, s.scene.levels);
                const bool spills = wide && s.scene.stackBound4 > stackCap;
                // 8-bit child boxes for trees read from global memory: 64-byte nodes, 4 vector loads
                // instead of 7 where the texture addresser bounds the traversal (blob70k: TA busy
                // 84%, 15.6 -> 17.7 G).  Automatic for the wavefront's Lambertian-triangle kernel
                // only: the megakernel reads the top of the tree (62-70% of the visits) from LDS,
                // where the float nodes need no decode (blob70k 19.0 G 8-bit, 20.4 G float, r2v).
                // (scenes with boxes near +-FLT_MAX have no 8-bit tree: quantize_bvh4 failed)
                // Hybrid (HIPPT_OPT_BVH_QUANT 2, megakernel): the top of the tree as float nodes in LDS
                // (no decode where most visits are) and 8-bit nodes below it (4 loads instead of 7
                // where the texture addresser binds); falls back to 8-bit nodes without a top.
                bool hybrid = wide && !ldsScene && !s.scene.nodes4q.empty() && s.pathMode == 0 && s.bvhQuant == 2 &&
                              s.ldsTopNodes != 0;
                bool quant = wide && !ldsScene && !s.scene.nodes4q.empty() &&
                             (s.bvhQuant == 1 || s.bvhQuant == 2 ||
                              (s.bvhQuant == -1 && !s.scene.full && s.pathMode == 1));
                // Half-precision planes (HIPPT_OPT_BVH_QUANT 3, megakernel and wavefront extend): the
                // float nodes' size and codes, 4 reads per visit instead of 7
                // half planes unless the scene's planes leave the half range (then float nodes)
                const bool half = wide && !ldsScene && s.bvhQuant == 3 && half_tree_ok(s.scene);
                // The top of a global-memory tree in LDS (megakernel and wavefront extend): the
                // breadth-first prefix of the node array that the LDS budget of the resident blocks
                // leaves beside the stack (automatic), or HIPPT_OPT_LDS_TOP_NODES nodes.  The
                // wavefront keeps its 8-bit nodes (blob70k: 8.28 G 8-bit, 7.53 G float, r2za).
                // Camera-ray pool (megakernel, 4-wide float nodes): on by default for LDS-resident
                // scenes and for the Lambertian kernel over a tree in global memory (its pool's LDS
                // comes out of the top of the tree).
                // Pinhole cameras at a nonzero origin start every ray at cam.origin exactly
                // (origin + 0*offset), so their pool entries carry no origin.
                // (round 3, r6j: also for the Lambertian kernel over a tree in global memory,
                // blob70k +1.8% though the pool's LDS comes out of the top; the general kernel
                // there loses 10%, random_scene)
                const bool pool = s.pathMode == 0 && wide && !quant &&
                                  (s.cameraPool == 1 || (s.cameraPool == -1 && (ldsScene || !s.scene.full)));
                if (hybrid) quant = false;  // (pool: off, as for 8-bit nodes)
                const bool pinhole = cam.lens_radius == 0.0f && cam.origin[0] != 0.0f && cam.origin[1] != 0.0f &&
                                     cam.origin[2] != 0.0f;
                const int poolWords = pool ? (pinhole ? hippt::kPoolWordsPinhole : hippt::kPoolWordsFull) : 0;
                unsigned topBytes = 0;
                if (topTree && s.ldsTopNodes != 0) {
                    const size_t nodeBytes = quant ? 64 : 128;  // hybrid: a float top
                    size_t n = size_t(std::min(numNodes, kTopOrderNodes));
                    if (s.ldsTopNodes > 0) {
                        n = std::min(n, size_t(s.ldsTopNodes));
                    } else {
                        const size_t stackBytes = hippt::mesh_lds_bytes(stackDepth, 0, 0, true, 0, 0, poolWords);
                        const size_t budget = hippt::mesh_lds_block_budget();
                        n = std::min(n, budget > stackBytes ? (budget - stackBytes) / nodeBytes : 0);
                    }
                    topBytes = unsigned(n * nodeBytes);
                }
                if (hybrid && topBytes == 0) {  // no LDS left for a top: plain 8-bit nodes
                    hybrid = false;
                    quant = true;
                }
                const int fmt = !wide    ? hippt::kWide2
                                : hybrid ? hippt::kWideHybrid
                                : quant  ? hippt::kWideQuant
                                : half   ? hippt::kWideHalf
                                         : hippt::kWideFloat;
                if (hybrid && !ensure_hybrid(c, int(topBytes / 128), err)) return false;
                if (half && !ensure_half(c, err)) return false;
                const long long occKey =
                    occupancy_key(s.scene.version, stackDepth, ldsScene, s.scene.full, wide, quant, spills) ^
                    ((long long)topBytes << 40) ^ ((long long)poolWords << 36) ^ ((long long)hybrid << 35) ^
                    ((long long)half << 34);
                if (c.occKey != occKey) {
                    const int ln = ldsScene ? numNodes : 0, lt = ldsScene ? numTris : 0, lm = ldsScene ? numMats : 0;
                    c.meshBlocksPerCu[0] = hippt::mesh_blocks_per_cu(false, s.scene.full, fmt, stackDepth, ln, lt,
                                                                     spills, topBytes, lm, poolWords);
                    c.meshBlocksPerCu[1] = hippt::mesh_blocks_per_cu(true, s.scene.full, fmt, stackDepth, ln, lt,
                                                                     spills, topBytes, lm, poolWords);
                    c.meshBlocksPerCuChain = poolWords && fmt == hippt::kWideFloat
                                                 ? hippt::mesh_blocks_per_cu(false, s.scene.full, fmt, stackDepth, ln,
                                                                             lt, spills, topBytes, lm, poolWords, true)
                                                 : 0;
                    c.occKey = occKey;
                }
                s.activeTopBytes = topBytes;
                s.activeBlocksPerCu = c.meshBlocksPerCu[cnt ? 1 : 0];
                int bpc = s.blocksPerCu > 0 ? s.blocksPerCu : c.meshBlocksPerCu[cnt ? 1 : 0];
                for (int b = 0; b < count; b += fpb) {
                    const int nf = std::min(fpb, count - b);
                    const unsigned total = bandPixels * unsigned(nf);
                    // the megakernel takes the previous batch's combine along; other batches flush it
                    const bool fuse = maxDepth > 0 && s.pathMode == 0 && s.fuseCombine != 0;
                    // chained batches (Ctx::chain): asynchronous camera-pool megakernel batches over
                    // 4-wide float nodes whose items fit the ring's slot bits
                    bool chained = fuse && !copy && !cnt && s.chainBatches != 0 &&
                                   poolWords != 0 &&
                                   fmt == hippt::kWideFloat && c.meshBlocksPerCuChain > 0 &&
                                   total <= (1u << hippt::kChainMaxShift);
                    RingPlan ring;
                    if (chained) {
                        ring = ring_plan(total, s.chainBatches, ldsScene, cap);
                        bool ok = ring.bytes != 0;
                        if (ok && !ensure_ring(c, ring, &ok, err)) return false;
                        chained = ok;
                    }
                    if ((!fuse || !chained) && !flush_chain(c, err)) return false;
                    if (!fuse && !flush_deferred(c, err)) return false;
                    float *scratch = nullptr;
                    if (!chained && !batch_scratch(c, need, &scratch, err)) return false;
                    if (maxDepth <= 0) {
                        // ray_color with depth <= 0 returns black without tracing (RayTracer.h:582-583)
                        HIP_TRY(hipMemsetAsync(scratch, 0, size_t(total) * 3 * sizeof(float), c.stream));
                    } else {
                        hippt::MeshParams p{};
                        p.nodes = hybrid ? c.nodes4h : quant ? c.nodes4q : half ? c.nodes4f : wide ? c.nodes4 : c.nodes;
                        p.tris = c.tris;
                        p.shade = c.shade;
                        p.mats = c.mats;
                        p.scratch = scratch;
                        p.queue = c.queue;
                        p.stats = c.stats;
                        p.cam = cam;
                        p.invW = 1.0f / float(std::max(1, s.width - 1));
                        p.invH = 1.0f / float(std::max(1, s.height - 1));
                        p.width = s.width;
                        p.height = s.height;
                        p.y0 = c.y0;
                        p.bandRows = rows;
                        p.rowStride = c.stride;
                        p.firstFrame = firstFrame + b;
                        p.frames = nf;
                        p.maxDepth = maxDepth;
                        p.bandPixels = bandPixels;
                        p.totalItems = total;
                        p.rcpBandPixels = 1.0f / float(bandPixels);
                        p.rcpWidth = 1.0f / float(s.width);
                        p.stackDepth = stackDepth;
                        p.numNodes = numNodes;
                        p.numTris = numTris;
                        p.numMats = numMats;
                        p.ldsScene = ldsScene ? 1 : 0;
                        p.full = s.scene.full ? 1 : 0;
                        // shade once fewer than this many lanes still traverse (re-swept in round 3
                        // under the sample-length item order, r5y-r6a: LDS scenes 24 with the exits
                        // below, Cornell 48.4 -> 53.7 G; global-memory trees 32, blob70k 24 and 40
                        // lower)
                        // (the general megakernel over a tree in global memory: 24, random_scene
                        // +5.8% over 32 with the exits below, r6c)
                        // Re-swept on round 6's kernels (r6aj/r6ak, alternating passes): a whole
                        // blob70k image 40 over 32 +0.5-0.7% (21,882 -> 22,031 M/s; 36 +0.5%, 44 and 48
                        // slower), configs[3]'s 4K image +0.6%, but its 1/8 shares 2.433 -> 2.471 ms:
                        // 40 with the loop exits 22 / 56 below (alone, 40 slowed the shares: r6ak);
                        // Cornell 28/32 within 0.2% of 24.
                        const bool fullMega = s.pathMode == 0 && s.scene.full;
                        // Lambertian batches over a tree in global memory, megakernel or wavefront (this
                        // wave threshold and the loop exits below; the wavefront's configs[4] 14,243 ->
                        // 14,436 M/s with 40 / 22 / 56, r6aq; blob70k's 1/4 and 1/8 row shares 4.705 ->
                        // 4.612 and 2.433 -> 2.391 ms, r6at)
                        const bool lambertGlobal = !ldsScene && !s.scene.full;
                        p.waveThreshold = s.waveThreshold >= 0    ? s.waveThreshold
                                          : ldsScene || fullMega ? 24
                                          : lambertGlobal        ? 40
                                                                 : 32;
                        // claim size: 512 items for the Lambertian kernels' chained and whole-image
                        // batches (Cornell 1080p/64 spp 7.255 -> 7.199 ms, blob70k 18.94 -> 18.91,
                        // r5s; chained 1/8 shares Cornell 1.062 -> 1.041, blob70k 2.546 -> 2.547,
                        // r5ab); 256 for small unchained batches (1/8 shares: Cornell 1.112 -> 1.137
                        // and blob70k 3.00 -> 3.22 with 512) and the general kernel (cornell_mixed
                        // 12.06 -> 12.22)
                        p.chunk = s.chunk > 0 ? s.chunk
                                  : s.pathMode == 0 && !s.scene.full && (chained || total >= (1u << 26)) ? 512u
                                                                                                         : 256u;
                        // Loop exits of the traversal round (measured): trees in global
                        // memory leave the node loop once <= 17 lanes still search for a leaf (r2
                        // sweep of the 4-wide kernels: blob70k, 21 levels, best at 17-18; blob64x34
                        // and random_scene, 16 and 12 levels, best at 15) and the leaf loop once
                        // <= 48 lanes hold a leaf; LDS scenes at 12 and 8 (round 3, with the item
                        // order: node exit 4-16 x leaf exit 8-16 within 0.6% of the best, Cornell
                        // 53.8 G; the round-2 values 4 and 48 gave 48.4 G), except that the general
                        // kernel and the wavefront keep leaf exit 4 (cornell_mixed +1.4%, Cornell
                        // wavefront +6% over 12; r6b)
                        // The general megakernel over a tree in global memory: 12 and 16 (random_scene,
                        // r6c).  The Lambertian kernels over a tree in global memory, with the wave
                        // threshold 40: 22 and 56 (blob70k whole image, alternating passes: 22,057 ->
                        // 22,372 M/s, +1.4%; 20-26 x 48-64 within 0.3% of it, 28 lower, r6ao/r6ap).
                        const bool lambertMega = s.pathMode == 0 && !s.scene.full;
                        p.leafExit = unsigned(s.leafExit >= 0 ? s.leafExit
                                              : ldsScene          ? (lambertMega ? 12 : 4)
                                              : fullMega          ? 12
                                              : lambertGlobal     ? 22
                                                                  : 17);
                        p.nodeExit = unsigned(s.nodeExit >= 0 ? s.nodeExit
                                              : ldsScene  ? 8
                                              : fullMega  ? 16
                                              : lambertGlobal ? 56
                                                              : 48);
                        p.wide = fmt;
                        p.stackCap = stackCap;
                        p.topBytes = topBytes;
                        p.refBits = ldsScene && wide ? packed_ref_bits(numNodes, numTris) : 0u;
                        p.rngTable = nullptr;
                        p.poolWords = poolWords;
                        // Pixel runs by estimated sample length, longest first, per XCD queue
                        // (megakernel; item_order.h): Cornell +2.4%, cornell_mixed +3%, blob70k
                        // +0.8% at full size; the slowest 1/8 Cornell share -2% (r5w)
                        if (s.pathMode == 0 && s.itemOrder != 0) {
                            const unsigned *table = nullptr;
                            // the runs' shape: HIPPT_OPT_PIXEL_TILE columns.  Automatic: 8x8 tiles for
                            // a band of consecutive rows (blob70k 1080p +0.45%, Cornell +0.6%, two
                            // alternating passes, r6d), row runs for an interleaved share (the tile's
                            // rows are `stride` image rows apart: the 1/8 shares neutral to -0.9%, r6f)
                            const int tile = s.pixelTile >= 0 ? s.pixelTile : c.stride == 1 ? 8 : 0;
                            const unsigned tileShift = tile == 8 ? 3u : tile == 16 ? 4u : tile == 32 ? 5u : 6u;
                            if (!ensure_order(c, cam, nf, maxDepth, s.itemOrder == 1, tileShift, &table, err))
                                return false;
                            if (table) {
                                p.runOrder = table;
                                p.runCount = unsigned(c.runCosts.size());
                                p.runTileShift = c.orderKey.tileShift;
                            }
                        }
                        p.poolOffset = unsigned(hippt::mesh_lds_bytes(stackDepth, ldsScene ? numNodes : 0,
                                                                      ldsScene ? numTris : 0, wide, topBytes,
                                                                      ldsScene ? numMats : 0));
                        if (s.rngTable && !rng_table(c, &p.rngTable, err)) return false;
                        if (s.pathMode == 1) {
                            if (!run_wavefront(c, p, cnt, spills, s.scene.stackBound4 + 3, err)) return false;
                        } else {
                            long long blocks =
                                (long long)c.cus * (chained && s.blocksPerCu <= 0 ? c.meshBlocksPerCuChain : bpc);
                            blocks = std::min<long long>(blocks, (total + hippt::kMeshBlock - 1) / hippt::kMeshBlock);
                            blocks = std::max<long long>(blocks, 1);
                            if (!ensure_spill(c, p, blocks, spills, s.scene.stackBound4 + 3, err)) return false;
                            s.activeChunk = int(p.chunk);
                            s.activeChainCap = 0;
                            if (chained) {
                                p.comb.format = s.pixelFormat;
                                if (!chain_batch(c, p, blocks, ring, err)) return false;
                                s.activeChainCap = int(c.chain.cap);
                                continue;  // launched or taken by the run's last launch; its combine
                                           // belongs to the run (Ctx::chain)
                            } else {
                                HIP_TRY(hipMemsetAsync(c.queue, 0, kQueueBytes, c.stream));
                                if (c.hasDeferred) {
                                    p.comb = c.deferred;
                                    c.hasDeferred = false;
                                }
                                p.combCtr = c.queue + kCombCtrWord;
                            }
                            EventPair ev;
                            if (!next_events(c, ev, err)) return false;
                            HIP_TRY(hipEventRecord(ev.a, c.stream));
                            HIP_TRY(hippt::launch_mesh(p, int(blocks), cnt, c.stream));
                            HIP_TRY(hipEventRecord(ev.b, c.stream));
                            c.pending.push_back({0, ev});
                        }
                    }
                    if (chained && maxDepth > 0) continue;  // its combine belongs to the run (Ctx::chain)
                    c.deferred = hippt::CombineParams{c.accum, c.out, scratch, bandPixels, total, firstFrame + b, nf,
                                                      s.pixelFormat};
                    c.hasDeferred = true;
                    if (!fuse && !flush_deferred(c, err)) return false;
                }
            }
        }
        if (copy && rows > 0 && c.hasDeferred && kLegacyZeroCopy) {
            // a blocking mesh frame: its combine writes the words into the pinned host frame too
            if (uint32_t *d = host_frame_on_device(dst)) {
                c.deferredHost = hippt::HostFrame{d, s.width, c.y0, c.stride};
                copied = true;
            }
        }
        if (copy && !flush_deferred(c, err)) return false;
        if (copy && rows > 0 && !copied) {
            if (!copy_rows_async(c, dst, c.out, sizeof(uint32_t), err)) return false;
        }
    }
    return true;
}

bool sync_locked(const char **err) {
    State &s = S();
    for (Ctx &c : s.ctxs) {
        if (!flush_deferred(c, err)) return false;
        HIP_TRY(hipSetDevice(c.device));
        HIP_TRY(hipStreamSynchronize(c.stream));
        for (auto &pe : c.pending)
            if (!account(pe, c, err)) return false;
        c.pending.clear();
        harvest_audit(c);
    }
    return true;
}

bool render_locked(int frameIndex, int count, int maxDepth, const unsigned int **hostPixels, const char **err) {
    if (!enqueue_locked(frameIndex, count, maxDepth, true, err)) return false;
    if (!sync_locked(err)) return false;
    if (hostPixels) *hostPixels = S().host;
    return true;
}

}  // namespace

// ---- reference ABI ----------------------------------------------------------------------------
extern "C" bool cudaPathTracerInit(int width, int height, const char **errorMessage) try {
    std::lock_guard<std::mutex> g(S().mu);
    return init_locked(width, height, errorMessage);
} catch (const std::exception &e) {
    return fail_free(errorMessage, e.what());
} catch (...) {
    return fail_free(errorMessage, "unknown exception");
}

extern "C" bool cudaPathTracerRender(int frameIndex, int maxDepth, const unsigned int **hostPixels,
                                     const char **errorMessage) try {
    std::lock_guard<std::mutex> g(S().mu);
    // the CUDA backend's ABI always hands out its ARGB words (HIPPT_OPT_PIXEL_FORMAT applies to
    // the hippt* render calls)
    // (restored on every way out, an exception caught below included: ADVICE r4)
    struct FormatScope {
        int &fmt;
        const int saved;
        ~FormatScope() { fmt = saved; }
    } scope{S().pixelFormat, S().pixelFormat};
    scope.fmt = HIPPT_PIXEL_ARGB;
    return render_locked(frameIndex, 1, maxDepth, hostPixels, errorMessage);
} catch (const std::exception &e) {
    return fail_free(errorMessage, e.what());
} catch (...) {
    return fail_free(errorMessage, "unknown exception");
}

extern "C" void cudaPathTracerShutdown(void) try {
    std::lock_guard<std::mutex> g(S().mu);
    destroy_all();
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}

extern "C" bool hipPathTracerInit(int width, int height, const char **errorMessage) try {
    return cudaPathTracerInit(width, height, errorMessage);
} catch (const std::exception &e) {
    return fail_free(errorMessage, e.what());
} catch (...) {
    return fail_free(errorMessage, "unknown exception");
}
extern "C" bool hipPathTracerRender(int frameIndex, int maxDepth, const unsigned int **hostPixels,
                                    const char **errorMessage) try {
    return cudaPathTracerRender(frameIndex, maxDepth, hostPixels, errorMessage);
} catch (const std::exception &e) {
    return fail_free(errorMessage, e.what());
} catch (...) {
    return fail_free(errorMessage, "unknown exception");
}
extern "C" void hipPathTracerShutdown(void) { cudaPathTracerShutdown(); }

// ---- scene --------------------------------------------------------------------------------------
extern "C" void hipptBuildCamera(const double lookfrom[3], const double lookat[3], const double vup[3],
                                 double vfovDeg, double aspect, double aperture, double focusDist, hipptCamera *out) try {
    static_assert(sizeof(hipptCamera) == sizeof(CameraF), "camera layout");
    CameraF c;
    build_camera(lookfrom, lookat, vup, vfovDeg, aspect, aperture, focusDist, c);
    std::memcpy(out, &c, sizeof(c));
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}

extern "C" bool hipptUseBuiltinScene(int sceneId, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    if (sceneId != HIPPT_SCENE_SPHERE4) return fail(err, "unknown built-in scene id");
    // a pending mesh combine belongs to the image rendered so far: enqueue it before the switch
    for (Ctx &c : S().ctxs)
        if (!flush_deferred(c, err)) return false;
    S().scene.kind = HIPPT_SCENE_SPHERE4;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptUploadScene(const float *verts, const int *triMaterial, int numTris, const float *spheres,
                                 const int *sphereMaterial, int numSpheres, const hipptMaterial *materials,
                                 int numMaterials, const double lookfrom[3], const double lookat[3],
                                 const double vup[3], double vfovDeg, double aperture, double focusDist,
                                 const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (numTris < 0 || numSpheres < 0) return fail(err, "negative primitive count");
    if ((numTris > 0 && (!verts || !triMaterial)) || (numSpheres > 0 && (!spheres || !sphereMaterial)) ||
        !materials || !lookfrom || !lookat || !vup)
        return fail(err, "null scene pointer");
    if (numMaterials <= 0) return fail(err, "scene needs at least one material");
    if (numTris + (long long)numSpheres >= (1LL << 27)) return fail(err, "too many primitives");
    for (int i = 0; i < numTris; ++i)
        if (triMaterial[i] < 0 || triMaterial[i] >= numMaterials) return fail(err, "triangle material out of range");
    for (int j = 0; j < numSpheres; ++j) {
        if (sphereMaterial[j] < 0 || sphereMaterial[j] >= numMaterials) return fail(err, "sphere material out of range");
        for (int a = 0; a < 4; ++a)
            if (!std::isfinite(spheres[4 * j + a])) return fail(err, "non-finite sphere");
    }
    bool full = numSpheres > 0;
    for (int m = 0; m < numMaterials; ++m) {
        const hipptMaterial &mt = materials[m];
        if (mt.kind < HIPPT_MAT_LAMBERTIAN || mt.kind > HIPPT_MAT_DIELECTRIC) return fail(err, "unknown material kind");
        if (!std::isfinite(mt.albedo[0]) || !std::isfinite(mt.albedo[1]) || !std::isfinite(mt.albedo[2]) ||
            !std::isfinite(mt.fuzz) || !std::isfinite(mt.ir))
            return fail(err, "non-finite material parameter");
        full = full || mt.kind != HIPPT_MAT_LAMBERTIAN;
    }
    // primitive id p: triangles 0..numTris-1, then spheres (the closest-hit tie order)
    const int numPrims = numTris + numSpheres;
    std::vector<float> boxes(size_t(numPrims) * 6);
    for (int i = 0; i < numTris; ++i) {
        const float *v = verts + 9 * size_t(i);
        float *bx = &boxes[6 * size_t(i)];
        for (int a = 0; a < 3; ++a) {
            bx[a] = std::min(v[a], std::min(v[3 + a], v[6 + a]));
            bx[3 + a] = std::max(v[a], std::max(v[3 + a], v[6 + a]));
        }
    }
    for (int j = 0; j < numSpheres; ++j) {
        const float *q = spheres + 4 * size_t(j);
        // slack for the FP32 root's error near the box faces (pt_oracle.c po_scene_create2)
        const float r = std::fabs(q[3]) * (1.0f + 1.0f / 4096.0f);
        float *bx = &boxes[6 * size_t(numTris + j)];
        for (int a = 0; a < 3; ++a) {
            bx[a] = q[a] - r;
            bx[3 + a] = q[a] + r;
        }
    }
    float extent = 0.0f;
    for (int i = 0; i < 3; ++i) extent = std::max(extent, float(std::fabs(lookfrom[i])));
    hippt::Bvh bvh;
    std::string msg;
    if (!hippt::build_bvh_boxes(boxes.data(), numPrims, extent, bvh, msg, s.bvh)) return fail(err, msg);
    SceneHost sc;  // the new scene, swapped in at the end (a failure keeps the old one)
    sc.version = s.scene.version;
    sc.nodes.assign(bvh.nodes.size() / 4, float4{});
    std::memcpy(sc.nodes.data(), bvh.nodes.data(), bvh.nodes.size() * sizeof(uint32_t));
    hippt::Bvh4 bvh4;
    hippt::collapse_bvh4(bvh, bvh4, s.bvh);
    if (s.bvh.collapse == -1) {
        // Automatic collapse: the SAH-optimal 4-wide tree for scenes that fit the LDS scene copy
        // (leaves of <= 2 primitives: Cornell +1.6-1.9%, cornell_mixed +1.0%, r3ap/r3aq), the
        // greedy one for trees read from global memory (SAH-optimal: blob70k -9%, random_scene -4%)
        auto fits = [&](const hippt::Bvh4 &b) {
            return hippt::mesh_lds_bytes(0, int(b.nodes.size() / hippt::kNode4Words), numPrims, true, 0,
                                         numMaterials) <= hippt::mesh_lds_scene_limit();
        };
        if (fits(bvh4)) {
            hippt::BvhParams p = s.bvh;
            p.collapse = 1;
            hippt::Bvh4 sah;
            hippt::collapse_bvh4(bvh, sah, p);
            if (fits(sah)) bvh4 = std::move(sah);
        }
    }
    hippt::order_bvh4_top(bvh4, kTopOrderNodes);
    sc.nodes4.assign(bvh4.nodes.size() / 4, float4{});
    std::memcpy(sc.nodes4.data(), bvh4.nodes.data(), bvh4.nodes.size() * sizeof(uint32_t));
    sc.numNodes4 = int(bvh4.nodes.size() / hippt::kNode4Words);
    std::vector<uint32_t> q;
    (void)hippt::quantize_bvh4(bvh4, q);  // empty on failure: the float nodes serve every path
    sc.nodes4q.assign(q.size() / 4, float4{});
    std::memcpy(sc.nodes4q.data(), q.data(), q.size() * sizeof(uint32_t));
    sc.bvh4 = bvh4;
    sc.q4 = q;
    sc.hybrid.clear();
    sc.hybridTop = -1;
    if (bvh4.nodes.size() / hippt::kNode4Words >= (1u << 24)) return fail(err, "4-wide BVH too large (2^24 nodes)");
    // device layouts of the 4-wide trees: an interior child's code is its node's BYTE offset (the
    // kernels address a node without a multiply; leaf codes and the root, 0, are unchanged)
    auto byte_codes = [](std::vector<float4> &v, int nodeWords, int codeWord, int stride) {
        auto *w = reinterpret_cast<int32_t *>(v.data());
        const size_t n = v.size() * 4 / size_t(nodeWords);
        for (size_t k = 0; k < n; ++k)
            for (int i = 0; i < 4; ++i) {
                int32_t &c = w[k * size_t(nodeWords) + size_t(codeWord + i)];
                if (c >= 0) c *= stride;
            }
    };
    byte_codes(sc.nodes4, hippt::kNode4Words, 24, hippt::kNode4Words * 4);
    byte_codes(sc.nodes4q, hippt::kNode4QWords, 12, hippt::kNode4QWords * 4);
    sc.nodes4f.clear();
    sc.halfState = 0;
    sc.levels4 = bvh4.levels;
    sc.stackBound4 = bvh4.stackBound;
    sc.tris.assign(size_t(numPrims) * 3, float4{});
    sc.shade.assign(size_t(numPrims), float4{});
    for (int k = 0; k < numPrims; ++k) {
        const int id = bvh.order[size_t(k)];
        if (id >= numTris) {  // sphere: (center, r) (r^2) (-, id, tag 1); shade (center, mat | flag)
            const float *q = spheres + 4 * size_t(id - numTris);
            sc.tris[3 * size_t(k)] = float4{q[0], q[1], q[2], q[3]};
            sc.tris[3 * size_t(k) + 1] = float4{q[3] * q[3], 0.0f, 0.0f, 0.0f};
            sc.tris[3 * size_t(k) + 2] = float4{0.0f, as_float(id), as_float(1), 0.0f};
            sc.shade[size_t(k)] =
                float4{q[0], q[1], q[2], as_float(sphereMaterial[id - numTris] | hippt::kShadeSphere)};
            continue;
        }
        const float *v = verts + 9 * size_t(id);
        // po_tri_setup (oracle) restated: e1 = v1-v0, e2 = v2-v0, n = cross/len
        float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        float cr[3], n[3];
        fcross(e1, e2, cr);
        const float len = std::sqrt(fdot(cr, cr));
        if (!(len > 0.0f)) {
            e1[0] = e1[1] = e1[2] = 0.0f;
            e2[0] = e2[1] = e2[2] = 0.0f;
            n[0] = n[1] = n[2] = 0.0f;
        } else {
            const float inv = 1.0f / len;
            for (int a = 0; a < 3; ++a) n[a] = cr[a] * inv;
        }
        sc.tris[3 * size_t(k)] = float4{v[0], v[1], v[2], e1[0]};
        sc.tris[3 * size_t(k) + 1] = float4{e1[1], e1[2], e2[0], e2[1]};
        sc.tris[3 * size_t(k) + 2] = float4{e2[2], as_float(id), 0.0f, 0.0f};
        sc.shade[size_t(k)] = float4{n[0], n[1], n[2], as_float(triMaterial[id])};
    }
    sc.mats.assign(size_t(numMaterials) * 2, float4{});
    for (int m = 0; m < numMaterials; ++m) {
        const hipptMaterial &mt = materials[m];
        // Metal(a, f): fuzz(f < 1 ? f : 1), RayTracer.h:494
        const float fuzz = mt.kind == HIPPT_MAT_METAL && !(mt.fuzz < 1.0f) ? 1.0f : mt.fuzz;
        sc.mats[2 * size_t(m)] = float4{mt.albedo[0], mt.albedo[1], mt.albedo[2], as_float(mt.kind)};
        sc.mats[2 * size_t(m) + 1] = float4{fuzz, mt.ir, 0.0f, 0.0f};
    }
    sc.numTris = numPrims;
    sc.numNodes = int(bvh.nodes.size() / hippt::kNodeWords);
    sc.levels = bvh.levels;
    sc.full = full;
    for (int i = 0; i < 3; ++i) {
        sc.lookfrom[i] = lookfrom[i];
        sc.lookat[i] = lookat[i];
        sc.vup[i] = vup[i];
    }
    sc.vfov = vfovDeg;
    sc.aperture = aperture;
    sc.focus = focusDist;
    sc.rawCamera = false;
    sc.kind = HIPPT_SCENE_MESH;
    ++sc.version;
    s.scene = std::move(sc);
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptUploadMesh(const float *verts, const int *triMaterial, int numTris, const float *albedo,
                                int numMaterials, const double lookfrom[3], const double lookat[3],
                                const double vup[3], double vfovDeg, double aperture, double focusDist,
                                const char **err) try {
    if (!albedo) return fail(err, "null scene pointer");
    if (numTris <= 0) return fail(err, "BVH requires at least one triangle");
    std::vector<hipptMaterial> mats(size_t(std::max(0, numMaterials)));
    for (int m = 0; m < numMaterials; ++m)
        mats[size_t(m)] = hipptMaterial{HIPPT_MAT_LAMBERTIAN, {albedo[3 * m], albedo[3 * m + 1], albedo[3 * m + 2]}, 0.0f,
                                        1.0f};
    return hipptUploadScene(verts, triMaterial, numTris, nullptr, nullptr, 0, mats.data(), numMaterials, lookfrom,
                            lookat, vup, vfovDeg, aperture, focusDist, err);
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

namespace {
struct MeshOwner {
    hippt::MeshData data;
    std::vector<const char *> names;
};
}  // namespace

extern "C" bool hipptReadMesh(const char *path, hipptMesh *out, const char **err) try {
    if (!path || !out) return fail(err, "null argument");
    std::memset(out, 0, sizeof(*out));
    std::unique_ptr<MeshOwner> own(new MeshOwner);
    std::string msg;
    if (!hippt::read_mesh(path, own->data, msg)) {
        std::lock_guard<std::mutex> g(S().mu);
        return fail(err, msg);
    }
    for (const std::string &n : own->data.groups) own->names.push_back(n.c_str());
    out->verts = own->data.verts.data();
    out->triGroup = own->data.group.data();
    out->numTris = int(own->data.group.size());
    out->numGroups = int(own->data.groups.size());
    out->groupNames = own->names.data();
    out->owner_ = own.release();
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" void hipptFreeMesh(hipptMesh *mesh) try {
    if (!mesh) return;
    delete static_cast<MeshOwner *>(mesh->owner_);
    std::memset(mesh, 0, sizeof(*mesh));
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}

extern "C" bool hipptSetCamera(const hipptCamera *camera, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    if (!camera) return fail(err, "null camera");
    std::memcpy(&S().scene.cam, camera, sizeof(CameraF));
    S().scene.rawCamera = true;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

// ---- devices ------------------------------------------------------------------------------------
extern "C" int hipptDeviceCount(void) try {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
} catch (const std::exception &e) {
    return 0;
} catch (...) {
    return 0;
}

extern "C" bool hipptSetDevices(const int *deviceIds, int numDevices, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (numDevices < 0 || (numDevices > 0 && !deviceIds)) return fail(err, "invalid device list");
    int avail = 0;
    HIP_TRY(hipGetDeviceCount(&avail));
    for (int i = 0; i < numDevices; ++i)
        if (deviceIds[i] < 0 || deviceIds[i] >= avail) return fail(err, "device id out of range");
    s.devices.assign(deviceIds, deviceIds + numDevices);
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptSetRowRange(int y0, int y1, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    if (y0 < 0 || (y1 > 0 && y1 < y0)) return fail(err, "invalid row range");
    S().rowY0 = y0;
    S().rowY1 = y1;
    S().rowPhase = 0;
    S().rowStride = 1;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptSetRowInterleave(int phase, int stride, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    if (stride < 1 || phase < 0 || phase >= stride) return fail(err, "invalid row interleave");
    S().rowPhase = phase;
    S().rowStride = stride;
    S().rowY0 = 0;
    S().rowY1 = 0;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

// ---- rendering ----------------------------------------------------------------------------------
extern "C" bool hipptRenderFrames(int firstFrame, int count, int maxDepth, const unsigned int **hostPixels,
                                  const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    return render_locked(firstFrame, count, maxDepth, hostPixels, err);
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptRenderFramesAsync(int firstFrame, int count, int maxDepth, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    return enqueue_locked(firstFrame, count, maxDepth, false, err);
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptSynchronize(const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    return sync_locked(err);
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptRenderFramesPresent(int firstFrame, int count, int maxDepth, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!s.ready) return fail(err, "HIP path tracer not initialized");
    const int b = s.presentNext;
    // mapped + coherent like State::host: the frame's kernel writes the hand-off frame itself
    if (!s.present[b])
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.present[b]), s.hostCount * sizeof(unsigned),
                              hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    if (!enqueue_locked(firstFrame, count, maxDepth, true, err, s.present[b])) return false;
    for (Ctx &c : s.ctxs) {
        HIP_TRY(hipSetDevice(c.device));
        if (!c.presentEv[b]) HIP_TRY(hipEventCreateWithFlags(&c.presentEv[b], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c.presentEv[b], c.stream));
        if (!harvest_locked(c, err)) return false;
    }
    if (s.latest == b) s.latest = -1;  // its image is being replaced
    s.presentPending[b] = true;
    s.presentSeq[b] = s.presentCalls++;
    s.presentFrames[b] = firstFrame + count;
    s.presentNext = b ^ 1;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptLatestFrame(const unsigned int **hostPixels, int *frames, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!s.ready) return fail(err, "HIP path tracer not initialized");
    for (int b = 0; b < 2; ++b) {
        if (!s.presentPending[b]) continue;
        bool done = true;
        for (Ctx &c : s.ctxs) {
            HIP_TRY(hipSetDevice(c.device));
            const hipError_t q = hipEventQuery(c.presentEv[b]);
            if (q == hipErrorNotReady) {
                done = false;
                break;
            }
            if (q != hipSuccess) return fail(err, std::string("hipEventQuery: ") + hipGetErrorString(q));
        }
        if (done) {
            s.presentPending[b] = false;
            if (s.latest < 0 || s.presentSeq[b] > s.presentSeq[s.latest]) s.latest = b;
        }
    }
    if (hostPixels) *hostPixels = s.latest >= 0 ? s.present[s.latest] : nullptr;
    if (frames) *frames = s.latest >= 0 ? s.presentFrames[s.latest] : 0;
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptReadback(unsigned int *pixels, float *accum, const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!s.ready) return fail(err, "HIP path tracer not initialized");
    if (!sync_locked(err)) return false;
    for (Ctx &c : s.ctxs) {
        HIP_TRY(hipSetDevice(c.device));
        if (pixels && !copy_rows_async(c, pixels, c.out, sizeof(uint32_t), err)) return false;
        if (accum && !copy_rows_async(c, accum, c.accum, sizeof(float4), err)) return false;
        HIP_TRY(hipStreamSynchronize(c.stream));
    }
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

extern "C" bool hipptResetAccumulation(const char **err) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!s.ready) return fail(err, "HIP path tracer not initialized");
    for (Ctx &c : s.ctxs) {
        if (!flush_deferred(c, err)) return false;
        HIP_TRY(hipSetDevice(c.device));
        const size_t px = size_t(c.rows) * size_t(s.width);
        HIP_TRY(hipMemsetAsync(c.accum, 0, px * sizeof(float4), c.stream));
        HIP_TRY(hipStreamSynchronize(c.stream));
    }
    return true;
} catch (const std::exception &e) {
    return fail_free(err, e.what());
} catch (...) {
    return fail_free(err, "unknown exception");
}

// A context's launch counters summed over their kStatSlots copies (hippt_device.h).
bool read_stats(const Ctx &c, unsigned long long (&v)[kStatWords]) {
    std::vector<unsigned long long> all(size_t(kStatSlots) * kStatWords);
    std::memset(v, 0, sizeof(v));
    if (hipSetDevice(c.device) != hipSuccess) return false;
    if (hipMemcpy(all.data(), c.stats, kStatBytes, hipMemcpyDeviceToHost) != hipSuccess) return false;
    for (int k = 0; k < kStatSlots; ++k)
        for (int i = 0; i < kStatWords; ++i) v[i] += all[size_t(k) * kStatWords + size_t(i)];
    return true;
}

// ---- counters / options -------------------------------------------------------------------------
extern "C" bool hipptGetStats(hipptStats *out) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!out) return false;
    std::memset(out, 0, sizeof(*out));
    const char *err = nullptr;
    if (s.ready && !sync_locked(&err)) return false;
    for (Ctx &c : s.ctxs) {
        unsigned long long v[kStatWords];
        if (!read_stats(c, v)) return false;
        out->segments += v[0];
        out->pixelSamples += v[1] + c.hostSamples;
        out->nodeVisits += v[2];
        out->triTests += v[3];
    }
    out->traceMs = s.traceMs;
    out->combineMs = s.combineMs;
    out->traceLaunches = s.traceLaunches;
    out->combineLaunches = s.combineLaunches;
    out->bvhNodes = s.scene.kind == HIPPT_SCENE_MESH ? s.scene.numNodes : 0;
    out->bvhDepth = s.scene.kind == HIPPT_SCENE_MESH ? s.scene.levels : 0;
    out->numTris = s.scene.kind == HIPPT_SCENE_MESH ? s.scene.numTris : 0;
    out->numDevices = int(s.ctxs.size());
    return true;
} catch (const std::exception &e) {
    return false;
} catch (...) {
    return false;
}

extern "C" int hipptGetCounters(unsigned long long *out, int n) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    if (!out || n <= 0) return 0;
    n = std::min(n, kStatWords);
    std::memset(out, 0, sizeof(unsigned long long) * size_t(n));
    const char *err = nullptr;
    if (s.ready && !sync_locked(&err)) return 0;
    for (Ctx &c : s.ctxs) {
        unsigned long long v[kStatWords];
        if (!read_stats(c, v)) return 0;
        v[1] += c.hostSamples;
        for (int i = 0; i < n; ++i) out[i] += v[i];
    }
    return n;
} catch (const std::exception &e) {
    return 0;
} catch (...) {
    return 0;
}

extern "C" void hipptResetStats(void) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    const char *err = nullptr;
    if (s.ready) sync_locked(&err);
    for (Ctx &c : s.ctxs) {
        (void)hipSetDevice(c.device);
        (void)hipMemset(c.stats, 0, kStatBytes);
        c.hostSamples = 0;
    }
    s.traceMs = s.combineMs = 0;
    s.traceLaunches = s.combineLaunches = 0;
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}

extern "C" bool hipptSetOption(int key, long long value) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    switch (key) {
    case HIPPT_OPT_COUNT_TRAVERSAL: s.countTraversal = value != 0; return true;
    case HIPPT_OPT_WAVE_THRESHOLD:
        if (value < -1 || value > 64) return false;
        s.waveThreshold = int(value);
        return true;
    case HIPPT_OPT_SCRATCH_MB:
        if (value < 1) return false;
        s.scratchMB = value;
        return true;
    case HIPPT_OPT_CHUNK:
        if (value != 0 && (value < 64 || value > (1 << 20) || value % 64)) return false;
        s.chunk = unsigned(value);
        return true;
    case HIPPT_OPT_BLOCKS_PER_CU:
        if (value < 0 || value > 8) return false;
        s.blocksPerCu = int(value);
        return true;
    case HIPPT_OPT_LDS_SCENE: s.ldsScene = value != 0; return true;
    case HIPPT_OPT_PATH_MODE:
        if (value != 0 && value != 1) return false;
        s.pathMode = int(value);
        return true;
    case HIPPT_OPT_WAVEFRONT_SLOTS:
        if (value < 64 || value > (1LL << 28)) return false;
        s.wfSlots = unsigned(value);
        return true;
    case HIPPT_OPT_BVH_LEAF:
        if (value < 1 || value > 15) return false;
        s.bvh.maxLeaf = int(value);
        return true;
    case HIPPT_OPT_BVH_TRAVERSAL_COST:
        if (value < 1 || value > 100000) return false;
        s.bvh.traversalCost = float(value) / 100.0f;
        return true;
    case HIPPT_OPT_BVH_MAX_DEPTH:
        if (value < 1 || value > hippt::kStackDepth) return false;
        s.bvh.maxDepth = int(value);
        return true;
    case HIPPT_OPT_DEVICE_ROWS:
        if (value < 0 || value > 1) return false;
        s.deviceInterleave = value == 1;
        return true;
    case HIPPT_OPT_LEAF_EXIT:
        if (value < -1 || value > 64) return false;
        s.leafExit = int(value);
        return true;
    case HIPPT_OPT_NODE_EXIT:
        if (value < -1 || value > 64) return false;
        s.nodeExit = int(value);
        return true;
    case HIPPT_OPT_BVH_SAH:
        if (value != 0 && value != 1) return false;
        s.bvh.sahMode = int(value);
        return true;
    case HIPPT_OPT_BVH_WIDTH:
        if (value != 0 && value != 2 && value != 4) return false;
        s.bvhWidth = int(value);
        return true;
    case HIPPT_OPT_STACK_CAP:
        if (value != 0 && (value < 4 || value > 30)) return false;
        s.stackCap = int(value);
        return true;
    case HIPPT_OPT_BVH_QUANT:
        if (value < -1 || value > 3) return false;
        s.bvhQuant = int(value);
        return true;
    case HIPPT_OPT_LDS_TOP_NODES:
        if (value < -1 || value > kTopOrderNodes) return false;
        s.ldsTopNodes = int(value);
        return true;
    case HIPPT_OPT_BVH_COLLAPSE:
        if (value < -1 || value > 1) return false;
        s.bvh.collapse = int(value);
        return true;
    case HIPPT_OPT_BVH_NODE_COST:
        if (value < 1 || value > 100000) return false;
        s.bvh.nodeCost = float(value) / 100.0f;
        return true;
    case HIPPT_OPT_BVH_LEAF4:
        if (value < 1 || value > 15) return false;
        s.bvh.maxLeaf4 = int(value);
        return true;
    case HIPPT_OPT_RNG_TABLE:
        if (value != 0 && value != 1) return false;
        s.rngTable = value == 1;
        return true;
    case HIPPT_OPT_PIXEL_FORMAT:
        if (value != HIPPT_PIXEL_ARGB && value != HIPPT_PIXEL_RGBA8) return false;
        s.pixelFormat = int(value);
        return true;
    case HIPPT_OPT_CAMERA_POOL:
        if (value < -1 || value > 1) return false;
        s.cameraPool = int(value);
        return true;
    case HIPPT_OPT_FUSE_COMBINE:
        if (value < -1 || value > 1) return false;
        s.fuseCombine = int(value);
        return true;
    case HIPPT_OPT_ITEM_ORDER:
        if (value < -1 || value > 1) return false;
        s.itemOrder = int(value);
        return true;
    case HIPPT_OPT_WAVEFRONT_SORT:
        if (value != -1 && value != 0 && value != 3 && value != 6) return false;
        s.wfSort = int(value);
        return true;
    case HIPPT_OPT_CHAIN:
        if (value < -1 || value > 16) return false;
        s.chainBatches = int(value);
        return true;
    case HIPPT_OPT_CHAIN_AUDIT:
        if (value != 0 && value != 1) return false;
        s.chainAudit = value == 1;
        return true;
    case HIPPT_OPT_PIXEL_TILE:
        if (value != -1 && value != 0 && value != 8 && value != 16 && value != 32) return false;
        s.pixelTile = int(value);
        return true;
    default: return false;
    }
} catch (const std::exception &e) {
    return false;
} catch (...) {
    return false;
}

extern "C" int hipptActiveBvhWidth(void) try {
    std::lock_guard<std::mutex> g(S().mu);
    return S().activeWidth;
} catch (const std::exception &e) {
    return 0;
} catch (...) {
    return 0;
}

extern "C" long long hipptGetOption(int key) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    switch (key) {
    case HIPPT_OPT_COUNT_TRAVERSAL: return s.countTraversal ? 1 : 0;
    case HIPPT_OPT_WAVE_THRESHOLD: return s.waveThreshold;
    case HIPPT_OPT_SCRATCH_MB: return s.scratchMB;
    case HIPPT_OPT_CHUNK: return s.chunk;
    case HIPPT_OPT_BLOCKS_PER_CU: return s.blocksPerCu;
    case HIPPT_OPT_LDS_SCENE: return s.ldsScene ? 1 : 0;
    case HIPPT_OPT_PATH_MODE: return s.pathMode;
    case HIPPT_OPT_WAVEFRONT_SLOTS: return s.wfSlots;
    case HIPPT_OPT_BVH_LEAF: return s.bvh.maxLeaf;
    case HIPPT_OPT_BVH_TRAVERSAL_COST: return (long long)std::lround(s.bvh.traversalCost * 100.0f);
    case HIPPT_OPT_BVH_MAX_DEPTH: return s.bvh.maxDepth;
    case HIPPT_OPT_DEVICE_ROWS: return s.deviceInterleave ? 1 : 0;
    case HIPPT_OPT_LEAF_EXIT: return s.leafExit;
    case HIPPT_OPT_NODE_EXIT: return s.nodeExit;
    case HIPPT_OPT_BVH_SAH: return s.bvh.sahMode;
    case HIPPT_OPT_BVH_WIDTH: return s.bvhWidth;
    case HIPPT_OPT_STACK_CAP: return s.stackCap;
    case HIPPT_OPT_BVH_QUANT: return s.bvhQuant;
    case HIPPT_OPT_LDS_TOP_NODES: return s.ldsTopNodes;
    case HIPPT_OPT_BVH_COLLAPSE: return s.bvh.collapse;
    case HIPPT_OPT_BVH_NODE_COST: return (long long)std::lround(s.bvh.nodeCost * 100.0f);
    case HIPPT_OPT_BVH_LEAF4: return s.bvh.maxLeaf4;
    case HIPPT_OPT_RNG_TABLE: return s.rngTable ? 1 : 0;
    case HIPPT_OPT_PIXEL_FORMAT: return s.pixelFormat;
    case HIPPT_OPT_CAMERA_POOL: return s.cameraPool;
    case HIPPT_OPT_FUSE_COMBINE: return s.fuseCombine;
    case HIPPT_OPT_ITEM_ORDER: return s.itemOrder;
    case HIPPT_OPT_WAVEFRONT_SORT: return s.wfSort;
    case HIPPT_OPT_CHAIN: return s.chainBatches;
    case HIPPT_OPT_CHAIN_AUDIT: return s.chainAudit ? 1 : 0;
    case HIPPT_OPT_PIXEL_TILE: return s.pixelTile;
    case HIPPT_INFO_LDS_TOP_BYTES: return s.activeTopBytes;
    case HIPPT_INFO_BLOCKS_PER_CU: return s.activeBlocksPerCu;
    case HIPPT_INFO_CHUNK: return s.activeChunk;
    case HIPPT_INFO_CHAIN_CAP: return s.activeChainCap;
    default: return -1;
    }
} catch (const std::exception &e) {
    return -1;
} catch (...) {
    return -1;
}

extern "C" int hipptChainAudit(unsigned int *words, int maxWords) try {
    std::lock_guard<std::mutex> g(S().mu);
    State &s = S();
    const char *e = nullptr;
    if (s.ready && !sync_locked(&e)) return -1;  // closes the open runs (their final flushes) first
    size_t n = 0;
    while (n < s.auditWords.size()) {
        const size_t recs = std::min(s.auditWords[n + 8], hippt::kAuditBatches) + 1u;
        const size_t len = (1 + recs) * hippt::kAuditWords;
        if (n + len > size_t(std::max(0, maxWords))) break;
        n += len;
    }
    if (words && n) std::memcpy(words, s.auditWords.data(), n * sizeof(unsigned));
    s.auditWords.erase(s.auditWords.begin(), s.auditWords.begin() + long(n));
    return int(n);
} catch (const std::exception &e) {
    return -1;
} catch (...) {
    return -1;
}

extern "C" const char *hipptLastError(void) { return S().error; }

// ---- host BVH builder -----------------------------------------------------------------------------
extern "C" hipptBvh *hipptBvhBuild(const float *verts, int numTris, float extentHint, const char **err) try {
    std::unique_ptr<hipptBvh> b(new hipptBvh());
    std::string msg;
    hippt::BvhParams params;
    {
        std::lock_guard<std::mutex> g(S().mu);
        params = S().bvh;  // the build options an upload would use
    }
    if (!verts || !hippt::build_bvh(verts, numTris, extentHint, b->bvh, msg, params)) {
        std::lock_guard<std::mutex> g(S().mu);
        fail(err, msg.empty() ? "null vertex pointer" : msg);
        return nullptr;
    }
    hippt::collapse_bvh4(b->bvh, b->bvh4, params);
    hippt::order_bvh4_top(b->bvh4, kTopOrderNodes);
    (void)hippt::quantize_bvh4(b->bvh4, b->bvh4q);  // empty for boxes near +-FLT_MAX
    return b.release();
} catch (const std::exception &e) {
    return (fail_free(err, e.what()), nullptr);
} catch (...) {
    return (fail_free(err, "unknown exception"), nullptr);
}

extern "C" int hipptBvhNodeCount(const hipptBvh *b) { return b ? int(b->bvh.nodes.size() / hippt::kNodeWords) : 0; }
extern "C" int hipptBvhDepth(const hipptBvh *b) { return b ? b->bvh.levels : 0; }
extern "C" void hipptBvhCopy(const hipptBvh *b, uint32_t *nodes, int *triOrder) try {
    if (!b) return;
    if (nodes) std::memcpy(nodes, b->bvh.nodes.data(), b->bvh.nodes.size() * sizeof(uint32_t));
    if (triOrder) std::memcpy(triOrder, b->bvh.order.data(), b->bvh.order.size() * sizeof(int));
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}
extern "C" void hipptBvhFree(hipptBvh *b) { delete b; }
extern "C" int hipptBvh4NodeCount(const hipptBvh *b) try {
    return b ? int(b->bvh4.nodes.size() / hippt::kNode4Words) : 0;
} catch (const std::exception &e) {
    return 0;
} catch (...) {
    return 0;
}
extern "C" int hipptBvh4Depth(const hipptBvh *b) { return b ? b->bvh4.levels : 0; }
extern "C" int hipptBvh4StackBound(const hipptBvh *b) { return b ? b->bvh4.stackBound : 0; }
extern "C" void hipptBvh4Copy(const hipptBvh *b, uint32_t *nodes) try {
    if (b && nodes) std::memcpy(nodes, b->bvh4.nodes.data(), b->bvh4.nodes.size() * sizeof(uint32_t));
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}
extern "C" int hipptBvh4QNodeCount(const hipptBvh *b) try {
    return b ? int(b->bvh4q.size() / hippt::kNode4QWords) : 0;
} catch (const std::exception &e) {
    return 0;
} catch (...) {
    return 0;
}
extern "C" void hipptBvh4QCopy(const hipptBvh *b, uint32_t *nodes) try {
    if (b && nodes) std::memcpy(nodes, b->bvh4q.data(), b->bvh4q.size() * sizeof(uint32_t));
} catch (...) {
    // an exception must not cross the C ABI (the caller is C or Qt code)
}
