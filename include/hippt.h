/*
 * hippt.h — C ABI of libhippt.so, the MI355X-native (gfx950) path-tracing backend.
 *
 * Drop-in boundary.  The first three entry points are EXACTLY the reference's
 * CUDA backend ABI, so CudaPathTracer.cpp links unchanged with
 * ENABLE_CUDA_BACKEND defined:
 *
 *   cudaPathTracerInit      replaces CudaPathTracerKernel.cu:188-237  (declared CudaPathTracer.cpp:5)
 *   cudaPathTracerRender    replaces CudaPathTracerKernel.cu:239-276  (declared CudaPathTracer.cpp:6)
 *   cudaPathTracerShutdown  replaces CudaPathTracerKernel.cu:278-288  (declared CudaPathTracer.cpp:7)
 *
 * Semantics kept from the reference: Init frees previous buffers and may be called
 * repeatedly (RayTracerFboItem.cpp:520-521 re-inits on frame 0); Render renders ONE
 * sample per pixel for the caller-supplied frameIndex (running average,
 * CudaPathTracerKernel.cu:157-169), blocks until the frame is on the host and returns
 * a library-owned W*H ARGB array (row 0 = v = 0) valid until the next Init/Shutdown;
 * errors are `false` + a library-owned message (null out-pointers allowed); Shutdown is
 * idempotent.  Unlike the reference, every entry point is serialised by an internal
 * mutex (the reference is called from two Qt threads without a lock).
 *
 * The default scene is the reference kernel's built-in 4-sphere scene
 * (CudaPathTracerKernel.cu:113-116).  The hippt* extensions add triangle-mesh scenes
 * (host SAH BVH build + upload), batched multi-sample rendering, multi-GPU row bands,
 * and counters.  The GL-backend shape (GpuPathTracer.h:9-38: renderFrame(spp, depth),
 * resetAccumulation) maps onto hipptRenderFrames / hipptResetAccumulation.
 *
 * No torch types, no HIP types: plain pointers and sizes.
 */
#ifndef HIPPT_H
#define HIPPT_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference ABI (CudaPathTracer.cpp:4-8) ---------------------------------- */
bool cudaPathTracerInit(int width, int height, const char **errorMessage);
bool cudaPathTracerRender(int frameIndex, int maxDepth, const unsigned int **hostPixels,
                          const char **errorMessage);
void cudaPathTracerShutdown(void);

/* Same functions under backend-neutral names. */
bool hipPathTracerInit(int width, int height, const char **errorMessage);
bool hipPathTracerRender(int frameIndex, int maxDepth, const unsigned int **hostPixels,
                         const char **errorMessage);
void hipPathTracerShutdown(void);

/* ---- scene description ---------------------------------------------------------- */
/* Camera as the kernels consume it: RayTracer.h Camera (:545-561) computed in FP64 and
 * stored FP32.  Layout is part of the ABI (80 bytes). */
typedef struct hipptCamera {
    float origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
    float lens_radius;
    float reserved;
} hipptCamera;

/* Builds a camera exactly like RayTracer.h Camera::Camera (:545-561). */
void hipptBuildCamera(const double lookfrom[3], const double lookat[3], const double vup[3], double vfovDeg,
                      double aspect, double aperture, double focusDist, hipptCamera *out);

enum { HIPPT_SCENE_SPHERE4 = 0, HIPPT_SCENE_MESH = 1 };

/* Selects the reference built-in 4-sphere scene (the default). */
bool hipptUseBuiltinScene(int sceneId, const char **errorMessage);

/* Triangle mesh: verts = numTris*9 floats (v0,v1,v2), triMaterial = numTris ints in
 * [0,numMaterials), albedo = numMaterials*3 floats (Lambertian, RayTracer.h:473-488).
 * Builds a binned-SAH BVH on the host and uploads it to every device on the next render.
 * The camera is given by RayTracer.h Camera parameters; the aspect ratio is width/height
 * of the current Init (as RayTracerFboItem.cpp:49-56 does). */
bool hipptUploadMesh(const float *verts, const int *triMaterial, int numTris, const float *albedo,
                     int numMaterials, const double lookfrom[3], const double lookat[3], const double vup[3],
                     double vfovDeg, double aperture, double focusDist, const char **errorMessage);

/* Materials of RayTracer.h :473-540.  LAMBERTIAN uses albedo; METAL albedo and fuzz (clamped
 * to <= 1 as Metal's constructor does, :494); DIELECTRIC the index of refraction ir. */
enum { HIPPT_MAT_LAMBERTIAN = 0, HIPPT_MAT_METAL = 1, HIPPT_MAT_DIELECTRIC = 2 };
typedef struct {
    int kind;
    float albedo[3];
    float fuzz;
    float ir;
} hipptMaterial;

/* General scene: triangles (as hipptUploadMesh) plus spheres = numSpheres*4 floats (center
 * xyz, radius; Sphere, RayTracer.h:274-322), each primitive with a material index into
 * materials[numMaterials].  Either count may be 0, not both.  Ties of the closest hit are
 * broken by primitive id: triangles 0..numTris-1, then spheres.  The reference app's scene
 * (random_scene(), RayTracer.h:599-643, which draws from a nondeterministic RNG) is uploaded
 * as its sphere list. */
bool hipptUploadScene(const float *verts, const int *triMaterial, int numTris, const float *spheres,
                      const int *sphereMaterial, int numSpheres, const hipptMaterial *materials, int numMaterials,
                      const double lookfrom[3], const double lookat[3], const double vup[3], double vfovDeg,
                      double aperture, double focusDist, const char **errorMessage);

/* Triangle mesh read from a Wavefront OBJ or PLY file (the reference has no mesh input):
 * verts = numTris*9 floats (polygons fan-triangulated), triGroup = numTris ints in
 * [0, numGroups): OBJ `usemtl` groups in order of first use (groupNames[g]; "" = faces before
 * any usemtl), PLY: 0.  Feed verts/triGroup to hipptUploadMesh/hipptUploadScene with one
 * material per group.  Library-owned; release with hipptFreeMesh. */
typedef struct {
    float *verts;
    int *triGroup;
    int numTris;
    int numGroups;
    const char *const *groupNames;
    void *owner_;
} hipptMesh;
bool hipptReadMesh(const char *path, hipptMesh *out, const char **errorMessage);
void hipptFreeMesh(hipptMesh *mesh);

/* Optional: replace the camera by a prebuilt one (used as-is, whatever the aspect). */
bool hipptSetCamera(const hipptCamera *camera, const char **errorMessage);

/* ---- devices and row bands ------------------------------------------------------- */
int hipptDeviceCount(void);
/* Render on these devices (one context per device, contiguous row bands); takes effect
 * at the next Init.  Default: the current HIP device only. */
bool hipptSetDevices(const int *deviceIds, int numDevices, const char **errorMessage);
/* Restrict this process to rows [y0, y1) of the image (one-process-per-GPU launch);
 * y1 <= 0 means "to the last row".  Takes effect at the next Init. */
bool hipptSetRowRange(int y0, int y1, const char **errorMessage);
/* Alternative: this process renders rows phase, phase+stride, phase+2*stride, ... (one process
 * per GPU with phase = rank, stride = world size balances the load: row bands of a scene differ
 * by up to 1.6x in cost).  Clears a row range; hipptSetRowRange clears the interleave.  Takes
 * effect at the next Init.  The image is bit-identical for any split. */
bool hipptSetRowInterleave(int phase, int stride, const char **errorMessage);

/* ---- rendering ------------------------------------------------------------------- */
/* Renders `count` samples per pixel as frames firstFrame..firstFrame+count-1; the
 * accumulation buffer ends exactly as after `count` single-frame Render calls.  Blocks
 * until the image is on the host (hostPixels may be null to skip the copy). */
bool hipptRenderFrames(int firstFrame, int count, int maxDepth, const unsigned int **hostPixels,
                       const char **errorMessage);
/* Enqueues the same work without waiting and without a device-to-host copy. */
bool hipptRenderFramesAsync(int firstFrame, int count, int maxDepth, const char **errorMessage);
bool hipptSynchronize(const char **errorMessage);
/* Interactive hand-off (replaces the blocking full-frame copy of CudaPathTracerKernel.cu:261-265
 * for hosts that can show the previous image): enqueues the frames, whose ARGB image lands in one
 * of two library-owned pinned frames (written by the kernel that produces it, or copied after
 * it), and returns without waiting. */
bool hipptRenderFramesPresent(int firstFrame, int count, int maxDepth, const char **errorMessage);
/* Never blocks: *hostPixels = the newest presented image whose transfer has completed (null if
 * none yet), *frames = the frame count accumulated in it.  The image stays valid until the
 * second hipptRenderFramesPresent call after the one that produced it (double buffering). */
bool hipptLatestFrame(const unsigned int **hostPixels, int *frames, const char **errorMessage);
/* Copies the current image (ARGB, W*H) and/or accumulation buffer (RGBA float, W*H*4)
 * of the process's row range into caller memory; rows outside the range are untouched. */
bool hipptReadback(unsigned int *pixels, float *accum, const char **errorMessage);
/* Zeroes the accumulation buffer (GpuPathTracer::resetAccumulation, GpuPathTracer.cpp:85-95). */
bool hipptResetAccumulation(const char **errorMessage);

/* ---- counters and options ---------------------------------------------------------- */
typedef struct hipptStats {
    unsigned long long segments;      /* closest-hit queries traced (rays x bounces) */
    unsigned long long pixelSamples;  /* pixel samples rendered */
    unsigned long long nodeVisits;    /* BVH interior nodes visited (HIPPT_OPT_COUNT_TRAVERSAL) */
    unsigned long long triTests;      /* ray-triangle tests (HIPPT_OPT_COUNT_TRAVERSAL) */
    double traceMs;                   /* summed device time of the path-trace kernel launches */
    double combineMs;                 /* summed device time of the accumulate kernel launches */
    int traceLaunches;
    int combineLaunches;
    int bvhNodes;                     /* scene info */
    int bvhDepth;
    int numTris;
    int numDevices;
} hipptStats;

bool hipptGetStats(hipptStats *out);
void hipptResetStats(void);
/* Raw device counters (profiling): [0] segments, [1] pixel samples, [2] node visits,
 * [3] triangle tests, [4 + 2k] / [5 + 2k] wave-level / lane-level passes of mesh-kernel
 * phase k (HIPPT_OPT_COUNT_TRAVERSAL builds only): 0 outer loop, 1 camera ray, 2 traversal
 * round, 3 interior node, 4 leaf, 5 triangle, 6 shading, 7 unit-sphere rejection.
 * Returns the number of words written (<= n, <= 32). */
int hipptGetCounters(unsigned long long *out, int n);

enum {
    HIPPT_OPT_COUNT_TRAVERSAL = 1,  /* 1: count node visits / triangle tests (slower) */
    HIPPT_OPT_WAVE_THRESHOLD = 2,   /* lanes still traversing below which a wave goes to shade; -1 (default):
                                       24 for LDS-resident scenes and spheres / Metal / Dielectric over trees
                                       in global memory, 40 for Lambertian scenes over trees in global memory
                                       (32 before round 6) */
    HIPPT_OPT_SCRATCH_MB = 3,       /* cap of the per-batch sample scratch per device (32768: one batch for 4K x 256 spp) */
    HIPPT_OPT_CHUNK = 4,            /* work items a wave takes from the global queue at once (64..2^20, a
                                       multiple of 64); 0 (default): automatic, 512 for chained or
                                       whole-image (>= 2^26 samples) batches of the Lambertian megakernel,
                                       else 256 */
    HIPPT_OPT_BLOCKS_PER_CU = 5,    /* persistent-grid residency (0 = occupancy query) */
    HIPPT_OPT_LDS_SCENE = 6,        /* 1 (default): small scenes are copied into LDS per block */
    HIPPT_OPT_PATH_MODE = 8,        /* 0 (default): persistent megakernel; 1: wavefront kernels */
    HIPPT_OPT_WAVEFRONT_SLOTS = 9,  /* wavefront path-state slots per device, 64..2^28 (default 2^27) */
    HIPPT_OPT_BVH_LEAF = 10,        /* max primitives per BVH leaf, 1..15 (default 2); applies at the next upload */
    HIPPT_OPT_BVH_TRAVERSAL_COST = 11, /* SAH node-step cost in 1/100 primitive tests; next upload */
    HIPPT_OPT_BVH_MAX_DEPTH = 12,   /* interior-level bound (LDS stack per lane), 1..32; next upload */
    HIPPT_OPT_DEVICE_ROWS = 13,     /* hipptSetDevices split: 1 (default) interleaved rows, 0 bands; next Init */
    HIPPT_OPT_LEAF_EXIT = 14        /* node loop yields to the leaf loop once <= this many lanes lack a
                                       leaf; -1 (default): automatic (LDS scenes 12, 4 for the general kernel
                                       and the wavefront; trees in global memory 12 for the general kernel,
                                       22 for Lambertian scenes (17 before round 6)) */
    , HIPPT_OPT_NODE_EXIT = 15      /* leaf loop yields to the node loop once <= this many lanes hold a leaf
                                       (0 = never); -1 (default): LDS scenes 8; trees in global memory 16 for
                                       the general kernel, 56 for Lambertian scenes (48 before round 6) */
    , HIPPT_OPT_BVH_SAH = 16        /* BVH split search: 1 (default) all axes, exact sweep SAH (32 bins on
                                       nodes over 65536 primitives); 0: 16 bins on the longest axis; next upload */
    , HIPPT_OPT_BVH_WIDTH = 17      /* traversal over the 4-wide (4) or 2-wide (2) BVH (megakernel and wavefront);
                                       0 (default): 4-wide */
    , HIPPT_OPT_STACK_CAP = 18      /* 4-wide traversal: LDS stack entries per lane, 4..30 (deeper stacks spill
                                       to global memory); 0 (default): the tree's bound, at most 19 (30 for
                                       LDS scenes; 13 for a megakernel over a tree in global memory
                                       whose bound exceeds 19, the rest of the LDS holding the top
                                       of the tree) */
    , HIPPT_OPT_BVH_QUANT = 19      /* 4-wide traversal of global-memory trees over 64-byte nodes with 8-bit
                                       child boxes (1) or 128-byte float nodes (0); 2: float top in LDS,
                                       8-bit nodes below (megakernel); 3: 128-byte nodes of half-precision
                                       planes, 4 reads per visit (megakernel and wavefront); -1 (default): 8-bit for
                                       the wavefront path's Lambertian-triangle scenes, else float */
    , HIPPT_OPT_LDS_TOP_NODES = 20  /* 4-wide traversal of global-memory trees: the top of the tree (this many
                                       nodes, breadth-first) is copied into every block's LDS and read from
                                       there; 0: none; -1 (default): automatic (what the LDS budget of the
                                       resident blocks leaves beside the stack) */
    , HIPPT_OPT_BVH_COLLAPSE = 21   /* 2-wide -> 4-wide collapse: 0 greedy (open the largest child), 1 SAH-optimal
                                       (dynamic programming), -1 (default) SAH-optimal for scenes that fit
                                       the LDS scene copy, else greedy; next upload (hipptBvhBuild: -1 =
                                       greedy) */
    , HIPPT_OPT_BVH_NODE_COST = 22  /* SAH-optimal collapse: a 4-wide node visit in 1/100 primitive tests; next upload */
    , HIPPT_OPT_BVH_LEAF4 = 23      /* SAH-optimal collapse: most primitives per 4-wide leaf, 1..15; next upload */
    , HIPPT_OPT_RNG_TABLE = 24      /* 1: random_in_unit_sphere's rejection loop as one lookup in a 16 GiB
                                       per-device table of its outcome for every 32-bit RNG state (built on
                                       first use); 0 (default): the loop.  Same results either way */
    , HIPPT_OPT_PIXEL_FORMAT = 25   /* output frame words of the hipptRenderFrames* calls: HIPPT_PIXEL_ARGB
                                       (default, the CUDA backend's) or HIPPT_PIXEL_RGBA8 (the GL / Vulkan
                                       backends'); cudaPathTracerRender always writes ARGB */
    , HIPPT_OPT_CAMERA_POOL = 26    /* megakernel over a 4-wide float-node tree: each wave generates the camera
                                       rays of its next 64 samples with all lanes at once into an LDS pool
                                       instead of one by one as paths end (1), or not (0); -1 (default):
                                       automatic (on except for the general kernel over a tree in global
                                       memory).  Same results either way */
    , HIPPT_OPT_FUSE_COMBINE = 27   /* megakernel: a batch's running average + tonemap runs inside the next
                                       batch's launch on the same device (beside its paths) instead of as a
                                       launch of its own, whenever nothing reads the image in between (1), or
                                       never (0); -1 (default): automatic.  Same results either way */
    , HIPPT_OPT_ITEM_ORDER = 28     /* megakernel: the work queues hand out runs of 64 pixels in order of an
                                       estimated sample length (camera rays and a few bounce directions on
                                       the host's tree), longest first, so that a wave's lanes hold samples
                                       of similar length (1), or in image order (0); -1 (default): automatic
                                       (on).  Same results either way */
    , HIPPT_OPT_WAVEFRONT_SORT = 29 /* wavefront: the shade kernel appends each block's scattered paths sorted by
                                       direction octant (3) or octant and a 2x2x2 cell of the scene box (6),
                                       so that a wave of the extend kernel traces rays of one kind; 0: in
                                       thread order; -1 (default): automatic (0).  Same results either way */
    , HIPPT_OPT_CHAIN = 30          /* megakernel, camera-pool kernels over 4-wide float nodes: asynchronous
                                       batches with the same scene, camera, rows and frames per batch (each
                                       the same frames again or the next ones) form a run, and a launch whose
                                       batch is drained goes on with the batches posted behind it, up to this
                                       many (1..16), so that the run pays the launch's tail once per that many
                                       batches; the next launch combines them beside its own paths and the
                                       image's readers flush the rest.  0: one launch per batch; -1
                                       (default): automatic (on; 8 batches for batches of more than 2^26
                                       samples, else 2..16 by the batch's size, at most 8 over LDS-resident
                                       scenes).  Same results either way */
    , HIPPT_OPT_CHAIN_AUDIT = 31    /* 1: chained launches record, per batch of each run, the work items they
                                       traced (count and a hash of their indices), the frames and the launch
                                       they traced them with, and the pixels, frames and launch of the batch's
                                       combine; read with hipptChainAudit.  0 (default): off.  Takes effect at
                                       the next run.  Same images either way (a testing aid) */
    , HIPPT_OPT_PIXEL_TILE = 32     /* the item order's (HIPPT_OPT_ITEM_ORDER) unit of 64 pixels: tiles of this
                                       many columns x 64 / it band rows (8, 16 or 32; the image width a
                                       multiple of it), or 64 consecutive pixels of a row (0); -1 (default):
                                       automatic (8 for a band of consecutive rows, 0 for interleaved row
                                       shares).  Same results either way */
};
/* Records of the chained runs closed since the last call (HIPPT_OPT_CHAIN_AUDIT), as 32-bit words:
 * per run a 16-word header  [0] 0xC4A1D17 [1] run id [2] device [3] batch 0's first frame [4] frames
 * from one batch to the next (-1: one batch) [5] frames per batch [6] band pixels [7] items per batch
 * [8] batches [9] launches [10] slots [11] batches beyond the records (their records pooled in the
 * last one) [12..15] 0, then min(batches, 256) + 1 records of 16 words: [0] items traced [1] pixels
 * combined [2..3] sum of hash(item) [4..5] sum of hash(pixel) over the combine (64-bit, mod 2^64;
 * hash(i) = the RNG hash of i ^ 0x5bd1e995) [6] 1 + largest first frame an item was traced with
 * [7] ~smallest [8] 1 + latest launch that traced items [9] ~earliest [10] 1 + latest launch that
 * combined pixels (the run's last flush is launch `launches`) [11] ~earliest [12] 1 + largest first
 * frame the combine used [13] ~smallest [14..15] 0.  Writes at most maxWords words (whole runs) and
 * returns the number written; runs that did not fit are kept for the next call.  Synchronises. */
int hipptChainAudit(unsigned int *words, int maxWords);
/* Output frame word formats (HIPPT_OPT_PIXEL_FORMAT).  Both map an accumulated colour c to
 * sqrt(clamp(c, 0, 1)) per channel.
 *   ARGB:  0xAARRGGBB, channel = uint(x * 255) truncated (CudaPathTracerKernel.cu:171-178).
 *   RGBA8: bytes R, G, B, A in memory (0xAABBGGRR), channel = x * 255 rounded to nearest, ties to
 *          even: the RGBA8 UNORM texel the GL (GpuPathTracer.cpp:284-285, GL_RGBA8 image) and
 *          Vulkan (pathtrace_vulkan.comp:113-114, VK_FORMAT_R8G8B8A8_UNORM, copied to
 *          VulkanPathTracer::hostPixels) backends store. */
enum { HIPPT_PIXEL_ARGB = 0, HIPPT_PIXEL_RGBA8 = 1 };
/* Read-only (hipptGetOption) facts of the last megakernel render: LDS bytes of the top of the tree,
 * persistent-grid blocks per CU, work items per claim (HIPPT_OPT_CHUNK as applied), batches a launch
 * may trace (HIPPT_OPT_CHAIN as applied: 0 = the batch was not chained). */
enum { HIPPT_INFO_LDS_TOP_BYTES = 100, HIPPT_INFO_BLOCKS_PER_CU = 101, HIPPT_INFO_CHUNK = 102,
       HIPPT_INFO_CHAIN_CAP = 103 };
bool hipptSetOption(int key, long long value);
long long hipptGetOption(int key);
/* BVH width (2 or 4) the last mesh render traversed (0 before any): what nodeVisits count. */
int hipptActiveBvhWidth(void);

const char *hipptLastError(void);

/* ---- host BVH builder (exposed for C++ hosts and tests) ------------------------------- */
/* Node = 16 x 32-bit words: child-0 box (lo xyz, hi xyz), child-1 box, child0, child1,
 * 2 reserved.  child >= 0: interior node index; child < 0: leaf, ~child = first<<4 | count. */
typedef struct hipptBvh hipptBvh;
hipptBvh *hipptBvhBuild(const float *verts, int numTris, float extentHint, const char **errorMessage);
int hipptBvhNodeCount(const hipptBvh *bvh);
int hipptBvhDepth(const hipptBvh *bvh);
/* nodes: NodeCount*16 words; triOrder: numTris ints (leaf order -> original triangle index). */
void hipptBvhCopy(const hipptBvh *bvh, uint32_t *nodes, int *triOrder);
void hipptBvhFree(hipptBvh *bvh);
/* The 4-wide tree the megakernel traverses (HIPPT_OPT_BVH_WIDTH 4), collapsed from the 2-wide
 * one (same leaves and triangle order).  Node = 32 words: lo.x[4] hi.x[4] lo.y[4] hi.y[4]
 * lo.z[4] hi.z[4] (floats), child[4] (codes as above; an unused slot holds an empty leaf under
 * a box far outside the scene), 4 reserved.  Depth = nodes on the deepest path; StackBound =
 * the most traversal-stack entries any ray can need. */
int hipptBvh4NodeCount(const hipptBvh *bvh);
int hipptBvh4Depth(const hipptBvh *bvh);
int hipptBvh4StackBound(const hipptBvh *bvh);
void hipptBvh4Copy(const hipptBvh *bvh, uint32_t *nodes);
/* The same 4-wide tree with 8-bit child boxes (HIPPT_OPT_BVH_QUANT), Bvh4NodeCount nodes of 16
 * words: origin xyz (float), scale x; lo.x hi.x lo.y hi.y lo.z hi.z (4 bytes each, byte i =
 * child i, plane = origin + byte * scale); scale y; scale z; child[4].  Every decoded box
 * contains the float box of hipptBvh4Copy; an unused slot has lo bytes 255 and hi bytes 0. */
void hipptBvh4QCopy(const hipptBvh *bvh, uint32_t *nodes);
/* Nodes of that 8-bit tree: Bvh4NodeCount, or 0 when the scene has none (boxes near +-FLT_MAX,
 * which no finite grid covers; the kernels then read the float nodes). */
int hipptBvh4QNodeCount(const hipptBvh *bvh);

#ifdef __cplusplus
}
#endif
#endif
