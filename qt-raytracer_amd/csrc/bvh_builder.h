// bvh_builder.h — host-side binned-SAH BVH builder for the HIP megakernel.
//
// Replaces the reference's BVHNode constructor (RayTracer.h:393-429: random split axis,
// full sort, median split, pointer tree of shared_ptr<Hitable>) with a flat,
// GPU-traversable layout.  Only the closest-hit RESULT must match the reference; the
// tree shape is free.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace hippt {

// Stack entries the kernel keeps per lane in LDS; the builder guarantees that no
// traversal needs more (interior levels <= kStackDepth).
constexpr int kStackDepth = 32;
// Default leaf size: 2 primitives (r3ag, alternating A/B on the final kernels: blob70k +1.3%, Cornell
// +1.1%, random_scene +0.3%, cornell_mixed +0.2% over 4; the 4-wide collapse leaves visit and test
// counts nearly unchanged, the leaf loop's per-lane trip counts less uneven).
constexpr int kMaxLeafTris = 2;
constexpr int kNodeWords = 16;  // 64 B: two child boxes + two child codes

// Build parameters: SAH with a traversal step costing `traversalCost` primitive tests, leaves of
// at most `maxLeaf` (<= 15, the leaf code's count field) primitives.
// maxDepth bounds the interior levels (= the kernel's LDS stack entries per lane, so it sets
// the occupancy of deep scenes); below the bound the split is SAH, near it object median.
struct BvhParams {
    int maxLeaf = kMaxLeafTris;
    float traversalCost = 1.0f;
    int maxDepth = kStackDepth;
    int sahMode = 1;  // 0: 16 bins on the longest centroid axis; 1: all axes, exact sweep (32 bins on big nodes)
    // 4-wide collapse: 0 opens the largest-area interior child until a node has 4 children; 1 the
    // SAH-optimal collapse (nodeCost = a 4-wide node visit in primitive tests; leaves may merge
    // 2-wide subtrees up to maxLeaf4 primitives); -1 automatic: the scene upload takes the
    // SAH-optimal tree when the scene fits the LDS scene copy, else greedy (collapse_bvh4 itself
    // treats -1 as greedy)
    int collapse = -1;
    float nodeCost = 2.0f;
    int maxLeaf4 = 4;
};

struct Bvh {
    std::vector<uint32_t> nodes;  // kNodeWords per interior node; node 0 is the root
    std::vector<int> order;       // leaf order -> original primitive index
    int levels = 0;               // interior levels on the deepest path (= max stack use)
    int leaves = 0;
};

// verts: numTris * 9 floats.  extentHint: largest |coordinate| any ray origin can have
// (camera position); boxes are padded by max(|coord|, extentHint) * 2^-16 so the
// kernel's FMA slab test is conservative.
bool build_bvh(const float *verts, int numTris, float extentHint, Bvh &out, std::string &err,
               const BvhParams &params = BvhParams());
// General primitives: boxes = numPrims * 6 floats (lo xyz, hi xyz); `order` maps leaf order
// to the primitive index.
bool build_bvh_boxes(const float *boxes, int numPrims, float extentHint, Bvh &out, std::string &err,
                     const BvhParams &params = BvhParams());

inline int32_t leaf_code(int first, int count) { return ~((first << 4) | count); }

// 4-wide BVH collapsed from a 2-wide one (same leaves, so the same primitive order): each
// node opens the interior child of largest surface area until it has 4 children.  128-byte
// nodes, children in SoA: lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4] code[4] pad[4];
// an unused slot holds an empty leaf under a box far outside the scene.
constexpr int kNode4Words = 32;
struct Bvh4 {
    std::vector<uint32_t> nodes;  // kNode4Words per node; node 0 is the root
    int levels = 0;               // nodes on the deepest root-to-leaf path
    int stackBound = 0;           // most entries a traversal stack can hold: max over nodes of
                                  // the (children - 1) pushes of it and its ancestors
};
void collapse_bvh4(const Bvh &bvh2, Bvh4 &out, const BvhParams &params = BvhParams());

// Renumbers the nodes so that the first `topNodes` are the tree's top in breadth-first order
// (node k's children come after it; any prefix of them is the shallowest nodes), the others
// following in their previous order.  The kernels copy such a prefix into LDS for trees read from
// global memory.  Returns the number of nodes ordered breadth-first.
int order_bvh4_top(Bvh4 &b, int topNodes);

// The 4-wide tree with 8-bit child boxes (Ylitie et al. 2017, "Efficient incoherent ray traversal
// on GPUs through compressed wide BVHs", reduced to 4 children): 64-byte nodes, same node
// indices, child codes and primitive order as Bvh4.  Words:
//   0-2  grid origin o (float xyz)           3   scale s.x (a power of two)
//   4-9  lo.x hi.x lo.y hi.y lo.z hi.z: byte i = child i's plane q, plane = o + q*s
//   10   scale s.y   11  scale s.z           12-15 child codes
// Planes are rounded outward (lo down, hi up), so every decoded box contains the Bvh4 box (which
// is already padded for the kernel's slab-test rounding).  An unused child slot has lo = 255,
// hi = 0 on every axis: read as near/far planes by the ray's octant it is always missed.
// Returns false (and leaves `out` empty) for trees with boxes near +-FLT_MAX, which no finite
// grid covers: such scenes have no 8-bit tree.
constexpr int kNode4QWords = 16;
bool quantize_bvh4(const Bvh4 &in, std::vector<uint32_t> &out);

// Hybrid device layout of a 4-wide tree (the megakernel over trees in global memory, with the top
// of the tree in LDS): nodes 0..topNodes-1 (the breadth-first top, order_bvh4_top) as 128-byte
// float nodes (Bvh4 words) at byte k*128, every other node k as its 64-byte 8-bit node (the
// quantize_bvh4 words `q` of the same tree) at byte topNodes*128 + (k - topNodes)*64.  Interior
// child codes become those BYTE offsets (a code below topNodes*128 is a float node), leaf codes
// stay.  The top's children may be 8-bit nodes; a bottom node's children are always bottom nodes
// (the breadth-first prefix holds every ancestor of its nodes).  `b` and `q` carry node-index
// codes.  Returns false if q is empty (no 8-bit tree) or topNodes is out of range.
bool hybrid_bvh4(const Bvh4 &b, const std::vector<uint32_t> &q, int topNodes, std::vector<uint32_t> &out);

// The 4-wide tree with IEEE half-precision child planes (HIPPT_OPT_BVH_QUANT 3), re-encoded in
// place of each 128-byte Bvh4 node (same node size, so the same node indices, byte offsets and
// child codes).  Each axis a has two 16-byte rows of halves at byte 32a: [lo[4] hi[4]] for rays
// with a positive direction on a, then [hi[4] lo[4]] for negative ones, so the octant's near and
// far planes are ONE aligned 16-byte read at the float node's near-row address (near planes in its
// words 0-1, far planes in words 2-3).  Bytes 96-111 the child codes (Bvh4 words 24-27), 112-127
// zero.  Planes are rounded outward (lo down, hi up; only the empty slots' infinite planes stay infinite), so
// every box contains the Bvh4 box and a kernel's slab test of it (v_fma_mix_f32: the half enters
// the FMA exactly) is the float node's test of a larger box.
// `in` is kNode4Words per node, in any code convention (the code words are copied).  Returns false
// (and leaves `out` empty) when a finite lo plane lies below -65504 or a finite hi plane above
// 65504: its half would be infinite, a box every ray enters; such scenes keep float nodes.
bool half_bvh4(const uint32_t *in, size_t numNodes, std::vector<uint32_t> &out);
uint16_t half_round_down(float x);  // the largest half <= x (x not NaN)
uint16_t half_round_up(float x);    // the smallest half >= x
float half_value(uint16_t h);

}  // namespace hippt
