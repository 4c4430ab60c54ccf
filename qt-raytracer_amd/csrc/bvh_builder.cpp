// bvh_builder.cpp — binned SAH builder producing the 64-byte two-box node layout read
// by hippt_kernels.hip.  See bvh_builder.h.
#include "bvh_builder.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace hippt {
namespace {

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float *l, const float *h) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], l[a]);
            hi[a] = std::max(hi[a], h[a]);
        }
    }
    void grow(const Box &b) { grow(b.lo, b.hi); }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

struct Prim {
    float lo[3], hi[3], c[3];
    int id;
};

constexpr int kMaxBins = 32;
constexpr int kSweepMax = 1 << 16;  // exact sweep SAH up to this many primitives per node

// Centroid order on one axis, ties by primitive id (a total order: deterministic splits).
struct by_centroid {
    int axis;
    bool operator()(const Prim &p, const Prim &q) const {
        return p.c[axis] < q.c[axis] || (p.c[axis] == q.c[axis] && p.id < q.id);
    }
};

int ceil_log2(long long v) {
    int r = 0;
    while ((1LL << r) < v) ++r;
    return r;
}

class Builder {
public:
    Builder(std::vector<Prim> &p, float pad, const BvhParams &params) : prims_(p), pad_(pad), par_(params) {}

    // Returns the child code for prims [b, e): interior node index or leaf code.
    int32_t build(int b, int e, int level, Box &bounds) {
        bounds = Box();
        Box cb;
        for (int i = b; i < e; ++i) {
            bounds.grow(prims_[i].lo, prims_[i].hi);
            cb.grow(prims_[i].c, prims_[i].c);
        }
        const int n = e - b;
        int axis = 0;
        float ext[3];
        for (int a = 0; a < 3; ++a) ext[a] = cb.hi[a] - cb.lo[a];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;

        int mid = -1;
        if (n <= 1) {
            mid = -1;
        } else if (level + 1 + ceil_log2((n + par_.maxLeaf - 1) / par_.maxLeaf) >= par_.maxDepth) {
            // depth guard: from here object-median halving bounds the remaining levels
            mid = n <= par_.maxLeaf ? -1 : median_split(b, e, axis);
        } else if (ext[axis] <= 0.0f) {
            mid = n > par_.maxLeaf ? b + n / 2 : -1;  // coincident centroids: split by index
        } else if (par_.sahMode == 0) {
            float best_cost;
            int best_bin;
            sah(b, e, axis, cb, best_cost, best_bin, 16);
            if (n <= par_.maxLeaf && float(n) <= best_cost) {
                mid = -1;
            } else {
                mid = partition_bins(b, e, axis, cb, best_bin, 16);
                if (mid == b || mid == e) mid = median_split(b, e, axis);
            }
        } else {
            // best split over all three axes: exact sweep SAH up to kSweepMax primitives, 32 bins above
            float best_cost = INFINITY;
            int best_axis = -1, best_pos = -1;
            for (int a = 0; a < 3; ++a) {
                if (!(ext[a] > 0.0f)) continue;
                float cost;
                int pos;
                if (n <= kSweepMax) {
                    sweep(b, e, a, cost, pos);
                } else {
                    sah(b, e, a, cb, cost, pos, 32);
                }
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_pos = pos;
                }
            }
            if (best_axis < 0 || (n <= par_.maxLeaf && float(n) <= best_cost)) {
                mid = n <= par_.maxLeaf ? -1 : median_split(b, e, axis);
            } else if (n <= kSweepMax) {
                mid = b + best_pos;  // left count
                std::nth_element(prims_.begin() + b, prims_.begin() + mid, prims_.begin() + e, by_centroid{best_axis});
            } else {
                mid = partition_bins(b, e, best_axis, cb, best_pos, 32);
                if (mid == b || mid == e) mid = median_split(b, e, best_axis);
            }
        }
        if (mid < 0) {
            ++leaves;
            return leaf_code(b, n);
        }
        const int node = int(nodes.size() / kNodeWords);
        nodes.resize(nodes.size() + kNodeWords, 0u);
        levels = std::max(levels, level + 1);
        Box lb, rb;
        const int32_t lc = build(b, mid, level + 1, lb);
        const int32_t rc = build(mid, e, level + 1, rb);
        write_node(node, lb, rb, lc, rc);
        return node;
    }

    void write_node(int node, const Box &l, const Box &r, int32_t lc, int32_t rc) {
        float w[12];
        for (int a = 0; a < 3; ++a) {
            w[a] = l.lo[a] - pad_;
            w[3 + a] = l.hi[a] + pad_;
            w[6 + a] = r.lo[a] - pad_;
            w[9 + a] = r.hi[a] + pad_;
        }
        uint32_t *dst = &nodes[size_t(node) * kNodeWords];
        std::memcpy(dst, w, sizeof(w));
        dst[12] = uint32_t(lc);
        dst[13] = uint32_t(rc);
        dst[14] = dst[15] = 0u;
    }

    std::vector<uint32_t> nodes;
    int levels = 0;
    int leaves = 0;

private:
    int median_split(int b, int e, int axis) {
        const int mid = b + (e - b) / 2;
        std::nth_element(prims_.begin() + b, prims_.begin() + mid, prims_.begin() + e, by_centroid{axis});
        return mid;
    }

    int partition_bins(int b, int e, int axis, const Box &cb, int best_bin, int nb) {
        const float lo = cb.lo[axis], scale = float(nb) / (cb.hi[axis] - cb.lo[axis]);
        auto it = std::partition(prims_.begin() + b, prims_.begin() + e, [&](const Prim &p) {
            return std::min(nb - 1, int((p.c[axis] - lo) * scale)) <= best_bin;
        });
        return int(it - prims_.begin());
    }

    // Exact SAH over the centroid order on `axis`: best_pos = primitives left of the split.
    void sweep(int b, int e, int axis, float &best_cost, int &best_pos) {
        const int n = e - b;
        order_.assign(prims_.begin() + b, prims_.begin() + e);
        std::sort(order_.begin(), order_.end(), by_centroid{axis});
        right_.resize(size_t(n));
        Box acc;
        for (int i = n - 1; i > 0; --i) {
            acc.grow(order_[size_t(i)].lo, order_[size_t(i)].hi);
            right_[size_t(i)] = acc.area();
        }
        acc.grow(order_[0].lo, order_[0].hi);
        const float pa = std::max(acc.area(), 1e-30f);
        best_cost = INFINITY;
        best_pos = n / 2;
        Box left;
        for (int i = 1; i < n; ++i) {
            left.grow(order_[size_t(i - 1)].lo, order_[size_t(i - 1)].hi);
            const float cost = par_.traversalCost + (left.area() * float(i) + right_[size_t(i)] * float(n - i)) / pa;
            if (cost < best_cost) {
                best_cost = cost;
                best_pos = i;
            }
        }
    }

    void sah(int b, int e, int axis, const Box &cb, float &best_cost, int &best_bin, int nb) {
        Box bins[kMaxBins];
        int counts[kMaxBins] = {0};
        const float lo = cb.lo[axis], scale = float(nb) / (cb.hi[axis] - cb.lo[axis]);
        for (int i = b; i < e; ++i) {
            int bin = std::min(nb - 1, int((prims_[i].c[axis] - lo) * scale));
            ++counts[bin];
            bins[bin].grow(prims_[i].lo, prims_[i].hi);
        }
        float right_area[kMaxBins];
        int right_count[kMaxBins];
        Box acc;
        int cnt = 0;
        for (int i = nb - 1; i > 0; --i) {
            acc.grow(bins[i]);
            cnt += counts[i];
            right_area[i] = acc.area();
            right_count[i] = cnt;
        }
        Box parent;
        for (int i = 0; i < nb; ++i) parent.grow(bins[i]);
        const float pa = std::max(parent.area(), 1e-30f);
        best_cost = INFINITY;
        best_bin = nb / 2 - 1;
        Box left;
        int lcnt = 0;
        for (int i = 0; i < nb - 1; ++i) {
            left.grow(bins[i]);
            lcnt += counts[i];
            if (lcnt == 0 || right_count[i + 1] == 0) continue;
            // one traversal step = traversalCost primitive tests
            float cost = par_.traversalCost + (left.area() * lcnt + right_area[i + 1] * right_count[i + 1]) / pa;
            if (cost < best_cost) {
                best_cost = cost;
                best_bin = i;
            }
        }
    }

    std::vector<Prim> order_;
    std::vector<float> right_;
    std::vector<Prim> &prims_;
    float pad_;
    BvhParams par_;
};

}  // namespace

bool build_bvh_boxes(const float *boxes, int numPrims, float extentHint, Bvh &out, std::string &err,
                     const BvhParams &params) {
    if (params.maxLeaf < 1 || params.maxLeaf > 15 || !(params.traversalCost > 0.0f) || params.maxDepth < 1 ||
        params.maxDepth > kStackDepth) {
        err = "invalid BVH build parameters";
        return false;
    }
    if (numPrims <= 0) {
        // RayTracer.h:398-400: a BVH over an empty range is an error.
        err = "BVH requires at least one primitive";
        return false;
    }
    if (numPrims >= (1 << 27)) {
        err = "too many primitives for the 27-bit leaf index";
        return false;
    }
    std::vector<Prim> prims(static_cast<size_t>(numPrims));
    float maxabs = std::fabs(extentHint);
    for (int i = 0; i < numPrims; ++i) {
        const float *bx = boxes + 6 * size_t(i);
        Prim &p = prims[size_t(i)];
        for (int a = 0; a < 3; ++a) {
            p.lo[a] = bx[a];
            p.hi[a] = bx[3 + a];
            p.c[a] = 0.5f * (p.lo[a] + p.hi[a]);
            if (!std::isfinite(p.lo[a]) || !std::isfinite(p.hi[a])) {
                err = "non-finite primitive coordinate";
                return false;
            }
            maxabs = std::max(maxabs, std::max(std::fabs(p.lo[a]), std::fabs(p.hi[a])));
        }
        p.id = i;
    }
    const float pad = std::max(maxabs, 1e-3f) * (1.0f / 65536.0f);
    Builder bld(prims, pad, params);
    Box rootBox;
    // Node 0 must be interior: reserve it, then build the children.
    int32_t code = bld.build(0, numPrims, 0, rootBox);
    if (code < 0) {
        // Whole scene fits one leaf: root holds that leaf and an empty leaf.
        bld.nodes.assign(kNodeWords, 0u);
        bld.write_node(0, rootBox, rootBox, code, leaf_code(0, 0));
        bld.levels = 1;
    }
    out.nodes = std::move(bld.nodes);
    out.levels = bld.levels;
    out.leaves = bld.leaves;
    out.order.resize(size_t(numPrims));
    for (int i = 0; i < numPrims; ++i) out.order[size_t(i)] = prims[size_t(i)].id;
    if (out.levels > params.maxDepth) {
        err = "BVH deeper than the depth bound (too few levels for the primitives at this leaf size)";
        return false;
    }
    return true;
}

bool build_bvh(const float *verts, int numTris, float extentHint, Bvh &out, std::string &err,
               const BvhParams &params) {
    if (numTris <= 0) {
        err = "BVH requires at least one triangle";
        return false;
    }
    std::vector<float> boxes(size_t(numTris) * 6);
    for (int i = 0; i < numTris; ++i) {
        const float *v = verts + 9 * size_t(i);
        float *bx = &boxes[6 * size_t(i)];
        for (int a = 0; a < 3; ++a) {
            bx[a] = std::min(v[a], std::min(v[3 + a], v[6 + a]));
            bx[3 + a] = std::max(v[a], std::max(v[3 + a], v[6 + a]));
        }
    }
    return build_bvh_boxes(boxes.data(), numTris, extentHint, out, err, params);
}

namespace {

struct Slot {
    int32_t code;
    float lo[3], hi[3];
};

class Collapser {
public:
    Collapser(const Bvh &b, Bvh4 &o) : in_(b), out_(o) {}

    void child(int node, int c, Slot &sl) const {
        const uint32_t *w = &in_.nodes[size_t(node) * kNodeWords];
        float f[12];
        std::memcpy(f, w, sizeof(f));
        for (int a = 0; a < 3; ++a) {
            sl.lo[a] = f[6 * c + a];
            sl.hi[a] = f[6 * c + 3 + a];
        }
        sl.code = int32_t(w[12 + c]);
    }

    static float area(const Slot &sl) {
        const float dx = sl.hi[0] - sl.lo[0], dy = sl.hi[1] - sl.lo[1], dz = sl.hi[2] - sl.lo[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }

    // Emits the 4-wide node for 2-wide node `node` (and its subtree); returns its index.
    int emit(int node, int pushesAbove, int level) {
        Slot slots[4];
        int n = 2;
        child(node, 0, slots[0]);
        child(node, 1, slots[1]);
        while (n < 4) {
            int best = -1;
            for (int i = 0; i < n; ++i)
                if (slots[i].code >= 0 && (best < 0 || area(slots[i]) > area(slots[best]))) best = i;
            if (best < 0) break;
            const int open = slots[best].code;
            child(open, 0, slots[best]);
            child(open, 1, slots[n++]);
        }
        const int idx = int(out_.nodes.size() / kNode4Words);
        out_.nodes.resize(out_.nodes.size() + kNode4Words, 0u);
        out_.levels = std::max(out_.levels, level);
        const int pushes = pushesAbove + (n - 1);
        out_.stackBound = std::max(out_.stackBound, pushes);
        int32_t codes[4];
        for (int i = 0; i < 4; ++i) codes[i] = i < n ? slots[i].code : leaf_code(0, 0);
        for (int i = 0; i < n; ++i)
            if (slots[i].code >= 0) codes[i] = emit(slots[i].code, pushes, level + 1);
        float f[24];
        for (int i = 0; i < 4; ++i)
            for (int a = 0; a < 3; ++a) {
                // unused slot: a point far outside any scene (an empty leaf if ever reached)
                f[8 * a + i] = i < n ? slots[i].lo[a] : kFar[a];
                f[8 * a + 4 + i] = i < n ? slots[i].hi[a] : kFar[a];
            }
        uint32_t *dst = &out_.nodes[size_t(idx) * kNode4Words];
        std::memcpy(dst, f, sizeof(f));
        for (int i = 0; i < 4; ++i) dst[24 + i] = uint32_t(codes[i]);
        return idx;
    }

private:
    static constexpr float kFar[3] = {3.0e38f, -1.0e20f, 7.0e33f};
    const Bvh &in_;
    Bvh4 &out_;
};

// SAH-optimal collapse (dynamic programming over the 2-wide tree, after Ylitie et al. 2017,
// reduced to 4 children): cost(n, i) = least expected cost of the 2-wide subtree n spread over
// at most i child slots of its 4-wide parent, where a slot is a leaf of at most maxLeaf
// primitives (a 2-wide subtree's primitives are contiguous, so any subtree can become one leaf:
// area * count * 1), a 4-wide node (area * nodeCost + its children's cost over 4 slots), or,
// for i > 1, the subtree's two children sharing the slots.  Areas are relative to the root's.
class SahCollapser {
public:
    SahCollapser(const Bvh &b, Bvh4 &o, float nodeCost, int maxLeaf)
        : in_(b), out_(o), cn_(nodeCost), maxLeaf_(std::max(1, std::min(maxLeaf, 15))) {
        const size_t n = in_.nodes.size() / kNodeWords;
        dp_.assign(n, Dp{});
        std::vector<int> order;  // preorder; children after parents -> reverse is bottom-up
        order.reserve(n);
        order.push_back(0);
        for (size_t h = 0; h < order.size(); ++h)
            for (int c = 0; c < 2; ++c) {
                const int32_t k = code(order[h], c);
                if (k >= 0) order.push_back(k);
            }
        for (size_t h = order.size(); h-- > 0;) solve(order[h]);
    }

    // Emits the 4-wide node for 2-wide node `node`; returns its index.
    int emit(int node, int pushesAbove, int level) {
        Slot slots[4];
        int n = 0;
        const Dp &d = dp_[size_t(node)];
        expand_child(node, 0, d.splitD4, slots, n);
        expand_child(node, 1, 4 - d.splitD4, slots, n);
        const int idx = int(out_.nodes.size() / kNode4Words);
        out_.nodes.resize(out_.nodes.size() + kNode4Words, 0u);
        out_.levels = std::max(out_.levels, level);
        const int pushes = pushesAbove + (n - 1);
        out_.stackBound = std::max(out_.stackBound, pushes);
        int32_t codes[4];
        for (int i = 0; i < 4; ++i) codes[i] = i < n ? slots[i].code : leaf_code(0, 0);
        for (int i = 0; i < n; ++i)
            if (slots[i].code >= 0) codes[i] = emit(slots[i].code, pushes, level + 1);
        float f[24];
        for (int i = 0; i < 4; ++i)
            for (int a = 0; a < 3; ++a) {
                f[8 * a + i] = i < n ? slots[i].lo[a] : kFar[a];
                f[8 * a + 4 + i] = i < n ? slots[i].hi[a] : kFar[a];
            }
        uint32_t *dst = &out_.nodes[size_t(idx) * kNode4Words];
        std::memcpy(dst, f, sizeof(f));
        for (int i = 0; i < 4; ++i) dst[24 + i] = uint32_t(codes[i]);
        return idx;
    }

private:
    struct Dp {
        float cost[5] = {0, 0, 0, 0, 0};  // cost(n, i), i = 1..4
        bool leaf = false;                // cost(n, 1) is the merged leaf (else a 4-wide node)
        bool spread[5] = {};              // cost(n, i) spreads the two children over i slots
        int split[5] = {};                // slots of child 0 when spread (i = 2..4)
        int splitD4 = 2;                  // child 0's slots in the 4-wide node's distribution
        int first = 0, count = 0;         // contiguous primitive range (count < 0: not contiguous)
    };

    int32_t code(int node, int c) const { return int32_t(in_.nodes[size_t(node) * kNodeWords + 12 + size_t(c)]); }

    void box(int node, int c, float *lo, float *hi) const {
        float f[12];
        std::memcpy(f, &in_.nodes[size_t(node) * kNodeWords], sizeof(f));
        for (int a = 0; a < 3; ++a) {
            lo[a] = f[6 * c + a];
            hi[a] = f[6 * c + 3 + a];
        }
    }

    static float area(const float *lo, const float *hi) {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }

    // cost(child c of node, i), its primitive range and whether it is a 2-wide leaf
    void child(int node, int c, int i, float &cost, int &first, int &count) const {
        const int32_t k = code(node, c);
        if (k >= 0) {
            cost = dp_[size_t(k)].cost[i];
            first = dp_[size_t(k)].first;
            count = dp_[size_t(k)].count;
            return;
        }
        float lo[3], hi[3];
        box(node, c, lo, hi);
        first = (~k) >> 4;
        count = (~k) & 15;
        cost = area(lo, hi) * float(count) / rootArea();
    }

    float rootArea() const {
        if (rootArea_ > 0) return rootArea_;
        float lo0[3], hi0[3], lo1[3], hi1[3], lo[3], hi[3];
        box(0, 0, lo0, hi0);
        box(0, 1, lo1, hi1);
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo0[a], lo1[a]);
            hi[a] = std::max(hi0[a], hi1[a]);
        }
        rootArea_ = std::max(area(lo, hi), 1e-30f);
        return rootArea_;
    }

    void solve(int node) {
        Dp &d = dp_[size_t(node)];
        float lo0[3], hi0[3], lo1[3], hi1[3], lo[3], hi[3];
        box(node, 0, lo0, hi0);
        box(node, 1, lo1, hi1);
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo0[a], lo1[a]);
            hi[a] = std::max(hi0[a], hi1[a]);
        }
        const float an = area(lo, hi) / rootArea();
        float c0[5], c1[5];
        int f0 = 0, n0 = 0, f1 = 0, n1 = 0;
        for (int i = 1; i <= 4; ++i) {
            child(node, 0, i, c0[i], f0, n0);
            child(node, 1, i, c1[i], f1, n1);
        }
        // the subtree's primitives as one range (the builder partitions in place)
        if (n0 >= 0 && n1 >= 0 && (n0 == 0 || n1 == 0 || f0 + n0 == f1)) {
            d.first = n0 == 0 ? f1 : f0;
            d.count = n0 + n1;
        } else {
            d.count = -1;
        }
        float D[5] = {0, INFINITY, INFINITY, INFINITY, INFINITY};
        int Ds[5] = {0, 0, 1, 1, 2};
        for (int j = 2; j <= 4; ++j)
            for (int k = 1; k < j; ++k) {
                const float c = c0[k] + c1[j - k];
                if (c < D[j]) {
                    D[j] = c;
                    Ds[j] = k;
                }
            }
        d.splitD4 = Ds[4];
        const float asNode = an * cn_ + D[4];
        const float asLeaf = d.count >= 0 && d.count <= maxLeaf_ ? an * float(d.count) : INFINITY;
        d.leaf = asLeaf <= asNode;
        d.cost[1] = std::min(asLeaf, asNode);
        for (int i = 2; i <= 4; ++i) {
            d.spread[i] = D[i] < d.cost[1];
            d.split[i] = Ds[i];
            d.cost[i] = std::min(d.cost[1], D[i]);
        }
    }

    // Appends the slots that child c of `node` becomes when given `i` slots.
    void expand_child(int node, int c, int i, Slot *slots, int &n) const {
        const int32_t k = code(node, c);
        if (k < 0) {
            Slot &sl = slots[n++];
            box(node, c, sl.lo, sl.hi);
            sl.code = k;
            return;
        }
        const Dp &d = dp_[size_t(k)];
        if (i > 1 && d.spread[i]) {
            expand_child(k, 0, d.split[i], slots, n);
            expand_child(k, 1, i - d.split[i], slots, n);
            return;
        }
        Slot &sl = slots[n++];
        box(node, c, sl.lo, sl.hi);
        sl.code = d.leaf ? leaf_code(d.first, d.count) : k;
    }

    static constexpr float kFar[3] = {3.0e38f, -1.0e20f, 7.0e33f};
    const Bvh &in_;
    Bvh4 &out_;
    float cn_;
    int maxLeaf_;
    std::vector<Dp> dp_;
    mutable float rootArea_ = 0.0f;
};

}  // namespace

void collapse_bvh4(const Bvh &bvh2, Bvh4 &out, const BvhParams &params) {
    out.nodes.clear();
    out.levels = 0;
    out.stackBound = 0;
    if (params.collapse == 1 && !bvh2.nodes.empty())
        SahCollapser(bvh2, out, params.nodeCost, params.maxLeaf4).emit(0, 0, 1);
    else
        Collapser(bvh2, out).emit(0, 0, 1);
}

int order_bvh4_top(Bvh4 &b, int topNodes) {
    const int n = int(b.nodes.size() / kNode4Words);
    if (n == 0) return 0;
    topNodes = std::max(1, std::min(topNodes, n));
    // BFS from the root for the first topNodes nodes; the rest keep their (preorder) order
    std::vector<int> newIdx(size_t(n), -1), bfs;
    bfs.reserve(size_t(topNodes));
    bfs.push_back(0);
    newIdx[0] = 0;
    for (size_t h = 0; h < bfs.size() && int(bfs.size()) < topNodes; ++h) {
        const uint32_t *w = &b.nodes[size_t(bfs[h]) * kNode4Words];
        for (int i = 0; i < 4 && int(bfs.size()) < topNodes; ++i) {
            const int32_t c = int32_t(w[24 + i]);
            if (c < 0) continue;
            newIdx[size_t(c)] = int(bfs.size());
            bfs.push_back(c);
        }
    }
    int next = int(bfs.size());
    for (int k = 0; k < n; ++k)
        if (newIdx[size_t(k)] < 0) newIdx[size_t(k)] = next++;
    std::vector<uint32_t> out(b.nodes.size());
    for (int k = 0; k < n; ++k) {
        uint32_t *d = &out[size_t(newIdx[size_t(k)]) * kNode4Words];
        std::memcpy(d, &b.nodes[size_t(k) * kNode4Words], kNode4Words * sizeof(uint32_t));
        for (int i = 0; i < 4; ++i) {
            const int32_t c = int32_t(d[24 + i]);
            if (c >= 0) d[24 + i] = uint32_t(newIdx[size_t(c)]);
        }
    }
    b.nodes.swap(out);
    return int(bfs.size());
}

bool quantize_bvh4(const Bvh4 &in, std::vector<uint32_t> &out) {
    const size_t n = in.nodes.size() / kNode4Words;
    out.assign(n * kNode4QWords, 0u);
    const int32_t unused = leaf_code(0, 0);
    for (size_t k = 0; k < n; ++k) {
        const uint32_t *w = &in.nodes[k * kNode4Words];
        float f[24];
        std::memcpy(f, w, sizeof(f));
        uint32_t *d = &out[k * kNode4QWords];
        bool used[4];
        for (int i = 0; i < 4; ++i) used[i] = int32_t(w[24 + i]) != unused;
        uint32_t qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
        float origin[3], scale[3];
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int i = 0; i < 4; ++i)
                if (used[i]) {
                    lo = std::min(lo, f[8 * a + i]);
                    hi = std::max(hi, f[8 * a + 4 + i]);
                }
            if (!(lo <= hi)) lo = hi = 0.0f;  // no used child (never built; kept total)
            if (!std::isfinite(lo) || !std::isfinite(hi)) {  // padded past FLT_MAX
                out.clear();
                return false;
            }
            // Smallest power-of-two scale s whose grid, with its origin at least one step below
            // lo, covers [lo, hi] with every plane at least one step outside (a plane on the grid
            // moves one more step out): every decoded plane lies outside the Bvh4 plane, which
            // the builder already padded by M * 2^-16 (M = the largest |coordinate| of any
            // primitive or the camera, bvh_builder.cpp build_bvh_boxes).  That global pad, not
            // the grid step, is what absorbs the kernel's roundings of q*(s*inv) +
            // (o*inv - o_ray*inv): each of its three roundings errs by at most 2^-24 of a term
            // bounded by M*|inv| (|o| and |o_ray| are at most ~M: ray origins are points on
            // primitives or the camera), about 2^-21 * M * |inv| in all, 2^5 times below the pad
            // even for a node far smaller than its distance from the ray origin.  The
            // differences are exact in double, the division by s too.
            const double ext = double(hi) - double(lo);
            int e = -100;
            if (ext > 0) {
                e = int(std::ceil(std::log2(ext / 253.0)));
                while (e > -100 && std::ldexp(253.0, e - 1) >= ext) --e;
                e = std::max(e, -100);
            }
            uint32_t ql[4], qh[4];
            float o = lo;
            for (;; ++e) {
                // boxes near +-FLT_MAX: no finite grid (origin or scale overflows) covers them;
                // the scene then has no 8-bit tree (the kernels use the float nodes)
                if (e > 126) {
                    out.clear();
                    return false;
                }
                const double s = std::ldexp(1.0, e);
                o = float(double(lo) - s);
                if (!std::isfinite(o)) {
                    out.clear();
                    return false;
                }
                if (double(o) > double(lo) - s) o = std::nextafter(o, -INFINITY);  // round down
                bool fits = true;
                for (int i = 0; i < 4 && fits; ++i) {
                    ql[i] = 255;  // unused: lo > hi on every axis
                    qh[i] = 0;
                    if (!used[i]) continue;
                    const double xl = (double(f[8 * a + i]) - double(o)) / s;
                    const double xh = (double(f[8 * a + 4 + i]) - double(o)) / s;
                    double l = std::floor(xl), h = std::ceil(xh);
                    if (l == xl) l -= 1.0;
                    if (h == xh) h += 1.0;
                    fits = l >= 0.0 && h <= 255.0;
                    ql[i] = uint32_t(std::max(l, 0.0));
                    qh[i] = uint32_t(std::min(h, 255.0));
                }
                if (fits) break;
            }
            origin[a] = o;
            scale[a] = float(std::ldexp(1.0, e));
            for (int i = 0; i < 4; ++i) {
                qlo[a] |= ql[i] << (8 * i);
                qhi[a] |= qh[i] << (8 * i);
            }
        }
        std::memcpy(&d[0], origin, 3 * sizeof(float));
        std::memcpy(&d[3], &scale[0], sizeof(float));
        for (int a = 0; a < 3; ++a) {
            d[4 + 2 * a] = qlo[a];
            d[5 + 2 * a] = qhi[a];
        }
        std::memcpy(&d[10], &scale[1], sizeof(float));
        std::memcpy(&d[11], &scale[2], sizeof(float));
        for (int i = 0; i < 4; ++i) d[12 + i] = w[24 + i];
    }
    return true;
}

bool hybrid_bvh4(const Bvh4 &b, const std::vector<uint32_t> &q, int topNodes, std::vector<uint32_t> &out) {
    const size_t n = b.nodes.size() / kNode4Words;
    out.clear();
    if (q.size() != n * kNode4QWords || topNodes < 1 || size_t(topNodes) > n) return false;
    const size_t top = size_t(topNodes);
    auto code = [&](int32_t c) -> uint32_t {
        if (c < 0) return uint32_t(c);  // leaf
        const size_t k = size_t(c);
        return uint32_t(k < top ? k * 128 : top * 128 + (k - top) * 64);
    };
    out.resize(top * kNode4Words + (n - top) * kNode4QWords);
    for (size_t k = 0; k < top; ++k) {
        uint32_t *d = &out[k * kNode4Words];
        std::memcpy(d, &b.nodes[k * kNode4Words], kNode4Words * sizeof(uint32_t));
        for (int i = 0; i < 4; ++i) d[24 + i] = code(int32_t(d[24 + i]));
    }
    for (size_t k = top; k < n; ++k) {
        uint32_t *d = &out[top * kNode4Words + (k - top) * kNode4QWords];
        std::memcpy(d, &q[k * kNode4QWords], kNode4QWords * sizeof(uint32_t));
        for (int i = 0; i < 4; ++i) {
            const int32_t c = int32_t(d[12 + i]);
            if (c >= 0 && size_t(c) < top) {  // never for a breadth-first top; kept total
                out.clear();
                return false;
            }
            d[12 + i] = code(c);
        }
    }
    return true;
}

float half_value(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const double mag = e == 31 ? (m ? NAN : INFINITY) : e == 0 ? std::ldexp(double(m), -24)
                                                               : std::ldexp(double(1024 + m), e - 25);
    return float((h & 0x8000u) ? -mag : mag);
}

// |x| truncated to a half (toward zero; finite values beyond the largest half give it), as bits
static uint16_t half_trunc_mag(double a) {
    if (std::isinf(a)) return 0x7C00u;
    if (a >= 65504.0) return 0x7BFFu;
    if (a < std::ldexp(1.0, -14)) return uint16_t(std::floor(std::ldexp(a, 24)));  // subnormal / zero
    int e = 0;
    const double f = std::frexp(a, &e);  // a = f * 2^e, f in [0.5, 1)
    const int m = int(std::floor(std::ldexp(f, 11))) - 1024;
    return uint16_t(((e + 14) << 10) | m);
}

uint16_t half_round_down(float x) {
    const double a = std::fabs(double(x));
    uint16_t h = half_trunc_mag(a);
    if (std::signbit(x)) {
        if (half_value(h) != float(a)) ++h;  // truncation rounded a negative value up: one step away
        h |= 0x8000u;
    }
    return h;
}

uint16_t half_round_up(float x) { return uint16_t(half_round_down(-x) ^ 0x8000u); }

bool half_bvh4(const uint32_t *in, size_t numNodes, std::vector<uint32_t> &out) {
    out.assign(numNodes * kNode4Words, 0u);
    for (size_t k = 0; k < numNodes; ++k) {
        const uint32_t *w = in + k * kNode4Words;
        uint16_t *h = reinterpret_cast<uint16_t *>(out.data() + k * kNode4Words);
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 4; ++i) {
                float lo, hi;
                std::memcpy(&lo, w + 8 * a + i, 4);
                std::memcpy(&hi, w + 8 * a + 4 + i, 4);
                // a finite plane beyond the half range would round to an infinite one: a box every
                // ray enters.  No half tree then (the caller keeps float nodes), like quantize_bvh4
                // for boxes no 8-bit grid covers.
                if ((std::isfinite(lo) && lo < -65504.0f) || (std::isfinite(hi) && hi > 65504.0f)) {
                    out.clear();
                    return false;
                }
                const uint16_t l = half_round_down(lo), u = half_round_up(hi);
                h[16 * a + i] = l;  // [lo hi]: positive direction
                h[16 * a + 4 + i] = u;
                h[16 * a + 8 + i] = u;  // [hi lo]: negative direction
                h[16 * a + 12 + i] = l;
            }
        std::memcpy(out.data() + k * kNode4Words + 24, w + 24, 16);  // codes at byte 96
    }
    return true;
}

}  // namespace hippt
