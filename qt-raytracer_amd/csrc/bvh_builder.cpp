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

constexpr int kBins = 16;

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
        } else {
            float best_cost;
            int best_bin;
            sah(b, e, axis, cb, best_cost, best_bin);
            const float leaf_cost = float(n);
            if (n <= par_.maxLeaf && leaf_cost <= best_cost) {
                mid = -1;
            } else {
                const float lo = cb.lo[axis], scale = kBins / ext[axis];
                auto it = std::partition(prims_.begin() + b, prims_.begin() + e, [&](const Prim &p) {
                    int bin = std::min(kBins - 1, int((p.c[axis] - lo) * scale));
                    return bin <= best_bin;
                });
                mid = int(it - prims_.begin());
                if (mid == b || mid == e) mid = median_split(b, e, axis);
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
        std::nth_element(prims_.begin() + b, prims_.begin() + mid, prims_.begin() + e,
                         [axis](const Prim &p, const Prim &q) {
                             return p.c[axis] < q.c[axis] || (p.c[axis] == q.c[axis] && p.id < q.id);
                         });
        return mid;
    }

    void sah(int b, int e, int axis, const Box &cb, float &best_cost, int &best_bin) {
        Box bins[kBins];
        int counts[kBins] = {0};
        const float lo = cb.lo[axis], scale = kBins / (cb.hi[axis] - cb.lo[axis]);
        for (int i = b; i < e; ++i) {
            int bin = std::min(kBins - 1, int((prims_[i].c[axis] - lo) * scale));
            ++counts[bin];
            bins[bin].grow(prims_[i].lo, prims_[i].hi);
        }
        float right_area[kBins];
        int right_count[kBins];
        Box acc;
        int cnt = 0;
        for (int i = kBins - 1; i > 0; --i) {
            acc.grow(bins[i]);
            cnt += counts[i];
            right_area[i] = acc.area();
            right_count[i] = cnt;
        }
        Box parent;
        for (int i = 0; i < kBins; ++i) parent.grow(bins[i]);
        const float pa = std::max(parent.area(), 1e-30f);
        best_cost = INFINITY;
        best_bin = kBins / 2 - 1;
        Box left;
        int lcnt = 0;
        for (int i = 0; i < kBins - 1; ++i) {
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

bool build_bvh(const float *verts, int numTris, float extentHint, Bvh &out, std::string &err) {
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
    return build_bvh_boxes(boxes.data(), numTris, extentHint, out, err);
}

}  // namespace hippt
