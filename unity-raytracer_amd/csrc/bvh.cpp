// bvh.cpp — binned-SAH BVH2 builder (host).  See bvh.h for the contract.
#include "bvh.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>

namespace rtb {
namespace {

constexpr int kBins = 32;
#ifdef RT_EXP_SAH_TRAV
constexpr float kTraversalCost = RT_EXP_SAH_TRAV;  // measuring builds only
#else
constexpr float kTraversalCost = 1.0f;  // relative to one primitive test
#endif
constexpr float kIntersectCost = 1.0f;

struct Box {
    float lo[3], hi[3];
    void reset() {
        for (int i = 0; i < 3; ++i) {
            lo[i] = std::numeric_limits<float>::infinity();
            hi[i] = -std::numeric_limits<float>::infinity();
        }
    }
    void grow(const float *l, const float *h) {
        for (int i = 0; i < 3; ++i) {
            lo[i] = std::min(lo[i], l[i]);
            hi[i] = std::max(hi[i], h[i]);
        }
    }
    void grow(const Box &b) { grow(b.lo, b.hi); }
    bool empty() const { return lo[0] > hi[0]; }
    float area() const {
        if (empty()) return 0.0f;
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

inline int ceil_log2(int n) {
    int k = 0;
    while ((1 << k) < n) ++k;
    return k;
}

inline bool same_group(const Prim &a, const Prim &b) { return a.kind == b.kind && a.gate == b.gate; }

struct Builder {
    std::vector<Prim> &P;
    int max_leaf;
    BuildResult &R;
    int empty_leaf = -1;

    int make_leaf(int begin, int end) {
        rtd::LeafDesc L;
        L.kind = P[begin].kind;
        L.gate = P[begin].gate;
        L.count = end - begin;
        if (L.kind == rtd::kLeafTri) {
            L.first = (int)R.tri_order.size();
            for (int i = begin; i < end; ++i) R.tri_order.push_back(P[i].payload);
        } else {
            L.first = (int)R.sph_order.size();
            for (int i = begin; i < end; ++i) R.sph_order.push_back(P[i].payload);
        }
        R.leaves.push_back(L);
        return ~((int)R.leaves.size() - 1);
    }

    int get_empty_leaf() {
        if (empty_leaf == -1) {
            rtd::LeafDesc L;
            L.first = 0; L.count = 0; L.kind = rtd::kLeafTri; L.gate = -1;
            R.leaves.push_back(L);
            empty_leaf = ~((int)R.leaves.size() - 1);
        }
        return empty_leaf;
    }

    // Returns the encoded child (>= 0 node, < 0 leaf); out = its bounds.
    int build(int begin, int end, int depth, Box &out) {
        const int n = end - begin;
        Box b, cb;
        b.reset();
        cb.reset();
        bool homo = true;
        for (int i = begin; i < end; ++i) {
            b.grow(P[i].lo, P[i].hi);
            cb.grow(P[i].c, P[i].c);
            homo = homo && same_group(P[i], P[begin]);
        }
        out = b;
        R.max_depth = std::max(R.max_depth, depth);
        if (n == 1) return make_leaf(begin, end);

        const bool forced = depth + ceil_log2(n) >= rtd::kMaxTreeDepth;
        int best_axis = -1, best_split = -1;
        float best_cost = std::numeric_limits<float>::infinity();
        if (!forced) {
            const float parent_area = std::max(b.area(), 1e-30f);
            for (int axis = 0; axis < 3; ++axis) {
                float ext = cb.hi[axis] - cb.lo[axis];
                if (!(ext > 0.0f)) continue;
                float scale = kBins / ext;
                Box bins[kBins];
                int cnt[kBins];
                for (int k = 0; k < kBins; ++k) { bins[k].reset(); cnt[k] = 0; }
                for (int i = begin; i < end; ++i) {
                    int k = std::min(kBins - 1, (int)((P[i].c[axis] - cb.lo[axis]) * scale));
                    bins[k].grow(P[i].lo, P[i].hi);
                    cnt[k]++;
                }
                float right_area[kBins];
                int right_cnt[kBins];
                Box acc;
                acc.reset();
                int c = 0;
                for (int k = kBins - 1; k > 0; --k) {
                    acc.grow(bins[k]);
                    c += cnt[k];
                    right_area[k] = acc.area();
                    right_cnt[k] = c;
                }
                acc.reset();
                c = 0;
                for (int k = 0; k < kBins - 1; ++k) {
                    acc.grow(bins[k]);
                    c += cnt[k];
                    int rc = right_cnt[k + 1];
                    if (c == 0 || rc == 0) continue;
                    float cost = kTraversalCost +
                                 kIntersectCost * (acc.area() * c + right_area[k + 1] * rc) / parent_area;
                    if (cost < best_cost) {
                        best_cost = cost;
                        best_axis = axis;
                        best_split = k + 1;
                    }
                }
            }
        }
        if (homo && n <= max_leaf && (best_axis < 0 || kIntersectCost * n <= best_cost))
            return make_leaf(begin, end);

        int mid = begin;
        if (!forced && best_axis >= 0) {
            const int axis = best_axis;
            const float lo = cb.lo[axis];
            const float scale = kBins / (cb.hi[axis] - cb.lo[axis]);
            Prim *m = std::partition(P.data() + begin, P.data() + end, [&](const Prim &p) {
                int k = std::min(kBins - 1, (int)((p.c[axis] - lo) * scale));
                return k < best_split;
            });
            mid = (int)(m - P.data());
        }
        if (mid == begin || mid == end) {
            if (!forced && !homo) {
                // group split: separate the first (kind, gate) group
                Prim first = P[begin];
                Prim *m = std::partition(P.data() + begin, P.data() + end,
                                         [&](const Prim &p) { return same_group(p, first); });
                mid = (int)(m - P.data());
            }
            if (mid == begin || mid == end) {
                int axis = 0;
                float ext = -1.0f;
                for (int a = 0; a < 3; ++a)
                    if (cb.hi[a] - cb.lo[a] > ext) { ext = cb.hi[a] - cb.lo[a]; axis = a; }
                mid = begin + n / 2;
                std::nth_element(P.data() + begin, P.data() + mid, P.data() + end,
                                 [&](const Prim &x, const Prim &y) { return x.c[axis] < y.c[axis]; });
            }
        }
        const int idx = (int)R.nodes.size();
        R.nodes.push_back(rtd::BvhNode{});
        Box lb, rb;
        int l = build(begin, mid, depth + 1, lb);
        int r = build(mid, end, depth + 1, rb);
        rtd::BvhNode &nd = R.nodes[idx];
        nd.a = make_float4(lb.lo[0], lb.hi[0], lb.lo[1], lb.hi[1]);
        nd.b = make_float4(rb.lo[0], rb.hi[0], rb.lo[1], rb.hi[1]);
        nd.c = make_float4(lb.lo[2], lb.hi[2], rb.lo[2], rb.hi[2]);
        nd.d = make_int4(l, r, 0, 0);
        return idx;
    }
};

}  // namespace

namespace {

float box_area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

struct Slot {
    int ref2;  // BVH2 child ref
    float lo[3], hi[3];
};

void child_boxes(const rtd::BvhNode &n, Slot &a, Slot &b) {
    a.ref2 = n.d.x;
    b.ref2 = n.d.y;
    a.lo[0] = n.a.x; a.hi[0] = n.a.y; a.lo[1] = n.a.z; a.hi[1] = n.a.w; a.lo[2] = n.c.x; a.hi[2] = n.c.y;
    b.lo[0] = n.b.x; b.hi[0] = n.b.y; b.lo[1] = n.b.z; b.hi[1] = n.b.w; b.lo[2] = n.c.z; b.hi[2] = n.c.w;
}

int collapse(const BuildResult &B, int node2, int depth, std::vector<rtd::BvhNode4> &out, int &max_depth,
             int empty_ref) {
    max_depth = std::max(max_depth, depth);
    const int idx = (int)out.size();
    out.push_back(rtd::BvhNode4{});
    Slot slots[4];
    int n = 2;
    child_boxes(B.nodes[node2], slots[0], slots[1]);
    while (n < 4) {
        int best = -1;
        float best_a = -1.0f;
        for (int i = 0; i < n; ++i)
            if (slots[i].ref2 >= 0) {
                const float a = box_area(slots[i].lo, slots[i].hi);
                if (a > best_a) { best_a = a; best = i; }
            }
        if (best < 0) break;
        Slot a, b;
        child_boxes(B.nodes[slots[best].ref2], a, b);
        slots[best] = a;
        slots[n++] = b;
    }
    int refs[4] = {empty_ref, empty_ref, empty_ref, empty_ref};
    float lo[3][4], hi[3][4];
    const float inf = std::numeric_limits<float>::infinity();
    for (int i = 0; i < 4; ++i) {
        bool empty = i >= n;
        if (!empty && slots[i].ref2 < 0) {
            const rtd::LeafDesc &L = B.leaves[~slots[i].ref2];
            if (L.count == 0) empty = true;
            else refs[i] = rtd::encode_leaf(L.first, L.count, L.kind);
        }
        for (int a = 0; a < 3; ++a) {
            lo[a][i] = empty ? inf : slots[i].lo[a];
            hi[a][i] = empty ? inf : slots[i].hi[a];
        }
    }
    for (int i = 0; i < n; ++i)
        if (slots[i].ref2 >= 0) refs[i] = collapse(B, slots[i].ref2, depth + 1, out, max_depth, empty_ref);
    rtd::BvhNode4 &nd = out[idx];
    nd.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
    nd.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
    nd.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
    nd.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
    nd.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
    nd.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
    nd.child = make_int4(refs[0], refs[1], refs[2], refs[3]);
    nd.pad = make_int4(0, 0, 0, 0);
    return idx;
}

}  // namespace

int collapse_bvh4(const BuildResult &B, std::vector<rtd::BvhNode4> &out, int empty_ref) {
    out.clear();
    if (B.nodes.empty()) return 0;
    out.reserve(B.nodes.size() / 2 + 1);
    int max_depth = 0;
    collapse(B, 0, 0, out, max_depth, empty_ref);
    return max_depth;
}

BuildResult build_bvh(std::vector<Prim> &prims, int max_leaf) {
    auto t0 = std::chrono::steady_clock::now();
    BuildResult R;
    if (prims.empty()) return R;
    R.nodes.reserve(prims.size());
    Builder B{prims, max_leaf, R};
    Box box;
    int root = B.build(0, (int)prims.size(), 0, box);
    if (root < 0) {
        // a single leaf: hang it under a root beside an empty leaf far away
        rtd::BvhNode nd;
        int e = B.get_empty_leaf();
        const float far = 1e30f;
        nd.a = make_float4(box.lo[0], box.hi[0], box.lo[1], box.hi[1]);
        nd.b = make_float4(far, far, far, far);
        nd.c = make_float4(box.lo[2], box.hi[2], far, far);
        nd.d = make_int4(root, e, 0, 0);
        R.nodes.push_back(nd);
        R.max_depth = 1;
    }
    R.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return R;
}

}  // namespace rtb
