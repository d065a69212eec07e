// lbvh.hip — on-device linear BVH build (see lbvh.h).
#include "lbvh.h"

#include <hipcub/hipcub.hpp>

#include "rt_math.h"

namespace rtl {
namespace {

using rtm::f3;
using rtm::mk;

constexpr int kThreads = 256;
constexpr int kLbvhLeaf = 4;  // max primitives per collapsed leaf (2-bit count field)
#ifdef RT_EXP_LBVH_NODECOST
constexpr float kLeafNodeCost = RT_EXP_LBVH_NODECOST;  // measuring builds only
#else
constexpr float kLeafNodeCost = 1.0f;  // a node step against one primitive test (k_small's leaf rule)
#endif

inline int blocks_for(int n) { return (n + kThreads - 1) / kThreads; }

__device__ __forceinline__ unsigned expand_bits(unsigned v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// Morton code of c quantised to `bits` (<= 10) bits per axis inside [lo, hi].
__device__ __forceinline__ unsigned morton(f3 c, const float lo[3], const float hi[3], int bits) {
    unsigned q[3];
    const float cv[3] = {c.x, c.y, c.z};
    const float cells = (float)(1u << bits);
    for (int a = 0; a < 3; ++a) {
        const float ext = hi[a] - lo[a];
        float t = ext > 0.0f ? (cv[a] - lo[a]) / ext : 0.5f;
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        q[a] = (unsigned)fminf(t * cells, cells - 1.0f);
    }
    return (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
}

__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

// 1. per reference rank: records, padded bounds, sort key
__global__ void k_prims(LbvhInput in, LbvhOutput out, int n, float4 *plo, float4 *phi, unsigned long long *keys,
                        int *vals, rtd::TriRec *tri_rank) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    float scene_lo[3], scene_hi[3], pad_abs;
    if (in.box_dev) {  // computed on the device this frame (scene_xform.hip k_scene_box)
        for (int a = 0; a < 3; ++a) {
            scene_lo[a] = in.box_dev[a];
            scene_hi[a] = in.box_dev[3 + a];
        }
        pad_abs = in.box_dev[6];
    } else {
        for (int a = 0; a < 3; ++a) {
            scene_lo[a] = in.scene_lo[a];
            scene_hi[a] = in.scene_hi[a];
        }
        pad_abs = in.pad_abs;
    }
    float lo[3], hi[3], cen[3];
    int gate = -1;
    if (r < in.mt || r >= in.mt + in.ns) {
        const float *v;
        const float *nn;
        int mat;
        if (r < in.mt) {
            int a = 0, b = in.mesh_count - 1;  // last mesh with rank_first <= r
            while (a < b) {
                const int m = (a + b + 1) >> 1;
                if (in.meshes[m].rank_first <= r) a = m; else b = m - 1;
            }
            const MeshDev M = in.meshes[a];
            const int g = M.geom_first + (r - M.rank_first);
            v = in.mesh_tris + (size_t)g * 9;
            nn = in.mesh_normals + (size_t)g * 3;
            mat = M.material;
            gate = a;
        } else {
            const int i = r - in.mt - in.ns;
            v = in.loose_tris + (size_t)i * 9;
            nn = in.loose_normals + (size_t)i * 3;
            mat = in.loose_mat[i];
        }
        const f3 v0 = ld3(v), v1 = ld3(v + 3), v2 = ld3(v + 6);
        const f3 e1 = v1 - v0, e2 = v2 - v0;  // RMath.cs:34-35
        rtd::TriRec tr;
        tr.p0 = make_float4(v0.x, v0.y, v0.z, e1.x);
        tr.p1 = make_float4(e1.y, e1.z, e2.x, e2.y);
        tr.p2 = make_float4(e2.z, __int_as_float(r), __int_as_float(gate), 0.0f);
        tri_rank[r] = tr;
        out.shade[r] = make_float4(nn[0], nn[1], nn[2], __int_as_float(mat));
        float ext = 0.0f;
        const float *vs[3] = {v, v + 3, v + 6};
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(vs[0][a], fminf(vs[1][a], vs[2][a]));
            hi[a] = fmaxf(vs[0][a], fmaxf(vs[1][a], vs[2][a]));
            ext = fmaxf(ext, hi[a] - lo[a]);
        }
        const float pad = pad_abs + ext * 1e-4f;
        for (int a = 0; a < 3; ++a) {
            cen[a] = 0.5f * (lo[a] + hi[a]);
            lo[a] -= pad;
            hi[a] += pad;
        }
    } else {
        const int i = r - in.mt;
        const float *sp = in.spheres + (size_t)i * 4;
        const float rad = sqrtf(sp[3]);
        rtd::SphRec sr;
        sr.cr = make_float4(sp[0], sp[1], sp[2], sp[3]);
        sr.misc = make_int4(r, -1, 0, 0);
        *(rtd::SphRec *)&tri_rank[r] = sr;
        out.shade[r] = make_float4(sp[0], sp[1], sp[2], __int_as_float(in.sphere_mat[i]));
        const float pad = pad_abs + rad * 1e-4f;
        for (int a = 0; a < 3; ++a) {
            cen[a] = sp[a];
            lo[a] = sp[a] - rad - pad;
            hi[a] = sp[a] + rad + pad;
        }
    }
    plo[r] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    phi[r] = make_float4(hi[0], hi[1], hi[2], 0.0f);
    // Two-level key: 30-bit Morton code in the scene box of the mesh's centre
    // (a loose triangle's or sphere's own centroid) | mesh id + 1 | Morton
    // code of the centroid inside the mesh's own AABB.  A mesh's triangles
    // stay contiguous (its subtree carries one exact mesh gate, Scene.cs:67,
    // and its small pieces collapse into multi-primitive leaves) while meshes
    // and loose primitives are still ordered spatially at the top.
    const f3 c = mk(cen[0], cen[1], cen[2]);
    unsigned long long key;
    if (gate >= 0) {
        const rtd::MeshGate g = in.gates[gate];
        const float mlo[3] = {g.lo.x, g.lo.y, g.lo.z}, mhi[3] = {g.hi.x, g.hi.y, g.hi.z};
        const f3 mc = mk(0.5f * (mlo[0] + mhi[0]), 0.5f * (mlo[1] + mhi[1]), 0.5f * (mlo[2] + mhi[2]));
        const int low_bits = 34 - in.mesh_bits;
        const int per_axis = low_bits >= 30 ? 10 : low_bits / 3;
        const unsigned long long low = per_axis > 0 ? morton(c, mlo, mhi, per_axis) : 0ull;
        key = ((unsigned long long)morton(mc, scene_lo, scene_hi, 10) << 34) |
              ((unsigned long long)(gate + 1) << low_bits) | low;
    } else {
        key = (unsigned long long)morton(c, scene_lo, scene_hi, 10) << 34;
    }
    keys[r] = key;
    vals[r] = r;
}

__global__ void k_kind(LbvhInput in, int n, const int *sorted_rank, int *is_sph) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = sorted_rank[i];
    is_sph[i] = (r >= in.mt && r < in.mt + in.ns) ? 1 : 0;
}

// 3. leaf-order primitive arrays, inline leaf refs, sorted boxes
__global__ void k_leaves(LbvhInput in, LbvhOutput out, int n, const int *sorted_rank, const int *sph_idx,
                         const rtd::TriRec *tri_rank, const float4 *plo, const float4 *phi, float4 *slo, float4 *shi,
                         int *leaf_ref, int *gate_pos) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) out.tris[in.mt + in.nl] = rtd::sentinel_tri();
    if (i >= n) return;
    const int r = sorted_rank[i];
    const bool sph = r >= in.mt && r < in.mt + in.ns;
    const int si = sph_idx[i];
    if (sph) {
        out.sphs[si] = *(const rtd::SphRec *)&tri_rank[r];
        leaf_ref[i] = rtd::encode_leaf(si, 1, rtd::kLeafSphere);
        gate_pos[i] = -2;  // spheres: never grouped with triangles
    } else {
        const int ti = i - si;
        const rtd::TriRec t = tri_rank[r];
        out.tris[ti] = t;
        leaf_ref[i] = rtd::encode_leaf(ti, 1, rtd::kLeafTri);
        gate_pos[i] = __float_as_int(t.p2.z);
    }
    slo[i] = plo[r];
    shi[i] = phi[r];
}

__device__ __forceinline__ int delta(const unsigned long long *k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const unsigned long long a = k[i], b = k[j];
    if (a == b) return 64 + __clz(i ^ j);
    return __clzll(a ^ b);
}

// 4. Karras 2012: internal node i covers a key range and splits it at the
// highest differing bit; parents recorded as (node << 1 | side).
__global__ void k_karras(int n, int empty_ref, const unsigned long long *k, const int *leaf_ref, const float4 *slo,
                         const float4 *shi, rtd::BvhNode *nodes, int *leaf_parent, int *node_parent, int2 *range) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 1) {
        if (i == 0) {  // lone leaf beside an empty slot (+inf box, sentinel leaf)
            const float4 lo = slo[0], hi = shi[0];
            const float inf = INFINITY;
            rtd::BvhNode nd;
            nd.a = make_float4(lo.x, hi.x, lo.y, hi.y);
            nd.b = make_float4(inf, inf, inf, inf);
            nd.c = make_float4(lo.z, hi.z, inf, inf);
            nd.d = make_int4(leaf_ref[0], empty_ref, 0, 0);
            nodes[0] = nd;
        }
        return;
    }
    if (i >= n - 1) return;
    const int d = delta(k, n, i, i + 1) - delta(k, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int first = min(i, j), last = max(i, j);
    range[i] = make_int2(first, last);
    int left, right;
    if (first == gamma) {
        left = leaf_ref[gamma];
        leaf_parent[gamma] = i << 1;
    } else {
        left = gamma;
        node_parent[gamma] = i << 1;
    }
    if (last == gamma + 1) {
        right = leaf_ref[gamma + 1];
        leaf_parent[gamma + 1] = (i << 1) | 1;
    } else {
        right = gamma + 1;
        node_parent[gamma + 1] = (i << 1) | 1;
    }
    nodes[i].d = make_int4(left, right, 0, 0);
    if (i == 0) node_parent[0] = -1;
}

typedef __attribute__((address_space(1))) unsigned gu32;

// Agent-scope relaxed atomics on global memory compile to sc1 (write-through
// / L2-bypassing) stores and loads: the hand-off between the two children of
// a node needs no release/acquire fence (cdna_hip_programming.md G16; a
// __threadfence() per level wrote back the whole L2 and cost 1.5 ms per
// build at 250k primitives).
__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store((gu32 *)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
    return __uint_as_float(__hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ void write_slot(rtd::BvhNode *nd, int side, float4 lo, float4 hi) {
    float *a = side ? &nd->b.x : &nd->a.x;
    st_sc1(a + 0, lo.x);
    st_sc1(a + 1, hi.x);
    st_sc1(a + 2, lo.y);
    st_sc1(a + 3, hi.y);
    float *c = &nd->c.x + 2 * side;
    st_sc1(c + 0, lo.z);
    st_sc1(c + 1, hi.z);
}

// 5. bottom-up boxes: each child writes its box into its parent's slot
// (sc1 stores, drained), then counts its arrival; the second arrival reads
// the sibling's slot with sc1 loads, unions both and climbs.
__global__ void k_bounds(int n, const float4 *slo, const float4 *shi, const int *leaf_parent,
                         const int *node_parent, rtd::BvhNode *nodes, int *flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (n < 2 || i >= n) return;
    float4 lo = slo[i], hi = shi[i];
    int ps = leaf_parent[i];
    while (ps >= 0) {
        const int p = ps >> 1, side = ps & 1;
        write_slot(&nodes[p], side, lo, hi);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot is visible before the count
        if (__hip_atomic_fetch_add((__attribute__((address_space(1))) int *)&flags[p], 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == 0)
            return;
        const float *o = side ? &nodes[p].a.x : &nodes[p].b.x;  // the sibling's slot
        const float *oc = &nodes[p].c.x + 2 * (1 - side);
        const float4 olo = make_float4(ld_sc1(o + 0), ld_sc1(o + 2), ld_sc1(oc + 0), 0.0f);
        const float4 ohi = make_float4(ld_sc1(o + 1), ld_sc1(o + 3), ld_sc1(oc + 1), 0.0f);
        lo = make_float4(fminf(lo.x, olo.x), fminf(lo.y, olo.y), fminf(lo.z, olo.z), 0.0f);
        hi = make_float4(fmaxf(hi.x, ohi.x), fmaxf(hi.y, ohi.y), fmaxf(hi.z, ohi.z), 0.0f);
        ps = node_parent[p];
    }
}

// 6b. depth of every internal node of the 2-wide tree (climb to the root;
// depths are small): the traversal stack bound of the 2-wide layout.
__global__ void k_depth(int n, const int *node_parent, int *max_depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    int d = 0;
    for (int ps = node_parent[i]; ps >= 0; ps = node_parent[ps >> 1]) ++d;
    // leaves sit one level below their parent
    atomicMax(max_depth, d + 1);
}

__device__ __forceinline__ void read_slot(const rtd::BvhNode &nd, int side, float lo[3], float hi[3]) {
    if (side) {
        lo[0] = nd.b.x; hi[0] = nd.b.y; lo[1] = nd.b.z; hi[1] = nd.b.w; lo[2] = nd.c.z; hi[2] = nd.c.w;
    } else {
        lo[0] = nd.a.x; hi[0] = nd.a.y; lo[1] = nd.a.z; hi[1] = nd.a.w; lo[2] = nd.c.x; hi[2] = nd.c.y;
    }
}

// The (up to) four slots of the 4-wide node made from 2-wide node i: start
// from its two children and expand, twice, the slot of largest surface area
// among the internal children that are not collapsed leaves (first such slot
// on ties) — the rule of the host builder's collapse (bvh.cpp collapse), so
// the root-level slots of big subtrees are split first.  Deterministic, so
// k_keep and k_collapse see the same slots.
struct Slots4 {
    int ref[4];    // 2-wide child refs: >= 0 internal node, < 0 leaf ref
    int start[4];  // first leaf position of each slot (when ranges are given)
    float lo[3][4], hi[3][4];
    int k;
};

__device__ __forceinline__ float half_area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

// 6a. small homogeneous subtrees (<= 4 primitives of one kind and one mesh
// gate, contiguous in leaf order) become one multi-primitive leaf in the
// 4-wide tree — fewer traversal steps, like the host SAH build's leaves —
// when the host builder's leaf rule holds for them (bvh.cpp: n primitive
// tests cost no more than a node step plus the children's area-weighted
// tests, here with the Karras split as the split): a wave packet tests every
// primitive of a leaf it enters on all its lanes, so over-full leaves of
// tiny far-apart triangles cost more than the node step they save.
__global__ void k_small(int n, const int2 *range, const int *gate_pos, const rtd::BvhNode *nodes, int *small) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int2 r = range[i];
    const int cnt = r.y - r.x + 1;
    bool ok = i != 0 && cnt <= kLbvhLeaf;  // the root stays a node
    if (ok) {
        const int g = gate_pos[r.x];
        for (int p = r.x + 1; p <= r.y; ++p) ok = ok && gate_pos[p] == g;
    }
    if (ok && cnt > 1) {
        const rtd::BvhNode nd = nodes[i];
        float l0[3], h0[3], l1[3], h1[3], lp[3], hp[3];
        read_slot(nd, 0, l0, h0);
        read_slot(nd, 1, l1, h1);
        for (int a = 0; a < 3; ++a) {
            lp[a] = fminf(l0[a], l1[a]);
            hp[a] = fmaxf(h0[a], h1[a]);
        }
        const int c0 = nd.d.x >= 0 ? range[nd.d.x].y - range[nd.d.x].x + 1 : 1;
        const float ap = fmaxf(half_area(lp, hp), 1e-30f);
        const float split =
            kLeafNodeCost + (half_area(l0, h0) * (float)c0 + half_area(l1, h1) * (float)(cnt - c0)) / ap;
        ok = (float)cnt <= split;
    }
    small[i] = ok ? 1 : 0;
}

// A slot's first leaf: a left child starts where its parent does; a right
// leaf child is its parent's last leaf (Karras: last == gamma + 1).
__device__ __forceinline__ int slot_start(const int2 *range, int parent, int side, int ref) {
    if (!range) return 0;
    return side == 0 ? range[parent].x : ref >= 0 ? range[ref].x : range[parent].y;
}

__device__ __forceinline__ void expand4(const rtd::BvhNode *nodes, const int *small, const int2 *range,
                                        bool any_internal, int i, Slots4 &S) {
    const rtd::BvhNode nd = nodes[i];
    S.ref[0] = nd.d.x;
    S.ref[1] = nd.d.y;
    S.k = 2;
    for (int s = 0; s < 2; ++s) {
        float l[3], h[3];
        read_slot(nd, s, l, h);
        for (int a = 0; a < 3; ++a) {
            S.lo[a][s] = l[a];
            S.hi[a][s] = h[a];
        }
        S.start[s] = slot_start(range, i, s, S.ref[s]);
    }
    while (any_internal && S.k < 4) {
        int best = -1;
        float best_a = -1.0f;
        for (int s = 0; s < S.k; ++s) {
            const int c = S.ref[s];
            if (c < 0 || small[c]) continue;
            const float l[3] = {S.lo[0][s], S.lo[1][s], S.lo[2][s]}, h[3] = {S.hi[0][s], S.hi[1][s], S.hi[2][s]};
            const float ar = half_area(l, h);
            if (ar > best_a) {
                best_a = ar;
                best = s;
            }
        }
        if (best < 0) break;
        const int p = S.ref[best];
        const rtd::BvhNode cn = nodes[p];
        const int gc[2] = {cn.d.x, cn.d.y}, dst[2] = {best, S.k};
        for (int g = 0; g < 2; ++g) {
            float l[3], h[3];
            read_slot(cn, g, l, h);
            for (int a = 0; a < 3; ++a) {
                S.lo[a][dst[g]] = l[a];
                S.hi[a][dst[g]] = h[a];
            }
            S.ref[dst[g]] = gc[g];
            S.start[dst[g]] = slot_start(range, p, g, gc[g]);
        }
        ++S.k;
    }
}

// 6c. every internal node's slots as if it were kept, sorted by first leaf
// (unused: start INT_MAX) — 32 B per node, so the walk below makes one
// round trip per step instead of re-expanding.
__global__ void k_slots(int n, const rtd::BvhNode *nodes, const int *small, const int2 *range, int4 *rec) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n - 1 || small[x]) return;
    Slots4 S;
    expand4(nodes, small, range, true, x, S);
    int r[4], st[4];
    for (int k = 0; k < 4; ++k) {  // a collapsed-leaf child reads as a leaf (-1): the walk stops there
        r[k] = k < S.k ? (S.ref[k] >= 0 && small[S.ref[k]] ? -1 : S.ref[k]) : -1;
        st[k] = k < S.k ? S.start[k] : INT_MAX;
    }
    for (int a = 1; a < 4; ++a)  // insertion sort by start
        for (int b = a; b > 0 && st[b - 1] > st[b]; --b) {
            const int ts = st[b]; st[b] = st[b - 1]; st[b - 1] = ts;
            const int tr = r[b]; r[b] = r[b - 1]; r[b - 1] = tr;
        }
    rec[2 * x] = make_int4(r[0], r[1], r[2], r[3]);
    rec[2 * x + 1] = make_int4(st[0], st[1], st[2], st[3]);
}

// 6d. which 2-wide nodes become 4-wide nodes: the root, and every internal
// slot (not a collapsed leaf) of a 4-wide node.  Each thread walks from the
// root over 4-wide nodes towards its own node x (the slot whose leaf range
// holds x's first leaf); x is kept when it is that slot, dropped when its
// range spans several slots (it was expanded into the 4-wide node above it)
// or lies inside a collapsed leaf.  Also the 4-wide depth (root 0), which
// bounds the traversal stack.
__global__ void k_keep(int n, const int4 *rec, const int *small, const int2 *range, int *keep, int *depth4) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n - 1) return;
    if (x == 0) {
        keep[0] = 1;
        return;
    }
    const int2 rx = range[x];
    int kept = 0, K = 0, kend = n - 1, lvl = 0;
    if (!small[x]) {
        while (true) {
            const int4 rr = rec[2 * K], ss = rec[2 * K + 1];
            const int r[4] = {rr.x, rr.y, rr.z, rr.w}, st[4] = {ss.x, ss.y, ss.z, ss.w};
            int s = 0;
            for (int k = 1; k < 4; ++k)
                if (st[k] <= rx.x) s = k;
            const int end = s < 3 && st[s + 1] != INT_MAX ? st[s + 1] - 1 : kend;
            const int c = r[s];
            if (c < 0 || rx.y > end) break;  // inside a (collapsed) leaf, or expanded into K's node
            ++lvl;
            if (c == x) {
                kept = 1;
                break;
            }
            K = c;
            kend = end;
        }
    }
    keep[x] = kept;
    if (kept) atomicMax(depth4, lvl);
}

// 7. collapse: every kept node writes its 4-wide node from its expanded
// slots; unused slots get +inf boxes and the sentinel leaf.  Child node refs
// are renumbered by the exclusive scan of the keep flags (the root stays 0).
__global__ void k_collapse(int n, int empty_ref, const rtd::BvhNode *nodes, const int *keep, const int *idx4,
                           const int *small, const int2 *range, const int *sph_idx, const int *is_sph,
                           rtd::BvhNode4 *out, int *info) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) info[1] = n > 1 ? idx4[n - 2] + keep[n - 2] : 1;  // 4-wide node count
    if (i >= (n > 1 ? n - 1 : 1) || (n > 1 && !keep[i])) return;
    // ref of an internal node c seen from a 4-wide node: a multi-primitive
    // leaf when its subtree is small, else its 4-wide index
    auto sub = [&](int c) {
        if (!small[c]) return idx4[c];
        const int2 r = range[c];
        const int f = r.x;
        const int sph = is_sph[f];
        return rtd::encode_leaf(sph ? sph_idx[f] : f - sph_idx[f], r.y - r.x + 1,
                                sph ? rtd::kLeafSphere : rtd::kLeafTri);
    };
    Slots4 S;
    expand4(nodes, small, nullptr, n > 1, i, S);
    for (int k = 0; k < S.k; ++k)
        if (S.ref[k] >= 0 && n > 1) S.ref[k] = sub(S.ref[k]);
    for (int k = S.k; k < 4; ++k) {
        for (int a = 0; a < 3; ++a) {
            S.lo[a][k] = INFINITY;
            S.hi[a][k] = INFINITY;
        }
        S.ref[k] = empty_ref;
    }
    rtd::BvhNode4 o;
    o.lox = make_float4(S.lo[0][0], S.lo[0][1], S.lo[0][2], S.lo[0][3]);
    o.hix = make_float4(S.hi[0][0], S.hi[0][1], S.hi[0][2], S.hi[0][3]);
    o.loy = make_float4(S.lo[1][0], S.lo[1][1], S.lo[1][2], S.lo[1][3]);
    o.hiy = make_float4(S.hi[1][0], S.hi[1][1], S.hi[1][2], S.hi[1][3]);
    o.loz = make_float4(S.lo[2][0], S.lo[2][1], S.lo[2][2], S.lo[2][3]);
    o.hiz = make_float4(S.hi[2][0], S.hi[2][1], S.hi[2][2], S.hi[2][3]);
    o.child = make_int4(S.ref[0], S.ref[1], S.ref[2], S.ref[3]);
    o.pad = make_int4(0, 0, 0, 0);
    out[n > 1 ? idx4[i] : 0] = o;
}

struct Layout {
    size_t keys_a, keys_b, vals_a, vals_b, plo, phi, tri_rank, is_sph, sph_idx, slo, shi, leaf_ref, leaf_parent,
        node_parent, flags, keep, idx4, rec, depth, range, gate_pos, small, cub, total;
    size_t cub_bytes;
};

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

Layout layout(int n) {
    Layout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    L.keys_a = take(sizeof(unsigned long long) * n);
    L.keys_b = take(sizeof(unsigned long long) * n);
    L.vals_a = take(sizeof(int) * n);
    L.vals_b = take(sizeof(int) * n);
    L.plo = take(sizeof(float4) * n);
    L.phi = take(sizeof(float4) * n);
    L.tri_rank = take(sizeof(rtd::TriRec) * n);
    L.is_sph = take(sizeof(int) * n);
    L.sph_idx = take(sizeof(int) * n);
    L.slo = take(sizeof(float4) * n);
    L.shi = take(sizeof(float4) * n);
    L.leaf_ref = take(sizeof(int) * n);
    L.leaf_parent = take(sizeof(int) * n);
    L.node_parent = take(sizeof(int) * n);
    L.flags = take(sizeof(int) * n);
    L.keep = take(sizeof(int) * n);
    L.idx4 = take(sizeof(int) * n);
    L.rec = take(2 * sizeof(int4) * n);
    L.depth = take(3 * sizeof(int));  // 2-wide depth, 4-wide node count, 4-wide depth
    L.range = take(sizeof(int2) * n);
    L.gate_pos = take(sizeof(int) * n);
    L.small = take(sizeof(int) * n);
    size_t sort_bytes = 0, scan_bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (unsigned long long *)nullptr,
                                             (unsigned long long *)nullptr, (int *)nullptr, (int *)nullptr, n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (int *)nullptr, (int *)nullptr, n);
    L.cub_bytes = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    L.cub = take(L.cub_bytes);
    L.total = off;
    return L;
}

}  // namespace

size_t lbvh_scratch_bytes(int n) { return layout(n < 1 ? 1 : n).total; }

const int *lbvh_info_ptr(const void *scratch, int n) {
    return (const int *)((const char *)scratch + layout(n < 1 ? 1 : n).depth);
}

hipError_t build_lbvh_gpu(const LbvhInput &in, const LbvhOutput &out, void *scratch, size_t scratch_bytes,
                          hipStream_t stream) {
    const int n = in.mt + in.ns + in.nl;
    if (n < 1) return hipSuccess;
    const Layout L = layout(n);
    if (scratch_bytes < L.total) return hipErrorInvalidValue;
    char *b = (char *)scratch;
    auto *keys_a = (unsigned long long *)(b + L.keys_a), *keys_b = (unsigned long long *)(b + L.keys_b);
    auto *vals_a = (int *)(b + L.vals_a), *vals_b = (int *)(b + L.vals_b);
    auto *plo = (float4 *)(b + L.plo), *phi = (float4 *)(b + L.phi);
    auto *tri_rank = (rtd::TriRec *)(b + L.tri_rank);
    auto *is_sph = (int *)(b + L.is_sph), *sph_idx = (int *)(b + L.sph_idx);
    auto *slo = (float4 *)(b + L.slo), *shi = (float4 *)(b + L.shi);
    auto *leaf_ref = (int *)(b + L.leaf_ref), *leaf_parent = (int *)(b + L.leaf_parent);
    auto *node_parent = (int *)(b + L.node_parent), *flags = (int *)(b + L.flags);
    auto *range = (int2 *)(b + L.range);
    auto *gate_pos = (int *)(b + L.gate_pos), *small = (int *)(b + L.small);
    void *cub = b + L.cub;

    hipLaunchKernelGGL(k_prims, dim3(blocks_for(n)), dim3(kThreads), 0, stream, in, out, n, plo, phi, keys_a, vals_a,
                       tri_rank);
    size_t cub_bytes = L.cub_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(cub, cub_bytes, keys_a, keys_b, vals_a, vals_b, n, 0,
                                                      in.key_bits, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_kind, dim3(blocks_for(n)), dim3(kThreads), 0, stream, in, n, vals_b, is_sph);
    cub_bytes = L.cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(cub, cub_bytes, is_sph, sph_idx, n, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_leaves, dim3(blocks_for(n)), dim3(kThreads), 0, stream, in, out, n, vals_b, sph_idx,
                       tri_rank, plo, phi, slo, shi, leaf_ref, gate_pos);
    hipLaunchKernelGGL(k_karras, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n,
                       rtd::encode_leaf(in.mt + in.nl, 1, rtd::kLeafTri), keys_b, leaf_ref, slo, shi,
                       out.nodes, leaf_parent, node_parent, range);
    e = hipMemsetAsync(flags, 0, sizeof(int) * n, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bounds, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n, slo, shi, leaf_parent,
                       node_parent, out.nodes, flags);
    int *depth = (int *)(b + L.depth);
    e = hipMemsetAsync(depth, 0, 3 * sizeof(int), stream);
    if (e != hipSuccess) return e;
    if (n > 1) {
        int *keep = (int *)(b + L.keep), *idx4 = (int *)(b + L.idx4);
        if (!out.nodes4)  // the 2-wide stack bound; the 4-wide one comes from k_keep
            hipLaunchKernelGGL(k_depth, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n, node_parent, depth);
        else {
            hipLaunchKernelGGL(k_small, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n, range, gate_pos, out.nodes,
                               small);
            int4 *rec = (int4 *)(b + L.rec);
            hipLaunchKernelGGL(k_slots, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n, out.nodes, small, range,
                               rec);
            hipLaunchKernelGGL(k_keep, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n, rec, small, range, keep,
                               depth + 2);
            cub_bytes = L.cub_bytes;
            e = hipcub::DeviceScan::ExclusiveSum(cub, cub_bytes, keep, idx4, n - 1, stream);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k_collapse, dim3(blocks_for(n)), dim3(kThreads), 0, stream, n,
                               rtd::encode_leaf(in.mt + in.nl, 1, rtd::kLeafTri), out.nodes, keep, idx4, small, range,
                               sph_idx, is_sph, out.nodes4, depth);
        }
    } else if (out.nodes4) {
        hipLaunchKernelGGL(k_collapse, dim3(1), dim3(kThreads), 0, stream, n,
                           rtd::encode_leaf(in.mt + in.nl, 1, rtd::kLeafTri), out.nodes, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr, out.nodes4, depth);
    }
    return hipGetLastError();
}

}  // namespace rtl
