// traverse.h — device-side BVH traversal shared by the megakernel
// (trace.hip) and the wavefront kernels (trace_wf.hip).
//
// Scene.IntersectRay (Data/Objects/Scene.cs:43-122) over the BVH of
// rt_device.h.  Results equal the brute-force scan: same candidate set (the
// exact scene and per-mesh AABB gates, padded node boxes), same winner
// (lowest distance, ties to the lowest reference rank).
#pragma once

#include <float.h>

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_math.h"

namespace rtt {

using rtd::kWaveSize;
using rtm::f3;
using rtm::mk;

struct Counts {
    unsigned primary, shadow, reflection, box, tri, sph, shading;
    unsigned scene_miss;  // camera samples rejected by the scene AABB gate (Scene.cs:54), COUNT launches
    unsigned moot;        // shadow rays whose answer cannot change the colour: not traced (shade.h same_bits)
#ifdef RT_FETCH_COUNT
    unsigned fetch;       // measuring builds: bytes requested (RT_FETCH_*)
#endif
};

// Measuring builds (-DRT_FETCH_COUNT, lib/variants/fetch; tools/fetch_bytes.py,
// bench.py roofline.fetched_bytes_per_launch): the bytes a frame's traversal
// and shading request from the cache hierarchy — a node (128 B), triangle
// (48 B), sphere (32 B) or mesh-gate (32 B) record, a cut box (32 B), the cut
// table (1,796 B), a shading record (16 B), a material (64 B), a light (32 B),
// a tile index (4 B).  A wave-uniform fetch (a packet's scalar loads) counts
// once per wave (RT_FETCH_WAVE: by its first active lane), a per-lane fetch
// once per lane (RT_FETCH_LANE).  The product build compiles none of it.
#ifdef RT_FETCH_COUNT
__device__ __forceinline__ bool fetch_lead() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l == __ffsll((long long)__ballot(1)) - 1;
}
#define RT_FETCH_LANE(c, n) ((c).fetch += (unsigned)(n))
#define RT_FETCH_WAVE(c, n) ((c).fetch += rtt::fetch_lead() ? (unsigned)(n) : 0u)
#else
#define RT_FETCH_LANE(c, n) ((void)0)
#define RT_FETCH_WAVE(c, n) ((void)0)
#endif

__device__ __forceinline__ float nudge(float v) { return fabsf(v) > 1e-20f ? v : copysignf(1e-20f, v); }

struct RayCtx {
    f3 o, d;     // exact ray (reference semantics)
    f3 ninv;     // node-test inverse (zero components nudged, approximate rcp)
    f3 inv_v;    // rcp(dir) = 1.0f / dir, exact — the reference's AABB gates
    f3 noi_v;    // o * ninv
    __device__ __forceinline__ f3 inv() const { return inv_v; }
    __device__ __forceinline__ f3 noi() const { return noi_v; }
};

__device__ __forceinline__ void setup_ray(RayCtx &r, f3 o, f3 d) {
    r.o = o;
    r.d = d;
    r.ninv = mk(__builtin_amdgcn_rcpf(nudge(d.x)), __builtin_amdgcn_rcpf(nudge(d.y)),
                __builtin_amdgcn_rcpf(nudge(d.z)));
    r.inv_v = mk(rtm::rcp_cr(d.x), rtm::rcp_cr(d.y), rtm::rcp_cr(d.z));
    r.noi_v = mk(o.x * r.ninv.x, o.y * r.ninv.y, o.z * r.ninv.z);
}

__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

// Load through the constant address space: with a wave-uniform address the
// backend emits a scalar (SMEM) load — one fetch per wave into SGPRs.
typedef const __attribute__((address_space(4))) int *const_i32_ptr;

template <typename T>
__device__ __forceinline__ T cload(const T *p) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized records only");
    const_i32_ptr q = (const_i32_ptr)p;
    union {
        T v;
        int w[sizeof(T) / 4];
    } u;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) u.w[i] = q[i];
    return u.v;
}

// Conservative slab test of both children of a node (padded boxes; FMA form).
__device__ __forceinline__ void test_children(const float4 a, const float4 b, const float4 c, const RayCtx &r,
                                              float tcull, bool &h0, bool &h1, float &tn0, float &tn1) {
    const f3 noi = r.noi();
    const float l0x = fmaf(a.x, r.ninv.x, -noi.x), u0x = fmaf(a.y, r.ninv.x, -noi.x);
    const float l0y = fmaf(a.z, r.ninv.y, -noi.y), u0y = fmaf(a.w, r.ninv.y, -noi.y);
    const float l0z = fmaf(c.x, r.ninv.z, -noi.z), u0z = fmaf(c.y, r.ninv.z, -noi.z);
    const float l1x = fmaf(b.x, r.ninv.x, -noi.x), u1x = fmaf(b.y, r.ninv.x, -noi.x);
    const float l1y = fmaf(b.z, r.ninv.y, -noi.y), u1y = fmaf(b.w, r.ninv.y, -noi.y);
    const float l1z = fmaf(c.z, r.ninv.z, -noi.z), u1z = fmaf(c.w, r.ninv.z, -noi.z);
    tn0 = fmaxf(fmaxf(fminf(l0x, u0x), fminf(l0y, u0y)), fmaxf(fminf(l0z, u0z), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(l0x, u0x), fmaxf(l0y, u0y)), fminf(fmaxf(l0z, u0z), tcull));
    tn1 = fmaxf(fmaxf(fminf(l1x, u1x), fminf(l1y, u1y)), fmaxf(fminf(l1z, u1z), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(l1x, u1x), fmaxf(l1y, u1y)), fminf(fmaxf(l1z, u1z), tcull));
    h0 = tn0 <= tf0;
    h1 = tn1 <= tf1;
}

// Resumable traversal state of one lane.  The stack is hybrid: the first
// kStackSize entries live in LDS (st, stride 64 lanes), deeper ones in a
// private (scratch) array that only very deep trees ever touch.
struct Trav {
    int node;         // current node (>= 0 internal, < 0 leaf ref)
    int sp;           // stack depth
    float tcull;      // node culling distance (closest: best_t; any: light distance bound)
    float best_t;     // float.MaxValue until the first hit (Scene.cs:45)
    int best_rank;    // -1 none; any-hit: 1 = occluded
    int gate_cached;  // last mesh whose exact AABB gate was evaluated
    bool gate_ok;
};

// Lane stack: LDS part (stride 64 lanes) + private overflow.  The overflow is
// accessed through a volatile pointer so the compiler can never fold the two
// loads into one generic (flat) load, and it lives outside Trav so the
// traversal state stays in registers.
struct Stack {
    int *lds;
    int *ovf;
    int n = rtd::kStackSize;  // entries in LDS (a constant of the kernel instance)
};

// Overflow accesses are volatile so the compiler never folds the LDS and
// private loads into one generic (flat) load.
typedef volatile int ovf_int;

__device__ __forceinline__ void push(Trav &t, const Stack &st, int v) {
    if (t.sp < st.n)
        st.lds[t.sp * kWaveSize] = v;
    else
        ((ovf_int *)st.ovf)[t.sp - st.n] = v;
    ++t.sp;
}

// false when the stack is empty
__device__ __forceinline__ bool pop(Trav &t, const Stack &st) {
    if (t.sp == 0) return false;
    --t.sp;
    if (t.sp < st.n)
        t.node = st.lds[t.sp * kWaveSize];
    else
        t.node = ((ovf_int *)st.ovf)[t.sp - st.n];
    return true;
}

// Starts a query.  Returns false when the ray misses the exact scene AABB
// gate (Scene.cs:54) — the query is then complete (miss).
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool trav_begin(const rtd::SceneDev &S, const RayCtx &r, float tlimit, Trav &t,
                                           Counts &cnt) {
    t.node = 0;
    t.sp = 0;
    t.best_t = FLT_MAX;
    t.best_rank = -1;
    t.tcull = ANY ? tlimit : FLT_MAX;
    t.gate_cached = -1;
    t.gate_ok = false;
    if (COUNT) cnt.box++;
    return S.has_prims && rtm::ref_slab(r.o, r.inv(), ld3(S.scene_lo), ld3(S.scene_hi));
}

// Primitive tests of one leaf (first, count, kind) behind the reference's
// per-mesh AABB gate (Scene.cs:67).  ANY: returns true on an occluder.
template <bool ANY, bool COUNT, bool UNIFORM = false>
__device__ __forceinline__ bool leaf(const rtd::SceneDev &S, const RayCtx &r, Trav &t, float d2, int first,
                                     int count, int kind, int gate, Counts &cnt) {
    if (gate >= 0) {
        if (gate != t.gate_cached) {
            t.gate_cached = gate;
            const rtd::MeshGate g = S.gates[gate];
            t.gate_ok = rtm::ref_slab(r.o, r.inv(), mk(g.lo.x, g.lo.y, g.lo.z), mk(g.hi.x, g.hi.y, g.hi.z));
            if (COUNT) cnt.box++;
            if (UNIFORM) RT_FETCH_WAVE(cnt, 32); else RT_FETCH_LANE(cnt, 32);
        }
        if (!t.gate_ok) return false;
    }
    if (UNIFORM) RT_FETCH_WAVE(cnt, (kind == rtd::kLeafTri ? 48 : 32) * count);
    else RT_FETCH_LANE(cnt, (kind == rtd::kLeafTri ? 48 : 32) * count);
    if (kind == rtd::kLeafTri) {
        for (int i = 0; i < count; ++i) {
            const rtd::TriRec tr = UNIFORM ? cload(S.tris + first + i) : S.tris[first + i];
            float th;
            if (COUNT) cnt.tri++;
            if (rtm::ref_triangle(r.o, r.d, mk(tr.p0.x, tr.p0.y, tr.p0.z), mk(tr.p0.w, tr.p1.x, tr.p1.y),
                                  mk(tr.p1.z, tr.p1.w, tr.p2.x), th)) {
                const int rank = __float_as_int(tr.p2.y);
                if (ANY) {
                    if (th * th < d2) {
                        t.best_rank = 1;
                        return true;
                    }
                } else if (th < t.best_t || (th == t.best_t && rank < t.best_rank)) {
                    t.best_t = th;
                    t.best_rank = rank;
                    t.tcull = th;
                }
            }
        }
    } else {
        for (int i = 0; i < count; ++i) {
            const rtd::SphRec sr = UNIFORM ? cload(S.sphs + first + i) : S.sphs[first + i];
            float th;
            if (COUNT) cnt.sph++;
            if (rtm::ref_sphere(r.o, r.d, mk(sr.cr.x, sr.cr.y, sr.cr.z), sr.cr.w, th)) {
                const int rank = sr.misc.x;
                if (ANY) {
                    if (th * th < d2) {
                        t.best_rank = 1;
                        return true;
                    }
                } else if (th < t.best_t || (th == t.best_t && rank < t.best_rank)) {
                    t.best_t = th;
                    t.best_rank = rank;
                    t.tcull = th;
                }
            }
        }
    }
    return false;
}

// One triangle record against the lane's ray; true = any-hit occluder found.
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool tri_rec(const RayCtx &r, Trav &t, float d2, const rtd::TriRec &tr, Counts &cnt) {
    float th;
    if (COUNT) cnt.tri++;
    if (rtm::ref_triangle(r.o, r.d, mk(tr.p0.x, tr.p0.y, tr.p0.z), mk(tr.p0.w, tr.p1.x, tr.p1.y),
                          mk(tr.p1.z, tr.p1.w, tr.p2.x), th)) {
        const int rank = __float_as_int(tr.p2.y);
        if (ANY) {
            if (th * th < d2) {
                t.best_rank = 1;
                return true;
            }
        } else if (th < t.best_t || (th == t.best_t && rank < t.best_rank)) {
            t.best_t = th;
            t.best_rank = rank;
            t.tcull = th;
        }
    }
    return false;
}

// Triangle leaf with the records fetched in pairs (indices clamped to the
// leaf, so the loads are unconditional and issue back to back): one memory
// latency per pair of triangles instead of one per triangle; the gate comes
// from the first record.
template <bool ANY, bool COUNT, bool MESH_ONLY = false>
__device__ __forceinline__ bool leaf_tris_batched(const rtd::SceneDev &S, const RayCtx &r, Trav &t, float d2,
                                                  int first, int count, Counts &cnt) {
    const rtd::TriRec *b = S.tris + first;
    const rtd::TriRec t0 = b[0];
    const rtd::TriRec t1 = b[count > 1 ? 1 : 0];
    const int gate = __float_as_int(t0.p2.z);
    RT_FETCH_LANE(cnt, 48 * (count > 2 ? 2 : count));
    if (MESH_ONLY && gate < 0) return false;  // a loose-triangle leaf (leaves are homogeneous in mesh)
    if (gate >= 0) {
        if (gate != t.gate_cached) {
            t.gate_cached = gate;
            const rtd::MeshGate g = S.gates[gate];
            t.gate_ok = rtm::ref_slab(r.o, r.inv(), mk(g.lo.x, g.lo.y, g.lo.z), mk(g.hi.x, g.hi.y, g.hi.z));
            if (COUNT) cnt.box++;
            RT_FETCH_LANE(cnt, 32);
        }
        if (!t.gate_ok) return false;
    }
    if (tri_rec<ANY, COUNT>(r, t, d2, t0, cnt)) return true;
    if (count > 1 && tri_rec<ANY, COUNT>(r, t, d2, t1, cnt)) return true;
    if (count > 2) {  // the second pair, fetched together after the first
        RT_FETCH_LANE(cnt, 48 * (count - 2));
        const rtd::TriRec t2 = b[2];
        const rtd::TriRec t3 = b[count > 3 ? 3 : 2];
        if (tri_rec<ANY, COUNT>(r, t, d2, t2, cnt)) return true;
        if (count > 3 && tri_rec<ANY, COUNT>(r, t, d2, t3, cnt)) return true;
    }
    return false;
}


// Conservative slab test of one child of a 4-wide node: its entry distance,
// or +inf when culled.
__device__ __forceinline__ float child_key(float lx, float hx, float ly, float hy, float lz, float hz,
                                           const RayCtx &r, float tcull) {
    const f3 noi = r.noi();
    const float ax = fmaf(lx, r.ninv.x, -noi.x), bx = fmaf(hx, r.ninv.x, -noi.x);
    const float ay = fmaf(ly, r.ninv.y, -noi.y), by = fmaf(hy, r.ninv.y, -noi.y);
    const float az = fmaf(lz, r.ninv.z, -noi.z), bz = fmaf(hz, r.ninv.z, -noi.z);
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tcull));
    return tn <= tf ? tn : INFINITY;
}

// child_key in exact arithmetic, (plane - o) * (1.0f / d) rounded per IEEE
// operation: the node test of the counting launch (RT_FLAG_COUNT_TESTS), whose
// box/triangle/sphere counts are the canonical per-frame counts SURVEY §8(d)
// prices — the CPU oracle's traversal of the same exported tree computes the
// identical values (oracle/rt_oracle.c bvh4_query), so the two walks visit
// the same nodes in the same order and their counts must agree exactly.
__device__ __forceinline__ float child_key_exact(float lx, float hx, float ly, float hy, float lz, float hz,
                                                 const RayCtx &r, float tcull) {
    const f3 o = r.o, iv = r.inv();
    const float ax = (lx - o.x) * iv.x, bx = (hx - o.x) * iv.x;
    const float ay = (ly - o.y) * iv.y, by = (hy - o.y) * iv.y;
    const float az = (lz - o.z) * iv.z, bz = (hz - o.z) * iv.z;
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tcull));
    return tn <= tf ? tn : INFINITY;
}

// child_key with the near/far planes already chosen by the ray's direction
// signs (near = lo for a positive inverse direction): max/min of the same
// plane distances, so the same result in fewer instructions.
__device__ __forceinline__ float child_key_nf(float nx, float fx, float ny, float fy, float nz, float fz,
                                              const RayCtx &r, float tcull) {
    const f3 noi = r.noi();
    const float an = fmaf(nx, r.ninv.x, -noi.x), af = fmaf(fx, r.ninv.x, -noi.x);
    const float bn = fmaf(ny, r.ninv.y, -noi.y), bf = fmaf(fy, r.ninv.y, -noi.y);
    const float cn = fmaf(nz, r.ninv.z, -noi.z), cf = fmaf(fz, r.ninv.z, -noi.z);
    const float tn = fmaxf(fmaxf(fmaxf(an, bn), cn), 0.0f);
    const float tf = fminf(fminf(fminf(af, bf), cf), tcull);
    return tn <= tf ? tn : INFINITY;
}

#define RT_CSWAP(i, j)                          \
    do {                                        \
        const bool sw_ = k##j < k##i;           \
        const float tk_ = sw_ ? k##j : k##i;    \
        k##j = sw_ ? k##i : k##j;               \
        k##i = tk_;                             \
        const int tr_ = sw_ ? c##j : c##i;      \
        c##j = sw_ ? c##i : c##j;               \
        c##i = tr_;                             \
    } while (0)

// One traversal step: an internal node (test its children, descend into the
// nearest, push the others far-first) or a leaf, then pop if needed.
// Returns true when the query is complete.  ANY: t.best_rank = 1 iff a hit
// with t*t < d2 exists — equivalent to the reference's closest-hit-then-
// compare (RayTracingSetup.cs:333-345) since t >= 0 makes t -> t*t monotone.
// MESH_ONLY: closest hit among mesh triangles only (sphere and loose-triangle
// leaves skipped) — the running winner of the reference's mesh loop, whose
// MeshIndex survives a later sphere/loose-triangle win (Scene.cs:64-85,94-97).
template <bool ANY, bool COUNT, bool MESH_ONLY = false>
__device__ __forceinline__ bool trav_step(const rtd::SceneDev &S, const RayCtx &r, Trav &t, float d2,
                                          const Stack &st, Counts &cnt) {
    if (t.node >= 0 && S.bvh4) {
        RT_FETCH_LANE(cnt, 128);
        const rtd::BvhNode4 *np = S.nodes4 + t.node;
        const float4 lx = np->lox, hx = np->hix, ly = np->loy, hy = np->hiy, lz = np->loz, hz = np->hiz;
        const int4 ch = np->child;
        float k0, k1, k2, k3;
        if (COUNT) {  // the canonical counts' exact node test (child_key_exact)
            k0 = child_key_exact(lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, r, t.tcull);
            k1 = child_key_exact(lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, r, t.tcull);
            k2 = child_key_exact(lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, r, t.tcull);
            k3 = child_key_exact(lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, r, t.tcull);
        } else {
            k0 = child_key(lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, r, t.tcull);
            k1 = child_key(lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, r, t.tcull);
            k2 = child_key(lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, r, t.tcull);
            k3 = child_key(lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, r, t.tcull);
        }
        if (COUNT) cnt.box += 4;
        int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
        RT_CSWAP(0, 1);  // sort the four keys (5 compare-swaps)
        RT_CSWAP(2, 3);
        RT_CSWAP(0, 2);
        RT_CSWAP(1, 3);
        RT_CSWAP(1, 2);
        if (k0 != INFINITY) {
            // push the other hit children far-first: bottom..top = c_{h-1} .. c1
            const int h = 1 + (k1 != INFINITY) + (k2 != INFINITY) + (k3 != INFINITY);
            if (t.sp + 3 <= st.n) {
                // branch-free: three unconditional LDS writes, sp advances by h-1
                const int s0 = h == 4 ? c3 : (h == 3 ? c2 : c1);
                const int s1 = h == 4 ? c2 : c1;
                int *p = st.lds + t.sp * kWaveSize;
                p[0] = s0;
                p[kWaveSize] = s1;
                p[2 * kWaveSize] = c1;
                t.sp += h - 1;
            } else {
                if (h >= 4) push(t, st, c3);
                if (h >= 3) push(t, st, c2);
                if (h >= 2) push(t, st, c1);
            }
            t.node = c0;
            return false;
        }
    } else if (t.node >= 0) {
        RT_FETCH_LANE(cnt, 64);
        const rtd::BvhNode *np = S.nodes + t.node;
        const float4 a = np->a, b = np->b, c = np->c;
        const int4 ch = np->d;
        bool h0, h1;
        float tn0, tn1;
        test_children(a, b, c, r, t.tcull, h0, h1, tn0, tn1);
        if (COUNT) cnt.box += 2;
        if (h0 && h1) {
            const bool first0 = tn0 <= tn1;
            push(t, st, first0 ? ch.y : ch.x);
            t.node = first0 ? ch.x : ch.y;
            return false;
        }
        if (h0 || h1) {
            t.node = h0 ? ch.x : ch.y;
            return false;
        }
    } else {
        const int v = ~t.node;
        const int first = v & ((1 << rtd::kLeafFirstBits) - 1);
        const int count = ((v >> rtd::kLeafFirstBits) & 3) + 1;
        const int kind = (v >> (rtd::kLeafFirstBits + 2)) & 1;
        if (kind == rtd::kLeafTri) {
            if (leaf_tris_batched<ANY, COUNT, MESH_ONLY>(S, r, t, d2, first, count, cnt)) return true;
        } else if (!MESH_ONLY) {
            const int gate = kind == rtd::kLeafTri ? __float_as_int(S.tris[first].p2.z) : S.sphs[first].misc.y;
            if (leaf<ANY, COUNT>(S, r, t, d2, first, count, kind, gate, cnt)) return true;
        }
    }
    return !pop(t, st);
}

#undef RT_CSWAP

// The lane id, through an opaque v_mbcnt pair: the compiler cannot keep a
// copy of it (or of anything derived from it) live across a long trace, where
// it would be spilled — it is recomputed where used (2 VALU).
__device__ __forceinline__ int lane_id() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Whole query in one call (megakernel / batch-intersect path).  `wave_st.lds`
// is the wave's LDS stack base; the lane's column is added here, per query.
template <bool ANY, bool COUNT, bool MESH_ONLY = false>
__device__ __forceinline__ bool traverse(const rtd::SceneDev &S, const RayCtx &r, float tlimit, float d2,
                                         float &best_t, int &best_rank, const Stack &wave_st, Counts &cnt) {
    Trav t;
    if (!trav_begin<ANY, COUNT>(S, r, tlimit, t, cnt)) {
        best_t = FLT_MAX;
        best_rank = -1;
        return false;
    }
    // the instance's LDS depth travels with the stack (the 5-wave instances
    // hold kStackShard entries in LDS and size their overflow for that)
    const Stack st{wave_st.lds + lane_id(), wave_st.ovf, wave_st.n};
    while (!trav_step<ANY, COUNT, MESH_ONLY>(S, r, t, d2, st, cnt)) {
    }
    best_t = t.best_t;
    best_rank = t.best_rank;
    return best_rank >= 0;
}

// Sum over the wave.  With every lane active (the kernels' epilogues) a DPP
// reduction (no LDS round trips); otherwise cross-lane shuffles.
__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    if (__ballot(1) == ~0ull) return __reduce_add_sync(~0ull, v);
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// The wave's sharded counter slot (rt_stats order, rt_device.h).
__device__ __forceinline__ unsigned long long *counter_slot(unsigned long long *counters) {
    return counters + (size_t)(blockIdx.x % rtd::kCounterSlots) * rtd::kCounterWords;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counts(const Counts &c, unsigned long long *counters) {
    // a wave whose rays were all counted already (or none): no reductions, no
    // atomics — a wave's slot is held until its atomics are acknowledged
    if (!COUNT && __ballot((c.primary | c.shadow | c.reflection | c.moot) != 0) == 0) return;
    unsigned long long *ctr = counter_slot(counters);
    const unsigned p = wave_sum(c.primary), s = wave_sum(c.shadow), r = wave_sum(c.reflection),
                   m = wave_sum(c.moot);
    unsigned b = 0, t = 0, q = 0, h = 0, g = 0;
    if (COUNT) {
        b = wave_sum(c.box);
        t = wave_sum(c.tri);
        q = wave_sum(c.sph);
        h = wave_sum(c.shading);
        g = wave_sum(c.scene_miss);
    }
    if ((threadIdx.x & 63) == 0) {
        if (p) atomicAdd(ctr + 0, (unsigned long long)p);
        if (s) atomicAdd(ctr + 1, (unsigned long long)s);
        if (r) atomicAdd(ctr + 2, (unsigned long long)r);
        if (m) atomicAdd(ctr + 8, (unsigned long long)m);
        if (COUNT) {
            if (b) atomicAdd(ctr + 3, (unsigned long long)b);
            if (t) atomicAdd(ctr + 4, (unsigned long long)t);
            if (q) atomicAdd(ctr + 5, (unsigned long long)q);
            if (h) atomicAdd(ctr + 6, (unsigned long long)h);
            if (g) atomicAdd(ctr + 7, (unsigned long long)g);
        }
    }
}

}  // namespace rtt
