// packet.h — wave-level ("packet") BVH4 traversal for coherent rays.
//
// All 64 lanes of a wave walk ONE path through the BVH: the union of the
// nodes any participating lane needs.  The node index, the stack and the leaf
// contents are wave-uniform, so node and primitive records are fetched once
// per wave with scalar loads, there is no lane divergence in the traversal
// control flow, and the stack is a tiny per-wave LDS array.  Each lane still
// runs the reference's exact tests on its own ray with its own culling
// distance, and keeps its own (t, rank) winner — the visiting order does not
// change the result (minimum distance, ties to the lowest rank), so answers
// equal traverse.h's per-lane traversal and the brute-force reference
// (Scene.cs:43-122).  Used for camera rays of a pixel tile and for their
// shadow rays to a point light, which are highly coherent.
#pragma once

#include <float.h>

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_math.h"
#include "traverse.h"

namespace rtp {

using rtm::f3;
using rtm::mk;
using rtt::Counts;
using rtt::RayCtx;

constexpr int kWaveStack = rtd::kStackTotal;  // 3 entries per BVH4 level

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

__device__ __forceinline__ float wave_key(float k, int rep) {
    if (__ballot(k != INFINITY) == 0) return INFINITY;
    const float kr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(k), rep));
    return kr != INFINITY ? kr : 3.0e38f;
}

// Per-lane outcome of a packet query.
struct PacketLane {
    float best_t;
    int best_rank;  // -1 none; any-hit: 1 = occluded
    float tcull;
    int gate_cached;
    bool gate_ok;
    bool live;      // still needs nodes (any-hit lanes retire on their first occluder)
};

// ANY: shadow query with predicate t*t < d2 (see traverse.h).  `part`: the
// lane takes part.  wstack: this wave's LDS stack (kWaveStack ints).
template <bool ANY, bool COUNT>
__device__ __forceinline__ void packet_trace(const rtd::SceneDev &S, const RayCtx &r, bool part, float tlimit,
                                             float d2, PacketLane &L, int *wstack, Counts &cnt) {
    L.best_t = FLT_MAX;
    L.best_rank = -1;
    L.tcull = ANY ? tlimit : FLT_MAX;
    L.gate_cached = -1;
    L.gate_ok = false;
    if (COUNT && part) cnt.box++;
    L.live = part && S.has_prims && rtm::ref_slab(r.o, r.inv(), rtt::ld3(S.scene_lo), rtt::ld3(S.scene_hi));
    if (__ballot(L.live) == 0) return;
    int node = 0;  // wave-uniform
    int sp = 0;    // wave-uniform
    while (true) {
        if (node >= 0) {
            const rtd::BvhNode4 nd = rtt::cload(S.nodes4 + node);  // scalar loads
            const float4 lx = nd.lox, hx = nd.hix, ly = nd.loy, hy = nd.hiy, lz = nd.loz, hz = nd.hiz;
            const int4 ch = nd.child;
            float k0 = INFINITY, k1 = INFINITY, k2 = INFINITY, k3 = INFINITY;
            if (L.live) {
                k0 = rtt::child_key(lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, r, L.tcull);
                k1 = rtt::child_key(lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, r, L.tcull);
                k2 = rtt::child_key(lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, r, L.tcull);
                k3 = rtt::child_key(lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, r, L.tcull);
                if (COUNT) cnt.box += 4;
            }
            // wave-wide order: children nobody needs get +inf; the others are
            // ordered by the entry distance of a representative live lane
            // (children it misses go last).  Order only affects speed.
            const unsigned long long live_m = __ballot(L.live);
            const int rep = __ffsll((long long)live_m) - 1;
            float q0 = wave_key(k0, rep), q1 = wave_key(k1, rep), q2 = wave_key(k2, rep), q3 = wave_key(k3, rep);
            int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
#define RT_PSWAP(i, j)                            \
    do {                                          \
        if (q##j < q##i) {                        \
            const float tq = q##i;                \
            q##i = q##j;                          \
            q##j = tq;                            \
            const int tc = c##i;                  \
            c##i = c##j;                          \
            c##j = tc;                            \
        }                                         \
    } while (0)
            RT_PSWAP(0, 1);
            RT_PSWAP(2, 3);
            RT_PSWAP(0, 2);
            RT_PSWAP(1, 3);
            RT_PSWAP(1, 2);
#undef RT_PSWAP
            if (q0 != INFINITY) {
                if (q3 != INFINITY) wstack[sp++] = c3;
                if (q2 != INFINITY) wstack[sp++] = c2;
                if (q1 != INFINITY) wstack[sp++] = c1;
                node = uni(c0);
                continue;
            }
        } else {
            const int v = ~node;
            const int first = v & ((1 << rtd::kLeafFirstBits) - 1);
            const int count = ((v >> rtd::kLeafFirstBits) & 3) + 1;
            const int kind = (v >> (rtd::kLeafFirstBits + 2)) & 1;
            const int gate = kind == rtd::kLeafTri ? __float_as_int(rtt::cload(&S.tris[first].p2).z)
                                                   : rtt::cload(&S.sphs[first].misc).y;
            if (L.live) {
                rtt::Trav t;
                t.best_t = L.best_t;
                t.best_rank = L.best_rank;
                t.tcull = L.tcull;
                t.gate_cached = L.gate_cached;
                t.gate_ok = L.gate_ok;
                const bool occ = rtt::leaf<ANY, COUNT, true>(S, r, t, d2, first, count, kind, gate, cnt);
                L.best_t = t.best_t;
                L.best_rank = t.best_rank;
                L.tcull = t.tcull;
                L.gate_cached = t.gate_cached;
                L.gate_ok = t.gate_ok;
                if (ANY && occ) L.live = false;
            }
            if (ANY && __ballot(L.live) == 0) return;
        }
        if (sp == 0) return;
        node = uni(wstack[--sp]);
    }
}

}  // namespace rtp
