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

// Wave-wide sort key of one child (bits of a float >= 0): +inf bits when no
// lane needs it, the representative lane's entry distance when it hits,
// FLT_MAX bits when only other lanes do.
constexpr unsigned kKeyNone = 0x7f800000u;
__device__ __forceinline__ unsigned wave_key_bits(float k, int rep) {
    const unsigned long long need = __ballot(k != INFINITY);
    const unsigned kr = (unsigned)__builtin_amdgcn_readlane(__float_as_int(k), rep);
    return need == 0 ? kKeyNone : (kr != kKeyNone ? kr : 0x7f7fffffu);
}

// Per-lane outcome of a packet query.
struct PacketLane {
    float best_t;
    int best_rank;  // -1 none; any-hit: 1 = occluded
    float tcull;
    int gate_cached;
    bool gate_ok;
    bool live;      // still needs nodes (any-hit lanes retire on their first occluder)
#ifdef RT_SEG_PROFILE
    unsigned nodes, leaves;  // wave-level visits (profiling builds)
#endif
};

// One triangle record against a packet lane's ray (reference MT test);
// true = any-hit occluder.
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool packet_tri(const RayCtx &r, PacketLane &L, float d2, const rtd::TriRec &tr,
                                           Counts &cnt) {
    float th;
    if (COUNT) cnt.tri++;
    if (rtm::ref_triangle(r.o, r.d, mk(tr.p0.x, tr.p0.y, tr.p0.z), mk(tr.p0.w, tr.p1.x, tr.p1.y),
                          mk(tr.p1.z, tr.p1.w, tr.p2.x), th)) {
        const int rank = __float_as_int(tr.p2.y);
        if (ANY) {
            if (th * th < d2) {
                L.best_rank = 1;
                return true;
            }
        } else if (th < L.best_t || (th == L.best_t && rank < L.best_rank)) {
            L.best_t = th;
            L.best_rank = rank;
            L.tcull = th;
        }
    }
    return false;
}

// Triangle leaf of a packet: records fetched with scalar loads two at a time
// (indices clamped to the leaf, so the loads issue back to back), the mesh
// gate (Scene.cs:67) evaluated by every live lane when the wave enters a
// different mesh.  Same tests in the same order as rtt::leaf.
template <bool ANY, bool COUNT>
__device__ __forceinline__ void packet_leaf_tris(const rtd::SceneDev &S, const RayCtx &r, PacketLane &L, int &wgate,
                                                 float d2, int first, int count, Counts &cnt) {
    const rtd::TriRec *tb = S.tris + first;
    const rtd::TriRec t0 = rtt::cload(tb);
    const rtd::TriRec t1 = rtt::cload(tb + (count > 1 ? 1 : 0));
    const int gate = uni(__float_as_int(t0.p2.z));
    if (gate >= 0 && gate != wgate) {
        const rtd::MeshGate g = rtt::cload(S.gates + gate);
        if (L.live) {
            L.gate_ok = rtm::ref_slab(r.o, r.inv(), mk(g.lo.x, g.lo.y, g.lo.z), mk(g.hi.x, g.hi.y, g.hi.z));
            L.gate_cached = gate;
            if (COUNT) cnt.box++;
        }
        wgate = gate;
    }
    if (!L.live || (gate >= 0 && !L.gate_ok)) return;
    if (packet_tri<ANY, COUNT>(r, L, d2, t0, cnt)) { L.live = false; return; }
    if (count > 1 && packet_tri<ANY, COUNT>(r, L, d2, t1, cnt)) { L.live = false; return; }
    if (count > 2) {
        const rtd::TriRec t2 = rtt::cload(tb + 2);
        const rtd::TriRec t3 = rtt::cload(tb + (count > 3 ? 3 : 2));
        if (packet_tri<ANY, COUNT>(r, L, d2, t2, cnt)) { L.live = false; return; }
        if (count > 3 && packet_tri<ANY, COUNT>(r, L, d2, t3, cnt)) { L.live = false; return; }
    }
}

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
#ifdef RT_SEG_PROFILE
    L.nodes = 0;
    L.leaves = 0;
#endif
    if (COUNT && part) cnt.box++;
    L.live = part && S.has_prims && rtm::ref_slab(r.o, r.inv(), rtt::ld3(S.scene_lo), rtt::ld3(S.scene_hi));
    if (__ballot(L.live) == 0) return;
    int node = 0;  // wave-uniform
    int sp = 0;    // wave-uniform
    int wgate = -2;  // mesh whose gate every live lane has evaluated (gate_ok), wave-uniform
    // the top entry of the wave stack is held in a register (all lanes the
    // same value); a pop hands it over at once and refills it from LDS, so
    // the LDS read overlaps the next node fetch instead of preceding it
    int topv = 0;
#define RT_PK_PUSH(v)                               \
    do {                                            \
        if (sp > 0) wstack[sp - 1] = topv;          \
        topv = (v);                                 \
        ++sp;                                       \
    } while (0)
    // direction signs of the live lanes: uniform for most packets (camera
    // tiles, shadow rays of a tile towards one light)
    const unsigned long long live0 = __ballot(L.live);
    const unsigned long long mx = __ballot(L.live && r.ninv.x < 0.0f), my = __ballot(L.live && r.ninv.y < 0.0f),
                             mz = __ballot(L.live && r.ninv.z < 0.0f);
    const bool same_signs = (mx == 0 || mx == live0) && (my == 0 || my == live0) && (mz == 0 || mz == live0);
    // plane-row offsets in the node (lo, hi per axis): near row first
    const int ox = uni(same_signs && mx != 0), oy = uni(same_signs && my != 0), oz = uni(same_signs && mz != 0);
    while (true) {
#ifdef RT_SEG_PROFILE
        if (node >= 0) L.nodes++; else L.leaves++;
#endif
        if (node >= 0) {
            float k0 = INFINITY, k1 = INFINITY, k2 = INFINITY, k3 = INFINITY;
            const int4 ch = rtt::cload(&S.nodes4[node].child);
            if (same_signs) {
                // the near and far plane rows of each axis are fetched
                // directly (scalar loads at per-wave offsets), then 3 FMA +
                // max3/min3 per child: the same entry/exit values as the
                // min/max form (FMA is monotone in the plane value)
                const float4 *pl = reinterpret_cast<const float4 *>(S.nodes4 + node);
                const float4 nx = rtt::cload(pl + ox), fx = rtt::cload(pl + (1 - ox));
                const float4 ny = rtt::cload(pl + 2 + oy), fy = rtt::cload(pl + (3 - oy));
                const float4 nz = rtt::cload(pl + 4 + oz), fz = rtt::cload(pl + (5 - oz));
                if (L.live) {
                    k0 = rtt::child_key_nf(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x, r, L.tcull);
                    k1 = rtt::child_key_nf(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y, r, L.tcull);
                    k2 = rtt::child_key_nf(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z, r, L.tcull);
                    k3 = rtt::child_key_nf(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w, r, L.tcull);
                    if (COUNT) cnt.box += 4;
                }
            } else {
                const rtd::BvhNode4 nd = rtt::cload(S.nodes4 + node);
                if (L.live) {
                    k0 = rtt::child_key(nd.lox.x, nd.hix.x, nd.loy.x, nd.hiy.x, nd.loz.x, nd.hiz.x, r, L.tcull);
                    k1 = rtt::child_key(nd.lox.y, nd.hix.y, nd.loy.y, nd.hiy.y, nd.loz.y, nd.hiz.y, r, L.tcull);
                    k2 = rtt::child_key(nd.lox.z, nd.hix.z, nd.loy.z, nd.hiy.z, nd.loz.z, nd.hiz.z, r, L.tcull);
                    k3 = rtt::child_key(nd.lox.w, nd.hix.w, nd.loy.w, nd.hiy.w, nd.loz.w, nd.hiz.w, r, L.tcull);
                    if (COUNT) cnt.box += 4;
                }
            }
            if (ANY) {
                // any-hit (shadow rays): the order cannot change the answer,
                // so the children any live lane needs are taken in slot order
                // without the wave-wide sort (C3 -6 %, C2 -3 %, C5 +-0)
                const bool n0 = __ballot(k0 != INFINITY) != 0, n1 = __ballot(k1 != INFINITY) != 0,
                           n2 = __ballot(k2 != INFINITY) != 0, n3 = __ballot(k3 != INFINITY) != 0;
                int nn = 0, nxt = 0;
                if (n3) { nxt = ch.w; ++nn; }
                if (n2) { if (nn) RT_PK_PUSH(nxt); nxt = ch.z; ++nn; }
                if (n1) { if (nn) RT_PK_PUSH(nxt); nxt = ch.y; ++nn; }
                if (n0) { if (nn) RT_PK_PUSH(nxt); nxt = ch.x; ++nn; }
                if (nn) {
                    node = uni(nxt);
                    continue;
                }
            } else {
            // closest hit, wave-wide order: children nobody needs get +inf;
            // the others are ordered by the entry distance of a
            // representative live lane (children it misses go last).  Order
            // only affects speed.  Keys are >= 0, so their bit patterns order
            // as unsigned integers and the whole ordering runs on the scalar
            // unit.
            const unsigned long long live_m = __ballot(L.live);
            const int rep = __ffsll((long long)live_m) - 1;
            unsigned q0 = wave_key_bits(k0, rep), q1 = wave_key_bits(k1, rep), q2 = wave_key_bits(k2, rep),
                     q3 = wave_key_bits(k3, rep);
            int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
#define RT_PSWAP(i, j)                            \
    do {                                          \
        const bool sw_ = q##j < q##i;             \
        const unsigned tq_ = sw_ ? q##j : q##i;   \
        q##j = sw_ ? q##i : q##j;                 \
        q##i = tq_;                               \
        const int tc_ = sw_ ? c##j : c##i;        \
        c##j = sw_ ? c##i : c##j;                 \
        c##i = tc_;                               \
    } while (0)
            RT_PSWAP(0, 1);
            RT_PSWAP(2, 3);
            RT_PSWAP(0, 2);
            RT_PSWAP(1, 3);
            RT_PSWAP(1, 2);
#undef RT_PSWAP
            if (q0 != kKeyNone) {
                if (q3 != kKeyNone) RT_PK_PUSH(c3);
                if (q2 != kKeyNone) RT_PK_PUSH(c2);
                if (q1 != kKeyNone) RT_PK_PUSH(c1);
                node = uni(c0);
                continue;
            }
            }
        } else {
            const int v = ~node;
            const int first = v & ((1 << rtd::kLeafFirstBits) - 1);
            const int count = ((v >> rtd::kLeafFirstBits) & 3) + 1;
            const int kind = (v >> (rtd::kLeafFirstBits + 2)) & 1;
            if (kind == rtd::kLeafTri) {
                packet_leaf_tris<ANY, COUNT>(S, r, L, wgate, d2, first, count, cnt);
            } else {
                const int gate = rtt::cload(&S.sphs[first].misc).y;
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
                if (gate >= 0) wgate = -2;  // the lanes' caches moved on their own
            }
            if (ANY && __ballot(L.live) == 0) return;
        }
        if (sp == 0) return;
        --sp;
        node = uni(topv);
        if (sp > 0) topv = wstack[sp - 1];
    }
#undef RT_PK_PUSH
}

}  // namespace rtp
