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

// 3 entries per BVH4 level, plus the cut entries a camera packet may start
// with (cut_start: at most kCutMax - 1 waiting below the first)
constexpr int kWaveStack = rtd::kStackTotal + rtd::kCutMax;

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// Box tests of a packet's internal node for every lane, retired or not (a
// retired lane's keys come out +inf through a -inf culling distance): no
// exec-mask branch around them (packet_trace's BL).  The megakernel's
// default (C3 +0.75 %, r07q); the levels kernel keeps the branch — without
// it its register allocation spilled more (16-spp instance 6 -> 16 VGPR
// spill slots; C5's scratch writes 1.91 -> 3.37 GB a frame, r07r).
// RT_EXP_PKBRANCH=0: the megakernel with the branch (measuring builds).
#ifdef RT_EXP_PKBRANCH
constexpr bool kPkBranchless = RT_EXP_PKBRANCH != 0;
#else
constexpr bool kPkBranchless = true;
#endif

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
    RT_FETCH_WAVE(cnt, 48 * count);
    const rtd::TriRec t0 = rtt::cload(tb);
    const rtd::TriRec t1 = rtt::cload(tb + (count > 1 ? 1 : 0));
    const int gate = uni(__float_as_int(t0.p2.z));
    if (gate >= 0 && gate != wgate) {
        RT_FETCH_WAVE(cnt, 32);
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

// The tile of a camera packet: its pixel rectangle [x0, x0 + w) x [y0, y0 +
// h) in image coordinates (the camera samples of every lane lie inside it).
struct TileRect {
    int x0, y0, w, h;
};

// Is the padded box (lo, hi) outside the half-space {p : n . (p - o) >= 0}?
// Conservative: the corner furthest along n is tested with a relative slack
// far above the rounding of the camera-relative dot product, and a NaN never
// culls.
__device__ __forceinline__ bool cut_outside(f3 n, f3 clo, f3 chi) {
    const float cx = n.x >= 0.0f ? chi.x : clo.x, cy = n.y >= 0.0f ? chi.y : clo.y,
                cz = n.z >= 0.0f ? chi.z : clo.z;
    const float v = fmaf(n.x, cx, fmaf(n.y, cy, n.z * cz));
    const float mag = fmaf(fabsf(n.x), fabsf(cx), fmaf(fabsf(n.y), fabsf(cy), fabsf(n.z) * fabsf(cz)));
    return v < -1e-5f * mag;
}

// Stack marker of a waiting cut entry (cut_select): above every node index
// (node counts stay below 2^kLeafFirstBits).
constexpr int kCutMark = 0x40000000;

// Where a camera packet starts (cut_select): state -1 at the root, 0 when no
// ray of the tile can hit anything, 1 at `node` with sp - 1 entries on the
// wave stack below `topv`.
struct CutStart {
    int node, sp, topv, state;
};

// Start of a camera packet below the top levels of the tree: the cut entries
// (rtd::CutTable, one per lane) whose padded boxes the tile's frustum touches
// are the only subtrees any of its camera rays can hit, so the packet starts
// with them on its stack — nearest first along the tile's central ray — and
// never visits the nodes above the cut.  Only the visiting order changes,
// never a result.  The frustum: the four planes through the camera position
// bounding the tile's pixels widened by one pixel on every side (FrameDev
// cut_*): every camera ray of the tile (RayTracingSetup.cs:291-296, rounded)
// lies at least a pixel inside them.  Writes the entries below the top two
// into wstack.  Every lane of the wave must be active (one entry per lane).
// One lane's cut entry (lane j holds entry j), loaded before the tile is
// known: the loads overlap the tile's own setup instead of following it.
struct CutLane {
    int n_all;
    f3 lo, hi;
    int ref;
};

__device__ __forceinline__ CutLane cut_load(const rtd::SceneDev &S) {
    CutLane c;
    const rtd::CutTable *T = S.cut;
    c.n_all = T ? rtt::cload(&T->count) : 0;
    const int j = rtt::lane_id() & (rtd::kCutMax - 1);
    if (T) {
        c.lo = mk(T->lo_x[j], T->lo_y[j], T->lo_z[j]);
        c.hi = mk(T->hi_x[j], T->hi_y[j], T->hi_z[j]);
        c.ref = T->ref[j];
    } else {
        c.lo = c.hi = mk(0.0f, 0.0f, 0.0f);
        c.ref = 0;
    }
    return c;
}

__device__ __forceinline__ CutStart cut_select(const rtd::SceneDev &S, const rtd::FrameDev &F, const TileRect &tr,
                                               int *wstack, const CutLane *pre = nullptr) {
    CutStart cs = {0, 0, 0, -1};
    const rtd::CutTable *T = S.cut;
    const int n_all = pre ? pre->n_all : rtt::cload(&T->count);
    if (n_all <= 0) return cs;
    const int j = rtt::lane_id();
    bool need = false;
    float key = INFINITY;
    int ref = 0;
    if (j < n_all) {
        const float xa = (float)(tr.x0 - 1), xb = (float)(tr.x0 + tr.w + 1);
        const float ya = (float)(tr.y0 - 1), yb = (float)(tr.y0 + tr.h + 1);
        const f3 o = rtt::ld3(F.cam_pos);
        const f3 lo = pre ? pre->lo : mk(T->lo_x[j], T->lo_y[j], T->lo_z[j]);
        const f3 hi = pre ? pre->hi : mk(T->hi_x[j], T->hi_y[j], T->hi_z[j]);
        ref = pre ? pre->ref : T->ref[j];
        const f3 clo = lo - o, chi = hi - o;
        const f3 ax = rtt::ld3(F.cut_ax), bx = rtt::ld3(F.cut_bx), ay = rtt::ld3(F.cut_ay), by = rtt::ld3(F.cut_by);
        const f3 nx0 = mk(fmaf(xa, bx.x, ax.x), fmaf(xa, bx.y, ax.y), fmaf(xa, bx.z, ax.z));
        const f3 nx1 = mk(-fmaf(xb, bx.x, ax.x), -fmaf(xb, bx.y, ax.y), -fmaf(xb, bx.z, ax.z));
        const f3 ny0 = mk(fmaf(ya, by.x, ay.x), fmaf(ya, by.y, ay.y), fmaf(ya, by.z, ay.z));
        const f3 ny1 = mk(-fmaf(yb, by.x, ay.x), -fmaf(yb, by.y, ay.y), -fmaf(yb, by.z, ay.z));
        need = !(cut_outside(nx0, clo, chi) || cut_outside(nx1, clo, chi) || cut_outside(ny0, clo, chi) ||
                 cut_outside(ny1, clo, chi));
        if (need) {
            // entry distance along the tile's central ray A + xc R + yc U (order only)
            const float xc = (float)tr.x0 + 0.5f * (float)tr.w, yc = (float)tr.y0 + 0.5f * (float)tr.h;
            const f3 A = rtt::ld3(F.cut_a), R = rtt::ld3(F.cut_r), U = rtt::ld3(F.cut_u);
            const f3 dc = mk(fmaf(yc, U.x, fmaf(xc, R.x, A.x)), fmaf(yc, U.y, fmaf(xc, R.y, A.y)),
                             fmaf(yc, U.z, fmaf(xc, R.z, A.z)));
            const float ix = __builtin_amdgcn_rcpf(rtt::nudge(dc.x)), iy = __builtin_amdgcn_rcpf(rtt::nudge(dc.y)),
                        iz = __builtin_amdgcn_rcpf(rtt::nudge(dc.z));
            const float l0 = clo.x * ix, h0 = chi.x * ix, l1 = clo.y * iy, h1 = chi.y * iy, l2 = clo.z * iz,
                        h2 = chi.z * iz;
            const float tn = fmaxf(fmaxf(fminf(l0, h0), fminf(l1, h1)), fmaxf(fminf(l2, h2), 0.0f));
            const float tf = fminf(fminf(fmaxf(l0, h0), fmaxf(l1, h1)), fmaxf(l2, h2));
            key = tn <= tf ? tn : INFINITY;
        }
    }
    const unsigned long long mask = __ballot(need);
    if (mask == 0) {
        cs.state = 0;
        return cs;
    }
    const int n = __popcll(mask);
    // rank among the touched entries: nearer key first, ties by lane
    int rank = 0;
    for (unsigned long long m = mask; m; m &= m - 1) {
        const int i = __ffsll((long long)m) - 1;
        const float ki = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(key), i));
        rank += (ki < key || (ki == key && i < j)) ? 1 : 0;
    }
    // rank 0 is visited first, rank 1 waits on top (topv), ranks >= 2 below
    // it far-first: wstack[n - 1 - rank].  The waiting ones go as markers
    // (kCutMark + entry): popped, an entry is visited only when a live lane
    // still enters its box before its closest hit so far (packet_trace).
    if (need && rank >= 2) wstack[n - 1 - rank] = kCutMark + j;
    cs.node = __builtin_amdgcn_readlane(ref, __ffsll((long long)__ballot(need && rank == 0)) - 1);
    if (n > 1) cs.topv = kCutMark + __ffsll((long long)__ballot(need && rank == 1)) - 1;
    cs.sp = n - 1;
    cs.state = 1;
    return cs;
}

// ANY: shadow query with predicate t*t < d2 (see traverse.h).  `part`: the
// lane takes part.  wstack: this wave's LDS stack (kWaveStack ints).
// cs (camera packets): the start cut_select chose (null or state -1: the root).
// hint (ANY, < 0: a leaf ref): a leaf to test first — the one that occluded
// the most lanes of this tile's shadow packet last time; the walk from the
// root then never visits it again (each live lane has tested it already, and
// any-hit order cannot change an answer).  hint_out: where the leaf that
// retires the most lanes this time is stored (0: none), by one lane.  HINT:
// compiled only into the split-tile instance of render_kernel (small shards
// and synchronous frames, whose time is their slowest waves: a 1/8 C3 shard
// -3 %); in the whole-frame instance the extra scalar state cost 4 % (r04a).
template <bool ANY, bool COUNT, bool HINT = false, bool BL = kPkBranchless>
__device__ __forceinline__ void packet_trace(const rtd::SceneDev &S, const RayCtx &r, bool part, float tlimit,
                                             float d2, PacketLane &L, int *wstack, Counts &cnt,
                                             const CutStart *cs = nullptr, int hint = 0, int *hint_out = nullptr) {
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
    if (cs && cs->state >= 0) {
        if (cs->state == 0) return;
        node = cs->node;
        sp = cs->sp;
        topv = cs->topv;
    }
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
    // one leaf (ref < 0) against every live lane
    auto visit_leaf = [&](int ref) {
        const int v = ~ref;
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
    };
#ifdef RT_EXP_PREFETCH
    // measuring builds: the internal children a packet will visit later (the
    // pushed ones) are pulled into L2 right away by LDS-DMA loads whose data
    // nobody reads (lanes 0..2, one 4-B word of each node line into a dump
    // area), so their scalar fetch at the pop hits L2
    __shared__ int pf_dump[rtd::kWaveSize];
    auto prefetch3 = [&](int a, int b, int c) {
        const int ln = rtt::lane_id();
        const int v = ln == 0 ? a : ln == 1 ? b : c;
        if (ln < 3 && v > 0)
            __builtin_amdgcn_global_load_lds((const void *)(S.nodes4 + v), (__attribute__((address_space(3))) void *)pf_dump, 4, 0, 0);
    };
#endif
    const int rep0 = __ffsll((long long)live0) - 1;  // closest hit: a live lane, fixed for the whole walk
    // any-hit: the leaf that retires the most lanes (the next frame's hint)
    int best_leaf = 0, best_retired = 0;  // wave-uniform
    int skip = 0;                         // the hinted leaf, never visited again
    auto note_hint = [&]() {
        if (!ANY || !HINT || !hint_out) return;
        if (rtt::lane_id() == __ffsll((long long)__ballot(1)) - 1) *hint_out = best_leaf;
    };
    if (ANY && HINT && hint < 0) {
        const unsigned long long before = __ballot(L.live);
        visit_leaf(hint);
        const unsigned long long after = __ballot(L.live);
        best_retired = __popcll(before & ~after);
        best_leaf = best_retired ? hint : 0;
        if (after == 0) {
            note_hint();
            return;
        }
        skip = hint;
    }
    while (true) {
        if (!ANY && node >= kCutMark) {
            // a waiting cut entry (cut_select): visited only if a live lane's
            // ray still enters its box before the lane's closest hit so far
            RT_FETCH_WAVE(cnt, 32);
            const rtd::CutBox b = rtt::cload(S.cut->box + (node - kCutMark));
            const int ref = __float_as_int(b.lo.w);
            float k = INFINITY;
            if (L.live) k = rtt::child_key(b.lo.x, b.hi.x, b.lo.y, b.hi.y, b.lo.z, b.hi.z, r, L.tcull);
            if (COUNT && L.live) cnt.box++;
            if (__ballot(k != INFINITY) == 0) {
                if (sp == 0) return;
                --sp;
                node = uni(topv);
                if (sp > 0) topv = wstack[sp - 1];
                continue;
            }
            node = uni(ref);
        }
#ifdef RT_SEG_PROFILE
        if (node >= 0) L.nodes++; else L.leaves++;
#endif
        if (node >= 0) {
            RT_FETCH_WAVE(cnt, 128);
            float k0, k1, k2, k3;
            const int4 ch = rtt::cload(&S.nodes4[node].child);
            // a retired lane culls every child through its culling distance
            // (tf = -inf < tn): the same +inf keys as skipping it, without an
            // exec-mask branch around the box tests (BL)
            const float tc = BL ? (L.live ? L.tcull : -INFINITY) : L.tcull;
            if (same_signs) {
                // the near and far plane rows of each axis are fetched
                // directly (scalar loads at per-wave offsets), then 3 FMA +
                // max3/min3 per child: the same entry/exit values as the
                // min/max form (FMA is monotone in the plane value)
                const float4 *pl = reinterpret_cast<const float4 *>(S.nodes4 + node);
                const float4 nx = rtt::cload(pl + ox), fx = rtt::cload(pl + (1 - ox));
                const float4 ny = rtt::cload(pl + 2 + oy), fy = rtt::cload(pl + (3 - oy));
                const float4 nz = rtt::cload(pl + 4 + oz), fz = rtt::cload(pl + (5 - oz));
                k0 = k1 = k2 = k3 = INFINITY;
                if (BL || L.live) {
                    k0 = rtt::child_key_nf(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x, r, tc);
                    k1 = rtt::child_key_nf(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y, r, tc);
                    k2 = rtt::child_key_nf(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z, r, tc);
                    k3 = rtt::child_key_nf(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w, r, tc);
                }
            } else {
                const rtd::BvhNode4 nd = rtt::cload(S.nodes4 + node);
                k0 = k1 = k2 = k3 = INFINITY;
                if (BL || L.live) {
                    k0 = rtt::child_key(nd.lox.x, nd.hix.x, nd.loy.x, nd.hiy.x, nd.loz.x, nd.hiz.x, r, tc);
                    k1 = rtt::child_key(nd.lox.y, nd.hix.y, nd.loy.y, nd.hiy.y, nd.loz.y, nd.hiz.y, r, tc);
                    k2 = rtt::child_key(nd.lox.z, nd.hix.z, nd.loy.z, nd.hiy.z, nd.loz.z, nd.hiz.z, r, tc);
                    k3 = rtt::child_key(nd.lox.w, nd.hix.w, nd.loy.w, nd.hiy.w, nd.loz.w, nd.hiz.w, r, tc);
                }
            }
            if (COUNT && L.live) cnt.box += 4;
            if (ANY) {
                // any-hit (shadow rays): the order cannot change the answer,
                // so the children any live lane needs are taken in slot order
                // without the wave-wide sort (C3 -6 %, C2 -3 %, C5 +-0)
                const bool n0 = __ballot(k0 != INFINITY) != 0 && (!HINT || ch.x != skip),
                           n1 = __ballot(k1 != INFINITY) != 0 && (!HINT || ch.y != skip),
                           n2 = __ballot(k2 != INFINITY) != 0 && (!HINT || ch.z != skip),
                           n3 = __ballot(k3 != INFINITY) != 0 && (!HINT || ch.w != skip);
                int nn = 0, nxt = 0;
                if (n3) { nxt = ch.w; ++nn; }
                if (n2) { if (nn) RT_PK_PUSH(nxt); nxt = ch.z; ++nn; }
                if (n1) { if (nn) RT_PK_PUSH(nxt); nxt = ch.y; ++nn; }
                if (n0) { if (nn) RT_PK_PUSH(nxt); nxt = ch.x; ++nn; }
#ifdef RT_EXP_PREFETCH
                if (nn > 1)  // the pushed ones (not the next node: its fetch follows at once)
                    prefetch3(n3 && nxt != ch.w ? ch.w : -1, n2 && nxt != ch.z ? ch.z : -1,
                              n1 && nxt != ch.y ? ch.y : -1);
#endif
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
            // (a closest-hit packet's lanes never retire: its representative is fixed)
            const int rep = rep0;
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
#ifdef RT_EXP_PREFETCH
                if (q1 != kKeyNone)
                    prefetch3(q3 != kKeyNone ? c3 : -1, q2 != kKeyNone ? c2 : -1, c1);
#endif
                node = uni(c0);
                continue;
            }
            }
        } else {
            const unsigned long long before = ANY && HINT ? __ballot(L.live) : 0ull;
            visit_leaf(node);
            if (ANY) {
                const unsigned long long after = __ballot(L.live);
                if (HINT) {
                    const int retired = __popcll(before & ~after);
                    if (retired > best_retired) {
                        best_retired = retired;
                        best_leaf = node;
                    }
                }
                if (after == 0) {
                    note_hint();
                    return;
                }
            }
        }
        if (sp == 0) {
            note_hint();
            return;
        }
        --sp;
        node = uni(topv);
        if (sp > 0) topv = wstack[sp - 1];
    }
#undef RT_PK_PUSH
}

}  // namespace rtp
