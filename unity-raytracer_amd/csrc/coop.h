// coop.h — one ray, one whole wave: the BVH4 traversal of a wave-uniform ray
// with its node and primitive tests spread over the 64 lanes.
//
// Scene.IntersectRay (Data/Objects/Scene.cs:43-122) for the megakernel's
// one-sample waves (trace.hip render_sample_wave): a lone shard's slowest
// pixels run as waves of ONE sample each, whose single ray chain (up to
// MaxReflectionBounces closest hits plus a shadow ray per light and hit,
// RayTracingSetup.cs:304-366) is the shard's critical path.  Per lane, that
// chain is a dependent node fetch per visited node (~500 cycles each when
// the wave runs alone, DESIGN.md §10 "Frame critical path"); here every
// iteration pops up to 16 stack entries and tests them at once — four lanes
// per entry: the four child boxes of an internal node, or the (<= 4)
// primitives of a leaf — so a query takes a few iterations per tree level
// instead of a fetch per node.
//
// Same answer as the per-lane walk (traverse.h), bit for bit: the winner is
// the lowest (t, reference rank) over the hits that pass the reference's
// gates, which does not depend on the order nodes are visited; node culling
// uses the same conservative child_key test against the running best
// distance (closest hit) or the light-distance bound (any hit); every
// primitive test is the same rtm:: function on the same operands.  Only the
// visiting order, and so the test counts, differ: never used by counting
// launches (their counts are the canonical per-lane walk's).
#pragma once

#include <float.h>

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_math.h"
#include "traverse.h"

namespace rtc {

using rtm::f3;
using rtm::mk;

constexpr int kPopMax = 16;  // entries tested per iteration (4 lanes each)
// (the fold buffer shade_wave writes is the wave's packet stack: asserted
// against rtp::kWaveStack next to shade_wave in trace.hip)

// Push the lanes' `push` entries (ref, key) onto the wave's LDS stack at sp.
// SORT (closest hit): nearest on top — an entry's position is the number of
// pushed entries that are farther (ties: the higher lane below), so the next
// pops take the nearest subtrees first and the running best culls the rest.
template <bool SORT>
__device__ __forceinline__ int push_entries(int2 *stk, int sp, bool push, float key, int ref, int lane) {
    const unsigned long long m = __ballot(push);
    if (m == 0) return sp;
    int pos;
    if (SORT) {
        pos = 0;
        unsigned long long mm = m;
        const int kb = __float_as_int(key);
        while (mm) {  // wave-uniform: one readlane per pushed entry
            const int j = __builtin_ctzll(mm);
            mm &= mm - 1;
            const float kj = __int_as_float(__builtin_amdgcn_readlane(kb, j));
            pos += (kj > key || (kj == key && j > lane)) ? 1 : 0;
        }
    } else {
        pos = __popcll(m & ((1ull << lane) - 1ull));
    }
    if (push) stk[sp + pos] = make_int2(ref, __float_as_int(key));
    // the next iteration's pops read entries other lanes wrote
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return sp + __popcll(m);
}

// The per-mesh exact AABB gate of the reference's mesh loop (Scene.cs:67).
__device__ __forceinline__ bool gate_pass(const rtd::SceneDev &S, const rtt::RayCtx &r, int gate) {
    if (gate < 0) return true;
    const rtd::MeshGate g = S.gates[gate];
    return rtm::ref_slab(r.o, r.inv(), mk(g.lo.x, g.lo.y, g.lo.z), mk(g.hi.x, g.hi.y, g.hi.z));
}

// Stack bound.  A wide step pops g <= 16 entries and pushes <= 4 g, so it
// runs only while the stack stays below `wide` entries (sp + 3 g <= wide);
// above that the walk pops one entry per step — a depth-first walk, which
// adds at most 3 entries per tree level below the entry it started from
// (3 (depth + 1) <= kStackTotal: the builders' depth guarantee, rt_device.h).
// With wide <= cap - kStackTotal the stack never exceeds cap entries.
constexpr int kStackReserve = rtd::kStackTotal;

// Returns the query's answer like rtt::traverse (closest: best_t / best_rank
// of the winner, true on a hit; ANY: true iff an occluder with t*t < d2
// exists).  stk: the wave's LDS stack of cap >= kStackReserve + kCutMax
// entries; `wide` <= cap - kStackReserve (a smaller value — a testing knob,
// rt_debug_set RT_DEBUG_SAMPLE_WAVE_STACK — makes more steps depth-first).
// Call with every lane of the wave active and r, tlimit, d2 equal in all
// lanes.
template <bool ANY>
__device__ __forceinline__ bool traverse_wave(const rtd::SceneDev &S, const rtt::RayCtx &r, float tlimit, float d2,
                                              float &best_t, int &best_rank, int2 *stk, int wide) {
    best_t = FLT_MAX;
    best_rank = -1;
    if (!(S.has_prims && rtm::ref_slab(r.o, r.inv(), rtt::ld3(S.scene_lo), rtt::ld3(S.scene_hi)))) return false;
    const int lane = rtt::lane_id();
    float tcull = ANY ? tlimit : FLT_MAX;
    int sp;
    // start: the top-level cut's subtrees, one per lane (trace.hip
    // build_cut_kernel: every leaf lies below exactly one entry), or the root
    const rtd::CutTable *T = S.cut;
    const int ncut = T ? rtt::cload(&T->count) : 0;
    if (ncut > 0) {
        float k = INFINITY;
        int ref = 0;
        if (lane < ncut) {
            k = rtt::child_key(T->lo_x[lane], T->hi_x[lane], T->lo_y[lane], T->hi_y[lane], T->lo_z[lane],
                               T->hi_z[lane], r, tcull);
            ref = T->ref[lane];
        }
        sp = push_entries<!ANY>(stk, 0, k != INFINITY, k, ref, lane);
    } else {
        if (lane == 0) stk[0] = make_int2(0, 0);  // the root, key +0
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        sp = 1;
    }
    const int grp = lane >> 2, slot = lane & 3;
    while (sp > 0) {  // wave-uniform
        int g = sp < kPopMax ? sp : kPopMax;
        if (sp + 3 * g > wide) g = 1;  // depth-first near the top (kStackReserve)
        int ref = 0;
        bool have = false;
        if (grp < g) {
            const int2 e = stk[sp - 1 - grp];
            ref = e.x;
            have = __int_as_float(e.y) <= tcull;  // re-culled by the best hit found since the push
        }
        sp -= g;
        float ck = INFINITY;
        int cref = 0;
        bool hit = false;
        float th = 0.0f;
        int rank = 0;
        if (have && ref >= 0) {  // internal node: lane `slot` tests child `slot` (planes stored SoA)
            const float *f = reinterpret_cast<const float *>(S.nodes4 + ref);
            ck = rtt::child_key(f[slot], f[4 + slot], f[8 + slot], f[12 + slot], f[16 + slot], f[20 + slot], r, tcull);
            cref = reinterpret_cast<const int *>(f)[24 + slot];
        } else if (have) {  // leaf: lane `slot` tests primitive `slot`
            const int v = ~ref;
            const int first = v & ((1 << rtd::kLeafFirstBits) - 1);
            const int count = ((v >> rtd::kLeafFirstBits) & 3) + 1;
            const int kind = (v >> (rtd::kLeafFirstBits + 2)) & 1;
            if (slot < count) {
                if (kind == rtd::kLeafTri) {
                    const rtd::TriRec tr = S.tris[first + slot];
                    // the leaf's gate is its first record's (leaves are homogeneous in mesh)
                    const int gate = __float_as_int(slot == 0 ? tr.p2.z : S.tris[first].p2.z);
                    if (gate_pass(S, r, gate) &&
                        rtm::ref_triangle(r.o, r.d, mk(tr.p0.x, tr.p0.y, tr.p0.z), mk(tr.p0.w, tr.p1.x, tr.p1.y),
                                          mk(tr.p1.z, tr.p1.w, tr.p2.x), th)) {
                        hit = true;
                        rank = __float_as_int(tr.p2.y);
                    }
                } else {
                    const rtd::SphRec sr = S.sphs[first + slot];
                    const int gate = slot == 0 ? sr.misc.y : S.sphs[first].misc.y;
                    if (gate_pass(S, r, gate) && rtm::ref_sphere(r.o, r.d, mk(sr.cr.x, sr.cr.y, sr.cr.z), sr.cr.w, th)) {
                        hit = true;
                        rank = sr.misc.x;
                    }
                }
            }
        }
        if (ANY) {
            if (__ballot(hit && th * th < d2) != 0) {
                best_rank = 1;
                return true;
            }
        } else {
            // the hits in lane order through the per-lane rule (traverse.h
            // leaf): the lowest (t, rank) wins whatever the order
            unsigned long long m = __ballot(hit);
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const float tj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(th), j));
                const int rj = __builtin_amdgcn_readlane(rank, j);
                if (tj < best_t || (tj == best_t && rj < best_rank)) {
                    best_t = tj;
                    best_rank = rj;
                    tcull = tj;
                }
            }
        }
        sp = push_entries<!ANY>(stk, sp, ck != INFINITY && ck <= tcull, ck, cref, lane);
    }
    return ANY ? false : best_rank >= 0;
}

}  // namespace rtc
