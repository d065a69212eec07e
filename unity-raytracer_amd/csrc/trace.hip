// trace.hip — gfx950 "megakernel" path: one lane = one sample, the whole
// Whitted chain of RayTracingSetup.Shade (Assets/RayTracer/Demo-RayTracing/
// RayTracingSetup.cs:304-366) in one launch.  Kept as the simple reference
// implementation next to the wavefront path (trace_wf.hip), plus the batch
// closest-hit and band reassembly kernels.
//
// Execution shape: one wave64 = one tile of pixels x all their samples
// (spp lanes per pixel, consecutive), so a pixel's samples are summed in the
// documented fixed order with cross-lane moves and no atomics.  Branchy scalar
// FP32 — no MFMA.  Built with -ffp-contract=off and correctly rounded f32
// divide/sqrt so every reference operation rounds exactly once.
#include <float.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "coop.h"
#include "kernels.h"
#include "packet.h"
#include "rt_device.h"
#include "rt_math.h"
#include "shade.h"
#include "traverse.h"

using namespace rtd;
using rtm::f3;
using rtm::mk;
using rtt::Counts;

namespace {

// Shade with the mirror recursion unrolled into a loop; the recursion's
// results are folded back to front so c0 + km0*(c1 + km1*(...)) rounds
// exactly like the reference.
// The camera rays of a pixel tile and the first level's shadow rays (all
// from one tile towards the same light, highly coherent) are traced as wave
// packets (packet.h, scalar node fetches); deeper levels per lane.  All lanes
// in a loop iteration are at the same depth, so the choice is wave-uniform.

// RT_SEG_PROFILE (profiling builds only): per-wave shader-clock time of the
// setup / camera-packet / first-level shadow-packet segments and the whole
// tile, summed into the (otherwise unused, non-counting) test-counter words.
#ifdef RT_SEG_PROFILE
#define RT_SEG(x) x
#else
#define RT_SEG(x)
#endif
struct SegClock {
    unsigned long long setup, prim, shadow, visits;
};

// Ambient + every point light of one hit (RayTracingSetup.cs:320-356), shadow
// rays traced per lane.  MOOT (the split-tile instances, whose waves hold a
// frame's longest mirror chains): a moot shadow ray (shade.h same_bits) is not
// traced, as in the packets — kept out of the common instance, where the test
// added 25 spill sites.
template <bool COUNT, bool MOOT = false>
__device__ __forceinline__ f3 shade_hit(const SceneDev &S, const rts::Surface &sf, const rtt::Stack &st,
                                        Counts &cnt) {
    RT_FETCH_LANE(cnt, 64);  // the material (the surface's 16-B record: rts::surface's caller)
    f3 col = rts::ambient(S, S.mats[sf.mat]);
    for (int l = 0; l < S.num_lights; ++l) {  // :327-356
        RT_FETCH_WAVE(cnt, 32);
        const rts::ShadowRay sr = rts::shadow_ray(sf, S.lights[l]);
        cnt.shadow++;
        rtt::RayCtx rs;
        rtt::setup_ray(rs, sr.o, sr.dir);
        float dt;
        int dr;
        if (MOOT && !COUNT) {
            const f3 lit = col + rts::light_term(S, sf, S.mats[sf.mat], S.lights[l], sr);
            if (rts::same_bits(lit, col)) {
                cnt.moot++;
                continue;
            }
            if (!rtt::traverse<true, COUNT>(S, rs, sqrtf(sr.d2) * 1.001f, sr.d2, dt, dr, st, cnt)) col = lit;
            continue;
        }
        if (rtt::traverse<true, COUNT>(S, rs, sqrtf(sr.d2) * 1.001f, sr.d2, dt, dr, st, cnt)) continue;
        col = col + rts::light_term(S, sf, S.mats[sf.mat], S.lights[l], sr);
    }
    return col;
}

// One level of a mirror chain without shading: the closest hit of (o, d) and,
// if it is a mirror below MaxReflectionBounces, the reflected ray (o, d
// updated).  0: miss, 1: mirror bounce, 2: the chain ends at this hit (sf).
template <bool COUNT>
__device__ __forceinline__ int walk_level(const SceneDev &S, const FrameDev &F, f3 &o, f3 &d, int level,
                                          const rtt::Stack &st, Counts &cnt, rts::Surface &sf) {
    rtt::RayCtx r;
    rtt::setup_ray(r, o, d);
    float bt;
    int br;
    if (!rtt::traverse<false, COUNT>(S, r, 0.0f, 0.0f, bt, br, st, cnt)) return 0;
    if (COUNT) cnt.shading++;
    sf = rts::surface(S, o, d, bt, br);
    if (S.mats[sf.mat].ka_mirror.w != 0.0f && level < F.max_bounces) {
        rts::reflect(sf, o, d);
        return 1;
    }
    return 2;
}

// A mirror chain deeper than the fold stack (MaxReflectionBounces > kMaxBounces,
// RayTracingSetup.cs:23,358: an unbounded int in the reference).  The chain
// from level l0 (ray o0/d0) has already been shaded and counted up to level
// lc = l0 + kMaxBounces, where (oc, dc) is the ray.  Same rounding as the
// recursion with O(kMaxBounces) storage: (1) walk from lc to the end of the
// chain (closest hits only) and shade its last hit; (2) from the deepest
// segment of kMaxBounces levels up, re-walk from (o0, d0) to the segment's
// first level, shade the segment's levels into the fold stack and fold them
// onto the running value.  Re-walks are deterministic, so they rebuild the
// same rays bit for bit; every reference ray is counted once (levels below lc
// were counted by the caller).
template <bool COUNT>
__device__ __noinline__ f3 deep_chain(const SceneDev &S, const FrameDev &F, f3 o0, f3 d0, int l0, f3 oc, f3 dc,
                                      const rtt::Stack &st, Counts &cnt) {
    const int lc = l0 + kMaxBounces;
    Counts none = {0, 0, 0, 0, 0, 0, 0, 0};
    rts::Surface sf;
    f3 term;
    int end = lc;  // level of the chain's last ray
    {
        f3 o = oc, d = dc;
        while (true) {
            // the level-lc ray was traversed and counted by the caller: walk it
            // again without counting its tests and its shading fetch
            const int k = walk_level<COUNT>(S, F, o, d, end, st, end == lc ? none : cnt, sf);
            if (k == 0) {
                term = rtt::ld3(F.bg255);  // :310-311
                break;
            }
            if (k == 2) {
                term = shade_hit<COUNT>(S, sf, st, cnt);
                break;
            }
            cnt.reflection++;
            ++end;
        }
    }
    // levels l0 .. end-1 are mirror bounces; fold them in segments, deepest first
    float fold_c[kMaxBounces][3];
    float fold_k[kMaxBounces][3];
    for (int seg = l0 + ((end - 1 - l0) / kMaxBounces) * kMaxBounces; seg >= l0; seg -= kMaxBounces) {
        f3 o = o0, d = d0;
        int level = l0;
        if (seg >= lc) {
            o = oc;
            d = dc;
            level = lc;
        }
        for (; level < seg; ++level) (void)walk_level<COUNT>(S, F, o, d, level, st, none, sf);
        const int seg_end = min(seg + kMaxBounces, end);
        for (; level < seg_end; ++level) {
            rtt::RayCtx r;
            rtt::setup_ray(r, o, d);
            float bt;
            int br;
            (void)rtt::traverse<false, COUNT>(S, r, 0.0f, 0.0f, bt, br, st, none);  // a mirror hit
            const rts::Surface sfl = rts::surface(S, o, d, bt, br);
            const f3 col = level >= lc ? shade_hit<COUNT>(S, sfl, st, cnt) : shade_hit<COUNT>(S, sfl, st, none);
            const DevMaterial m = S.mats[sfl.mat];
            const int i = level - seg;
            fold_c[i][0] = col.x; fold_c[i][1] = col.y; fold_c[i][2] = col.z;
            fold_k[i][0] = m.km.x; fold_k[i][1] = m.km.y; fold_k[i][2] = m.km.z;
            rts::reflect(sfl, o, d);
        }
        for (int i = seg_end - seg - 1; i >= 0; --i)
            term = mk(fold_c[i][0], fold_c[i][1], fold_c[i][2]) + mk(fold_k[i][0], fold_k[i][1], fold_k[i][2]) * term;
    }
    return term;
}

// Shade levels depth0.. of one sample with per-lane traversal: the mirror
// recursion unrolled into a loop, its results folded back to front so
// c + km*(c' + km'*(...)) rounds exactly like the reference.  DEEP (frames with
// MaxReflectionBounces > kMaxBounces only): a chain that outgrows the fold
// stack continues in deep_chain.
template <bool COUNT, bool DEEP, bool MOOT = false>
__device__ __forceinline__ f3 shade_levels(const SceneDev &S, const FrameDev &F, f3 o, f3 d, int depth0,
                                           const rtt::Stack &st, Counts &cnt) {
    float fold_c[kMaxBounces][3];
    float fold_k[kMaxBounces][3];
    const f3 o0 = o, d0 = d;
    int depth = depth0;
    f3 term;
    while (true) {
        rtt::RayCtx r;
        rtt::setup_ray(r, o, d);
        float bt;
        int br;
        if (!rtt::traverse<false, COUNT>(S, r, 0.0f, 0.0f, bt, br, st, cnt)) {  // :310-311
            term = rtt::ld3(F.bg255);
            break;
        }
        if (COUNT) cnt.shading++;
        RT_FETCH_LANE(cnt, 16);
        const rts::Surface sf = rts::surface(S, o, d, bt, br);
        if (DEEP && depth - depth0 == kMaxBounces && S.mats[sf.mat].ka_mirror.w != 0.0f && depth < F.max_bounces) {
            return deep_chain<COUNT>(S, F, o0, d0, depth0, o, d, st, cnt);
        }
        const f3 col = shade_hit<COUNT, MOOT>(S, sf, st, cnt);
        const DevMaterial m = S.mats[sf.mat];
        if (m.ka_mirror.w != 0.0f && depth < F.max_bounces) {  // :358-363
            fold_c[depth - depth0][0] = col.x; fold_c[depth - depth0][1] = col.y; fold_c[depth - depth0][2] = col.z;
            fold_k[depth - depth0][0] = m.km.x; fold_k[depth - depth0][1] = m.km.y; fold_k[depth - depth0][2] = m.km.z;
            rts::reflect(sf, o, d);
            ++depth;
            cnt.reflection++;
            continue;
        }
        term = col;
        break;
    }
    for (int k = depth - depth0 - 1; k >= 0; --k)
        term = mk(fold_c[k][0], fold_c[k][1], fold_c[k][2]) + mk(fold_k[k][0], fold_k[k][1], fold_k[k][2]) * term;
    return term;
}


// The first hit's shadow packets keep the lane's hit and colours in LDS (the
// lane stack's column, 16 entries) rather than in registers across the packet
// loop (measuring builds: -DRT_EXP_STASH; A/B pending).
#ifdef RT_EXP_STASH
constexpr bool kShadowStash = true;
#else
constexpr bool kShadowStash = false;
#endif
static_assert(kStackSize >= 16, "the shadow-packet stash takes 16 lane-stack entries");

// Shade (RayTracingSetup.cs:304-366) of one camera sample.  The first hit is
// traced and shaded with wave packets (camera rays of a tile, then their
// shadow rays to each light: packet.h, scalar node fetches); the mirror
// chain below it (a few percent of samples) runs per lane (shade_levels).
// The counting launch keeps the per-ray traversal's canonical counts.
template <bool COUNT, bool DEEP, bool HINT, bool MOOT>
__device__ __forceinline__ f3 shade_path(const SceneDev &S, const FrameDev &F, f3 o, f3 d, const rtt::Stack &st,
                                         int *wstack, Counts &cnt, SegClock &sg, const rtp::CutStart &cs,
                                         int tile) {
    (void)sg;
    (void)tile;
    if (COUNT || !S.bvh4) return shade_levels<COUNT, DEEP>(S, F, o, d, 0, st, cnt);
    RT_SEG(const unsigned long long tq0 = __builtin_amdgcn_s_memtime();)
    rtt::RayCtx r;
    rtt::setup_ray(r, o, d);
    rtp::PacketLane P;
    rtp::packet_trace<false, COUNT>(S, r, true, 0.0f, 0.0f, P, wstack, cnt, &cs);
    RT_SEG(sg.visits += P.nodes + ((unsigned long long)P.leaves << 32);
           const unsigned long long tq1 = __builtin_amdgcn_s_memtime(); sg.setup = tq0; sg.prim = tq1 - tq0;)
    if (P.best_rank < 0) return rtt::ld3(F.bg255);  // :310-311
    // HINT: this tile's occluder hints of the last frame (one per light, < kHintLights)
    int *const hints = HINT && F.shadow_hint ? F.shadow_hint + (size_t)tile * kHintLights : nullptr;
    int4 hv = make_int4(0, 0, 0, 0);
    if (HINT && hints) hv = rtt::cload(reinterpret_cast<const int4 *>(hints));
    RT_FETCH_LANE(cnt, 16 + 64);  // the hit's shading record and material
    rts::Surface sf = rts::surface(S, o, d, P.best_t, P.best_rank);
    f3 col = rts::ambient(S, S.mats[sf.mat]);
    for (int l = 0; l < S.num_lights; ++l) {  // :327-356
        RT_FETCH_WAVE(cnt, 32);
        const rts::ShadowRay sr = rts::shadow_ray(sf, S.lights[l]);
        // a moot shadow ray (shade.h same_bits) is not traced
        f3 lit = col + rts::light_term(S, sf, S.mats[sf.mat], S.lights[l], sr);
        const bool moot = rts::same_bits(lit, col);
        cnt.shadow++;
        cnt.moot += moot;
        rtt::RayCtx rs;
        rtt::setup_ray(rs, sr.o, sr.dir);
        rtp::PacketLane Q;
        RT_SEG(const unsigned long long tw0 = __builtin_amdgcn_s_memtime();)
        const bool hl = HINT && hints && l < kHintLights;
        const int h = !hl ? 0 : l == 0 ? hv.x : l == 1 ? hv.y : l == 2 ? hv.z : hv.w;
        if (kShadowStash) {
            // the hit and both colours wait in the lane's LDS stack column
            // (unused by packets; the mirror chain's per-lane walks come after
            // the last light) instead of in registers the packet loop needs
            volatile int *vs = st.lds + rtt::lane_id();
            const float v[15] = {sf.p.x, sf.p.y, sf.p.z, sf.n.x, sf.n.y, sf.n.z, sf.view.x, sf.view.y, sf.view.z,
                                 col.x, col.y, col.z, lit.x, lit.y, lit.z};
#pragma unroll
            for (int i = 0; i < 15; ++i) vs[i * kWaveSize] = __float_as_int(v[i]);
            vs[15 * kWaveSize] = sf.mat;
            rtp::packet_trace<true, COUNT, HINT>(S, rs, !moot, sqrtf(sr.d2) * 1.001f, sr.d2, Q, wstack, cnt, nullptr,
                                                 h, hl ? hints + l : nullptr);
            vs = st.lds + rtt::lane_id();
            auto ld = [&](int i) { return __int_as_float(vs[i * kWaveSize]); };
            sf.p = mk(ld(0), ld(1), ld(2));
            sf.n = mk(ld(3), ld(4), ld(5));
            sf.view = mk(ld(6), ld(7), ld(8));
            col = mk(ld(9), ld(10), ld(11));
            lit = mk(ld(12), ld(13), ld(14));
            sf.mat = vs[15 * kWaveSize];
        } else {
            rtp::packet_trace<true, COUNT, HINT>(S, rs, !moot, sqrtf(sr.d2) * 1.001f, sr.d2, Q, wstack, cnt, nullptr,
                                                 h, hl ? hints + l : nullptr);
        }
        RT_SEG(sg.shadow += __builtin_amdgcn_s_memtime() - tw0;
               sg.visits += Q.nodes + ((unsigned long long)Q.leaves << 32);)
        if (moot || Q.best_rank == 1) continue;
        col = lit;
    }
    const DevMaterial m = S.mats[sf.mat];
    if (m.ka_mirror.w != 0.0f && 0 < F.max_bounces) {  // :358-363
        cnt.reflection++;
        f3 ro, rd;
        rts::reflect(sf, ro, rd);
        const f3 below = shade_levels<COUNT, DEEP, MOOT>(S, F, ro, rd, 1, st, cnt);
        return col + mk(m.km.x, m.km.y, m.km.z) * below;
    }
    return col;
}

// Waves per SIMD the register budget must allow.  Whole frames: 6 (80
// VGPRs) — with the per-lane LDS stack at 16 entries (rt_device.h
// kStackSize) six waves fit a CU's LDS too; at 24 entries the LDS capped the
// CU at 23 one-wave workgroups, so earlier "6 waves" builds only spilled more.
// C3 -7 % single frame / -5 % frames in flight, C2 -5 % / -2 % (r04h).  Small
// frames (row shards of <= kShardTiles tiles, whose time is their slowest
// waves): 5 (96 VGPRs, fewer spills) — 6 made a 1/8 shard 3-9 % slower.
#ifdef RT_EXP_MKWAVES
constexpr int kMkMinWaves = RT_EXP_MKWAVES;  // measuring builds only
#else
constexpr int kMkMinWaves = 6;
#endif
#ifdef RT_EXP_MKWSHARD
constexpr int kMkMinWavesShard = RT_EXP_MKWSHARD;  // measuring builds only
#else
constexpr int kMkMinWavesShard = 5;
#endif
// LDS stack entries of the 5-wave instances: 24 (a 1/2 C3 shard, single frame:
// 0.199 ms with 16 entries, 0.186 with 24, r04i; the LDS does not bind at five waves)
constexpr int kStackShard = 24;
// Waves of one finely split tile: 64 >> F.s16_shift — 16 waves of one
// pixel's four samples (shift 2), or in small shards 64 waves of one sample
// (shift 0, rt_frame.cpp lpt_prepare): a pixel's four samples then meet in
// F.split_samples and the last to arrive sums them (render_tile).
__device__ __forceinline__ int s16_shift(const FrameDev &F) { return __builtin_amdgcn_readfirstlane(F.s16_shift); }
constexpr int kShardTiles = rtk::kShardTilesMax;  // a 1/2 shard of 1080p at 4 spp
// ... but a shard of more tiles than this with other frames in flight beside
// it takes the 6-wave split instance: a 1/4 C3 share in flight -11.4 % per
// frame (0.0812 -> 0.0719 ms), a 1/8 share +8 %, lone shards +7 to +21 % (r06j);
// then (r06k) 1/2 -13.6 %, 1/4 -9.8 %, 1/8 +-0
#ifdef RT_EXP_SHARDW6
constexpr int kShardW6InFlight = RT_EXP_SHARDW6;  // measuring builds only
#else
constexpr int kShardW6InFlight = 24000;
#endif
// Waves per megakernel workgroup.  A workgroup's slot is recycled only when
// all of its waves are done, and path lengths vary a lot between tiles, so
// small workgroups keep the CUs fuller near the end of each wave "round".
constexpr int kMkWaves = 1;
constexpr int kMkThreads = kMkWaves * kWaveSize;


// The hand-off of a one-sample wave's sample (a lone shard's finely split
// pixel, F.s16_shift 0): the sample goes to the pixel's slots, then the
// pixel's arrival count; the fourth arrival sums the four samples in sample
// order (as sample_sum) and stores the pixel.  Two forms (A/B: RT_EXP_RELACQ):
// * relaxed (the default): the samples as agent-scope (write-through) stores,
//   an explicit wait for them before a relaxed count, agent-scope loads after
//   it — the hand-off a release / acquire pair gives, on gfx950, without the
//   L2 write-back an agent-scope release costs; argued from the ISA (the
//   samples reach the device's coherence point before the count; the last
//   arrival reads that point, after its count returned), and checked by
//   tests/test_gpu_parity.py::test_one_sample_handoff_under_concurrent_streams;
// * release / acquire: a release fetch-add of the count and an acquire fence
//   in the last arrival — the C++ memory model's hand-off at agent scope.  A
//   lone 1/8 C3 share 0.100 -> 0.143 ms (+42 %, three alternating rounds,
//   r07g): each release writes back the L2.
#ifdef RT_EXP_RELACQ
constexpr bool kRelAcqHandoff = true;  // measuring builds only
#else
constexpr bool kRelAcqHandoff = false;
#endif
__device__ __forceinline__ void split_handoff(const FrameDev &F, int sidx, int slot, f3 color, size_t pixel) {
    typedef __attribute__((address_space(1))) unsigned gu32;
    typedef __attribute__((address_space(1))) int gi32;
    float *sp = F.split_samples + ((size_t)sidx * kWaveSize + slot) * 4;
    __hip_atomic_store((gu32 *)sp, __float_as_uint(color.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32 *)(sp + 1), __float_as_uint(color.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32 *)(sp + 2), __float_as_uint(color.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int *cp = F.split_count + sidx * (kWaveSize / 4) + (slot >> 2);
    bool last;
    if (kRelAcqHandoff) {
        last = __hip_atomic_fetch_add((gi32 *)cp, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == 3;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sample is visible before the count
        last = __hip_atomic_fetch_add((gi32 *)cp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3;
    }
    if (!last) return;
    const float *b = F.split_samples + ((size_t)sidx * kWaveSize + (slot & ~3)) * 4;
    auto ld = [](const float *q) {
        return __uint_as_float(__hip_atomic_load((gu32 *)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    f3 v = mk(ld(b), ld(b + 1), ld(b + 2));
    for (int k = 1; k < 4; ++k) v = v + mk(ld(b + 4 * k), ld(b + 4 * k + 1), ld(b + 4 * k + 2));
    v = v * 0.25f;
    rts::store_pixel(F, pixel, v);
    __hip_atomic_store((gi32 *)cp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next frame's
}

// One tile (a wave) of the megakernel: trace every sample, sum a pixel's
// samples in row-major sample order ((s0 + s1) + s2) + ..., store.
// part >= 0: this wave takes only the lanes l with (l >> pshift) == part:
// one of the four (pshift 4: 16 lanes) or sixteen (pshift 2: 4 lanes) waves
// an expensive tile is split into.
// Returns true when the tile was answered by the sky test (no exact rays).
template <bool COUNT, bool DEEP, bool Q4, bool HINT, bool MOOT>
__device__ __forceinline__ bool render_tile(const SceneDev &S, const FrameDev &F, const rtt::Stack &st,
                                            int *wstack, int tile, int part, int pshift, int lane, Counts &cnt,
                                            SegClock &sg, int sidx) {
    (void)sidx;
    // the cut entries do not depend on the tile: their loads are issued first
    rtp::CutLane cl;
    if (!COUNT) cl = rtp::cut_load(S);
    if (!COUNT && S.cut) RT_FETCH_WAVE(cnt, 7 * 4 * kCutMax + 4);  // the cut table's SoA entries and count
    int px, ly, gy, s;
#ifdef RT_EXP_ONESAMPLE
    // measuring builds only (wrong images): a sixteenth-wave traces its pixel's first sample alone
    const bool active = rts::slot_pixel<Q4 ? 2 : 0>(F, tile, lane, px, ly, gy, s) &&
                        (part < 0 || ((lane >> pshift) == part && (pshift != 2 || (lane & 3) == RT_EXP_ONESAMPLE)));
#else
    const bool active =
        rts::slot_pixel<Q4 ? 2 : 0>(F, tile, lane, px, ly, gy, s) && (part < 0 || (lane >> pshift) == part);
#endif
    f3 color = mk(0.0f, 0.0f, 0.0f);
    // a wave whose samples all surely miss the padded Scene.AABB is background
    // without its exact rays (shade.h sky_maybe; the counting launch traces all)
    bool sky = false;
#ifndef RT_EXP_NOSKY
    if (!COUNT) sky = __ballot(active && (!F.sky_test || rts::sky_maybe<Q4 ? 2 : 0>(F, px, gy, s))) == 0;
#endif
    // the camera packet's start below the top-level cut (every lane active here)
    rtp::CutStart cs = {0, 0, 0, -1};
    if (!COUNT && !sky && F.cut_test) cs = rtp::cut_select(S, F, rts::tile_rect<Q4 ? 2 : 0>(F, tile), wstack, &cl);
    if (active) {
        if (COUNT) cnt.primary += 1;  // otherwise F.primary_total, added once per launch
        if (sky) {
            color = rtt::ld3(F.bg255);  // :310-311
        } else {
            f3 o, d;
            rts::primary_ray<Q4 ? 2 : 0>(F, px, gy, s, o, d);
            if (COUNT) {  // trivially cheap camera samples: they miss Scene.AABB (Scene.cs:54)
                rtt::RayCtx rg;
                rtt::setup_ray(rg, o, d);
                cnt.scene_miss +=
                    !(S.has_prims && rtm::ref_slab(o, rg.inv(), rtt::ld3(S.scene_lo), rtt::ld3(S.scene_hi)));
            }
            color = shade_path<COUNT, DEEP, HINT, MOOT>(S, F, o, d, st, wstack, cnt, sg, cs, tile);
        }
    }
    const f3 sum = rts::sample_sum(color, rtt::lane_id(), Q4 ? 4 : F.spp);
    // the slot -> pixel mapping is recomputed from the (scalar) tile index and
    // the lane id (v_mbcnt, opaque to the compiler so it is not kept live)
    // rather than kept live across the trace, where it would be spilled
    int tile2 = __builtin_amdgcn_readfirstlane(tile);
    asm volatile("" : "+s"(tile2));
    const int lane2 = rtt::lane_id();
    const bool active2 =
        rts::slot_pixel<Q4 ? 2 : 0>(F, tile2, lane2, px, ly, gy, s) && (part < 0 || (lane2 >> pshift) == part);
    if (HINT && !COUNT && pshift == 0 && (Q4 || F.spp == 4)) {
        // a one-sample wave of a split pixel: the hand-off of its sample to
        // the pixel's last arrival (split_handoff)
        if (active2) split_handoff(F, sidx, lane2, color, (size_t)ly * F.res_x + px);
        return sky;
    }
    if (active2 && s == 0) {
        f3 v = sum;
        if (Q4)
            v = v * 0.25f;  // == v / 4: the same real number, rounded once
        else if (F.spp > 1)
            v = (F.spp & (F.spp - 1)) == 0 ? v * F.inv_spp : v / (float)F.spp;  // likewise for 2^k
        rts::store_pixel(F, (size_t)ly * F.res_x + px, v);
    }
    return sky;
}


// Shade (RayTracingSetup.cs:304-366) of one camera sample with every lane of
// the wave on it: the same operations as shade_path / shade_levels (values
// equal in all lanes), each closest-hit and shadow query a whole-wave
// traversal.  The mirror fold (c + km*(...), back to front) sits in the
// wave's LDS: `fold` holds 6 floats per level (kMaxBounces levels).  Tallies
// are wave-uniform.
// (the fold sits in the wave's packet-stack LDS, wstack: rtp::kWaveStack ints)
static_assert(kMaxBounces * 6 <= rtp::kWaveStack, "a one-sample wave's mirror fold fits its packet stack");
__device__ __forceinline__ f3 shade_wave(const SceneDev &S, const FrameDev &F, f3 o, f3 d, int2 *stk, int wide,
                                         float *fold, unsigned &n_sh, unsigned &n_rf, unsigned &n_mo) {
    int depth = 0;
    f3 term;
    while (true) {
        rtt::RayCtx r;
        rtt::setup_ray(r, o, d);
        float bt;
        int br;
        if (!rtc::traverse_wave<false>(S, r, 0.0f, 0.0f, bt, br, stk, wide)) {  // :310-311
            term = rtt::ld3(F.bg255);
            break;
        }
        const rts::Surface sf = rts::surface(S, o, d, bt, br);
        f3 col = rts::ambient(S, S.mats[sf.mat]);
        for (int l = 0; l < S.num_lights; ++l) {  // :327-356
            const rts::ShadowRay sr = rts::shadow_ray(sf, S.lights[l]);
            ++n_sh;
            // a moot shadow ray (shade.h same_bits) is not traced
            const f3 lit = col + rts::light_term(S, sf, S.mats[sf.mat], S.lights[l], sr);
            if (rts::same_bits(lit, col)) {
                ++n_mo;
                continue;
            }
            rtt::RayCtx rs;
            rtt::setup_ray(rs, sr.o, sr.dir);
            float dt;
            int dr;
            if (!rtc::traverse_wave<true>(S, rs, sqrtf(sr.d2) * 1.001f, sr.d2, dt, dr, stk, wide)) col = lit;
        }
        const DevMaterial m = S.mats[sf.mat];
        if (m.ka_mirror.w != 0.0f && depth < F.max_bounces) {  // :358-363
            float *q = fold + depth * 6;  // every lane stores the same values
            q[0] = col.x;
            q[1] = col.y;
            q[2] = col.z;
            q[3] = m.km.x;
            q[4] = m.km.y;
            q[5] = m.km.z;
            rts::reflect(sf, o, d);
            ++depth;
            ++n_rf;
            continue;
        }
        term = col;
        break;
    }
    for (int k = depth - 1; k >= 0; --k) {
        const float *q = fold + k * 6;
        term = mk(q[0], q[1], q[2]) + mk(q[3], q[4], q[5]) * term;
    }
    return term;
}

// A one-sample wave (a lone shard's finely split tile, F.s16_shift 0): the
// sample render_tile's lane `part` would trace, traced by the whole wave
// (shade_wave), then the same write-through hand-off to the pixel's other
// three samples.  Returns true when the sample was answered by the sky test.
template <bool Q4>
__device__ __forceinline__ bool render_sample_wave(const SceneDev &S, const FrameDev &F, const rtt::Stack &st,
                                                   int *fold_lds, int tile, int part, int sidx, Counts &cnt) {
    constexpr int FX = Q4 ? 2 : 0;
    int px, ly, gy, s;
    const bool active = rts::slot_pixel<FX>(F, tile, part, px, ly, gy, s);
    // render_tile's sky test of its one active lane
    const bool sky = !(active && (!F.sky_test || rts::sky_maybe<FX>(F, px, gy, s)));
    if (!active) return sky;
    unsigned n_sh = 0, n_rf = 0, n_mo = 0;
    f3 color;
    if (sky) {
        color = rtt::ld3(F.bg255);  // :310-311
    } else {
        f3 o, d;
        rts::primary_ray<FX>(F, px, gy, s, o, d);
        // the wave's per-lane LDS stack area, free in a one-sample wave, holds the wave's stack
        int2 *stk = reinterpret_cast<int2 *>(st.lds);
        const int full = st.n * kWaveSize / 2 - rtc::kStackReserve;
        const int knob = __builtin_amdgcn_readfirstlane(F.sample_wave_stack);
        color = shade_wave(S, F, o, d, stk, knob > 0 && knob < full ? knob : full, reinterpret_cast<float *>(fold_lds), n_sh,
                           n_rf, n_mo);
    }
    if (rtt::lane_id() == 0) {
        cnt.shadow += n_sh;
        cnt.reflection += n_rf;
        cnt.moot += n_mo;
        split_handoff(F, sidx, part, color, (size_t)ly * F.res_x + px);  // render_tile's, for lane `part`'s sample
    }
    return sky;
}

// A tile of a sky batch (render_kernel, the last F.sky_batch_tiles of the
// order): render_tile's sky test — false when any sample may meet the scene
// (the caller renders the tile in full) — and otherwise its background
// pixels: the same samples (Shade's background, RayTracingSetup.cs:310-311),
// the same in-order sum and mean as render_tile's sky tiles.
template <bool Q4>
__device__ __forceinline__ bool sky_tile(const FrameDev &F, int tile) {
    constexpr int FX = Q4 ? 2 : 0;
    int px, ly, gy, s;
    const bool active = rts::slot_pixel<FX>(F, tile, rtt::lane_id(), px, ly, gy, s);
    if (__ballot(active && (!F.sky_test || rts::sky_maybe<FX>(F, px, gy, s))) != 0) return false;
    if (active && s == 0) {
        const f3 bg = rtt::ld3(F.bg255);
        const int spp = Q4 ? 4 : F.spp;
        f3 v = bg;
        for (int k = 1; k < spp; ++k) v = v + bg;  // rts::sample_sum's order
        if (Q4)
            v = v * 0.25f;
        else if (F.spp > 1)
            v = (F.spp & (F.spp - 1)) == 0 ? v * F.inv_spp : v / (float)F.spp;
        rts::store_pixel(F, (size_t)ly * F.res_x + px, v);
    }
    return true;
}

// One-sample waves traced by the whole wave (render_sample_wave, the SAMPLE
// instances); measuring builds may switch it off (-DRT_EXP_NOCOOP: the
// sample's lane alone, render_tile).
#ifdef RT_EXP_NOCOOP
constexpr bool kCoopSampleWaves = false;
#else
constexpr bool kCoopSampleWaves = true;
#endif

// The frame of batch tile t (t = f * frame_tiles + tile, wave-uniform) by the
// batch's magic multiplier (no integer division), and its tile in the frame.
__device__ __forceinline__ const FrameDev &batch_frame(const FrameBatch &B, int t, int &tile) {
    unsigned q = __umulhi((unsigned)t, B.frame_tiles_magic);
    int r = t - (int)q * B.frame_tiles;
    if (r >= B.frame_tiles) {
        ++q;
        r -= B.frame_tiles;
    }
    tile = r;
    return B.f[q];
}

// SPLIT: the variant launched when a frame splits tiles (a separate instance, so
// the common kernel's code and register allocation stay as they are); DEEP:
// the one for MaxReflectionBounces > kMaxBounces (deep_chain); Q4: frames of
// 2x2 spp in 4x4-pixel tiles (shade.h primary_ray / slot_pixel); SAMPLE:
// the lone-shard frames whose finely split tiles run as one-sample waves
// (F.s16_shift 0), each traced by its whole wave (render_sample_wave) — its
// own instance, so the shard instance that frames in flight run keeps its
// register allocation (the whole-wave path beside it: +11 VGPR and +65 SGPR
// spill slots, in-flight 1/2 and 1/4 shares 9-14 % slower, r05n).
//
// BATCH (render_batch_kernel): the frames of a FrameBatch in one launch — the
// batch's tiles are one index space (frame f's tile t is f * frame_tiles + t),
// dispatched and measured by one longest-first order; each wave renders its
// tile with its own frame's constants (camera, sky and frustum constants,
// output), the dispatch fields (order, splits, tallies) are the batch's and
// equal in every frame's block.
template <bool COUNT, bool SPLIT, bool DEEP, bool Q4, int W, bool SAMPLE, bool BATCH>
__device__ __forceinline__ void render_wave(const SceneDev &S, const FrameDev &F, const FrameBatch *B) {
    // the per-lane LDS stack: kStackSize entries where six waves per SIMD must
    // fit the CU's LDS, kStackShard at five (fewer overflows to scratch)
    constexpr int SS = W >= 6 ? kStackSize : kStackShard;
    __shared__ int stack_mem[kMkWaves * SS * kWaveSize];
    __shared__ int wstack_mem[kMkWaves * rtp::kWaveStack];
    const int lane = threadIdx.x & 63;
    // wave-uniform (an SGPR; with one-wave workgroups simply the block index)
    const int wave = kMkWaves == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int ovf[kStackTotal - SS];
    const rtt::Stack st{stack_mem + wave * SS * kWaveSize, ovf, SS};  // + lane per query (traverse)
    int *const wstack = wstack_mem + wave * rtp::kWaveStack;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
#ifdef RT_EXP_PERSIST
    // measuring builds: persistent waves over a whole frame's non-split
    // launch — resident waves take longest-first tile positions p = 8 k + x
    // from their XCD's counter (x = blockIdx % 8, the dispatch's XCD), until
    // the frame's tiles are used up; tallies and costs as below
    if (!COUNT && !SPLIT && F.persist_waves > 0) {
        const int x = blockIdx.x & 7;
        int *const ctr = F.persist_ctr + x * 16;
        if (!F.wave_counts && blockIdx.x == 0 && lane == 0) atomicAdd(rtt::counter_slot(F.counters), F.primary_total);
        SegClock sg = {0ull, 0ull, 0ull, 0ull};
        for (;;) {
            int k = 0;
            if (rtt::lane_id() == 0) k = atomicAdd(ctr, 1);
            const int pos = __builtin_amdgcn_readfirstlane(k) * 8 + x;
            if (pos >= F.num_tiles) break;  // wave-uniform
            int tile = pos;
            if (F.tile_order) tile = rtt::cload(F.tile_order + pos);
            tile = __builtin_amdgcn_readfirstlane(tile);
            const unsigned long long t0 = F.tile_cost ? __builtin_amdgcn_s_memtime() : 0ull;
            const bool sky = render_tile<COUNT, DEEP, Q4, false, false>(S, F, st, wstack, tile, -1, 4,
                                                                          rtt::lane_id(), cnt, sg, pos);
            if (F.tile_cost && rtt::lane_id() == 0)
                F.tile_cost[tile] = sky ? 0u : max(1u, tile_cost_key(__builtin_amdgcn_s_memtime() - t0, -1, 4));
        }
        if (F.wave_counts) {
            unsigned sh = 0, rf = 0, mo = 0;
            if (__ballot((cnt.shadow | cnt.reflection | cnt.moot) != 0) != 0) {
                sh = rtt::wave_sum(cnt.shadow);
                rf = rtt::wave_sum(cnt.reflection);
                mo = rtt::wave_sum(cnt.moot);
            }
            if (rtt::lane_id() == 0) F.wave_counts[blockIdx.x] = make_uint4(sh, rf, mo, F.count_tag);
        } else {
            rtt::flush_counts<COUNT>(cnt, F.counters);
        }
        return;
    }
#endif
    const int wid = blockIdx.x * kMkWaves + wave;
    const int split16 = SPLIT ? F.split16_tiles : 0;
    const int split = SPLIT ? F.split_tiles : 0;
    const int s16sh = SPLIT ? s16_shift(F) : 2;  // one finely split tile: 64 >> s16sh waves
    // (the order's last F.sky_batch_tiles positions: sky_batch_kernel's)
    if (wid >= F.num_tiles - (COUNT ? 0 : F.sky_batch_tiles) + ((64 >> s16sh) - 1) * split16 + 3 * split)
        return;  // wave-uniform
#ifdef RT_WAVE_CLOCK
    const unsigned long long rc0 = __builtin_amdgcn_s_memrealtime();  // constant 100 MHz clock
#endif
    // dispatch order: the previous frame's most expensive tiles first
    // (F.tile_order); SPLIT: the first split16_tiles of them as sixteen
    // waves of one pixel's 4 samples each, the next split_tiles as four
    // quarter-waves each (16 lanes: a smaller, more coherent packet, a
    // shorter wave)
    int idx, part = -1, pshift = 4;
    if (SPLIT && wid < (split16 << (6 - s16sh))) {
        idx = wid >> (6 - s16sh);
        part = wid & ((64 >> s16sh) - 1);
        pshift = s16sh;
    } else if (SPLIT && wid < (split16 << (6 - s16sh)) + 4 * split) {
        const int w1 = wid - (split16 << (6 - s16sh));
        idx = split16 + (w1 >> 2);
        part = w1 & 3;
    } else {
        idx = wid - ((64 >> s16sh) - 1) * split16 - 3 * split;
    }
    // the tile index is wave-uniform and kept in an SGPR: the slot -> pixel
    // integer math runs on the scalar unit and nothing of it is spilled
    int tile = idx;
    if (F.tile_order) tile = rtt::cload(F.tile_order + idx);
    tile = __builtin_amdgcn_readfirstlane(tile);
    if (F.tile_order) RT_FETCH_WAVE(cnt, 4);
    // a batch: the frame of the batch tile and its tile within the frame
    int ftile = tile;
    const FrameDev &FF = BATCH ? batch_frame(*B, tile, ftile) : F;
    // the launch's camera samples (one per active lane of every tile, computed
    // by the host: rt_device.h active_samples), counted once per launch
    if (!COUNT && !F.wave_counts && wid == 0 && lane == 0) atomicAdd(rtt::counter_slot(F.counters), F.primary_total);
    const unsigned long long t0 = F.tile_cost ? __builtin_amdgcn_s_memtime() : 0ull;
    SegClock sg = {0ull, 0ull, 0ull, 0ull};
    RT_SEG(const unsigned long long ts0 = __builtin_amdgcn_s_memtime();)
    // the shadow occluder hints (packet.h HINT) pay off in small frames only:
    // the 5-wave split instance (row shards), not the whole-frame one
    constexpr bool HINT = SPLIT && W < 6;
    bool sky;
    // a one-sample wave (pshift 0: render_tile's hand-off case) with its whole
    // wave on the sample's ray chain (wave-uniform test)
    if (SAMPLE && kCoopSampleWaves && HINT && !COUNT && !DEEP && pshift == 0 && (Q4 || F.spp == 4) && S.bvh4 &&
        F.max_bounces <= kMaxBounces)
        sky = render_sample_wave<Q4>(S, FF, st, wstack, ftile, part, idx, cnt);
    else
        sky = render_tile<COUNT, DEEP, Q4, HINT, SPLIT>(S, FF, st, wstack, ftile, part, pshift, lane, cnt, sg, idx);
    const int lane_e = rtt::lane_id();  // not kept live across the trace
    if (F.tile_cost && lane_e == 0 && part <= 0) {
        // a sky tile's key is 0: the next frames dispatch the sky tiles last, in row order
        F.tile_cost[tile] = sky ? 0u : max(1u, tile_cost_key(__builtin_amdgcn_s_memtime() - t0, part, pshift));
    }
#ifdef RT_SEG_PROFILE
    if (!COUNT) {
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        // the lanes' copies are equal (uniform clocks); lane 0 may be idle, take the max
        unsigned long long su = sg.setup ? sg.setup - ts0 : 0ull, pr = sg.prim, sh = sg.shadow, vi = sg.visits;
        for (int off = 32; off > 0; off >>= 1) {
            su = max(su, (unsigned long long)__shfl_xor((long long)su, off));
            pr = max(pr, (unsigned long long)__shfl_xor((long long)pr, off));
            sh = max(sh, (unsigned long long)__shfl_xor((long long)sh, off));
            vi = max(vi, (unsigned long long)__shfl_xor((long long)vi, off));
        }
        if (lane == 0) {
            unsigned long long *ctr = F.counters + (size_t)(blockIdx.x % kCounterSlots) * kCounterWords;
            atomicAdd(ctr + 3, vi);  // packet visits: internal | leaves << 32
            atomicAdd(ctr + 4, pr);
            atomicAdd(ctr + 5, sh);
            atomicAdd(ctr + 6, ts1 - ts0);
            atomicAdd(ctr + 7, su);  // tile start -> camera packet (slot mapping, sky test, cut, primary ray)
        }
    }
#endif
#ifdef RT_WAVE_CLOCK
    if (F.wave_clock && lane_e == 0) {
        // plain vector store (the wave's start and duration; the host finds the slowest waves)
        const unsigned long long rc1 = __builtin_amdgcn_s_memrealtime();
        F.wave_clock[wid] = make_uint4((unsigned)rc0, (unsigned)(rc0 >> 32), (unsigned)(rc1 - rc0),
                                       (unsigned)tile | ((unsigned)(part + 1) << 24));
    }
#endif
#ifndef RT_EXP_NOFLUSH
    if (!COUNT && F.wave_counts) {
        // the wave's tallies by a plain store (reduced by wave_counts_kernel
        // after the launch): an atomic holds the wave's slot for its whole
        // round trip, a store beside the pixel store costs next to nothing
        unsigned sh = 0, rf = 0, mo = 0;
        if (__ballot((cnt.shadow | cnt.reflection | cnt.moot) != 0) != 0) {
            sh = rtt::wave_sum(cnt.shadow);
            rf = rtt::wave_sum(cnt.reflection);
            mo = rtt::wave_sum(cnt.moot);
        }
        if (lane_e == 0) F.wave_counts[wid] = make_uint4(sh, rf, mo, F.count_tag);
    } else {
        rtt::flush_counts<COUNT>(cnt, F.counters);
    }
#endif
#ifdef RT_FETCH_COUNT
    {  // measuring builds: the wave's fetched bytes into counter word 9
        const unsigned fb = rtt::wave_sum(cnt.fetch);
        if (lane_e == 0 && fb) atomicAdd(rtt::counter_slot(F.counters) + 9, (unsigned long long)fb);
    }
#endif
}

template <bool COUNT, bool SPLIT = false, bool DEEP = false, bool Q4 = false, int W = kMkMinWaves,
          bool SAMPLE = false>
__global__ __launch_bounds__(kMkThreads, W) void render_kernel(SceneDev S, FrameDev F) {
    render_wave<COUNT, SPLIT, DEEP, Q4, W, SAMPLE, false>(S, F, nullptr);
}

// The frames of a batch in one launch (rt_render_device_batch: frames in
// flight of one layout, e.g. the frames of one gather group of a rank's row
// band): whole frames' 6-wave instances, Q4 only; B.f[0] holds the batch's
// dispatch fields.
template <bool SPLIT>
__global__ __launch_bounds__(kMkThreads, kMkMinWaves) void render_batch_kernel(SceneDev S, FrameBatch B) {
    render_wave<false, SPLIT, false, true, kMkMinWaves, false, true>(S, B.f[0], &B);
}

// The sky tail of a longest-first order (the last F.sky_batch_tiles
// positions: the tiles the last measurement found to be sky), rtk::kSkyBatch
// tiles a wave, launched after render_kernel on its stream.  A sky tile is a
// background store (sky_tile), too little work for a wave of its own: 60 % of
// a whole C3 frame's waves and 12 % of its wave time were such tiles
// (wclk_r05s).  A tile that is not sky this frame (the order predates a
// camera or scene change) is rendered in full, as render_kernel's whole-frame
// instance would; its tallies go to the counters directly.
#ifdef RT_EXP_SKYW
constexpr int kSkyWaves = RT_EXP_SKYW;  // measuring builds only
#else
constexpr int kSkyWaves = kMkMinWaves;
#endif
// The tallies of a launch's waves (F.wave_counts, as wave_counts_kernel) by
// one-wave blocks: block b of nb sums entries b, b + 64 nb, ... lane-strided.
__device__ __forceinline__ void wave_counts_part(const FrameDev &F, int waves, int b, int nb) {
    unsigned long long sh = 0, rf = 0, mo = 0;
    for (int i = b * kWaveSize + (int)(threadIdx.x & 63); i < waves; i += nb * kWaveSize) {
        const uint4 v = F.wave_counts[i];
        if (v.w != F.count_tag) continue;
        sh += v.x;
        rf += v.y;
        mo += v.z;
    }
    for (int off = 32; off > 0; off >>= 1) {
        sh += __shfl_xor(sh, off);
        rf += __shfl_xor(rf, off);
        mo += __shfl_xor(mo, off);
    }
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *ctr = F.counters + (size_t)(b % kCounterSlots) * kCounterWords;
        if (b == 0 && F.primary_total) atomicAdd(ctr + 0, F.primary_total);
        if (sh) atomicAdd(ctr + 1, sh);
        if (rf) atomicAdd(ctr + 2, rf);
        if (mo) atomicAdd(ctr + 8, mo);
    }
}

// The sky kernels' argument block: the scene, the frame (or the batch) and the grid split.
template <bool BATCH>
struct SkyArgs {
    SceneDev S;
    typename std::conditional<BATCH, FrameBatch, FrameDev>::type P;  // the frame, or the batch (P.f[0]: dispatch)
    int sky_blocks, waves;
};
__device__ __forceinline__ const FrameDev &head(const FrameDev &F) { return F; }
__device__ __forceinline__ const FrameDev &head(const FrameBatch &B) { return B.f[0]; }
// The frame of tile t of the argument block's frame or batch (and the tile in
// it).  (No pointer cast between the two: a cast of the by-value argument
// makes the compiler copy the whole block into scratch at kernel entry.)
__device__ __forceinline__ const FrameDev &frame_of(const FrameDev &F, int t, int &tile) {
    tile = t;
    return F;
}
__device__ __forceinline__ const FrameDev &frame_of(const FrameBatch &B, int t, int &tile) {
    return batch_frame(B, t, tile);
}
// A tile of a sky tail that is not sky this frame (the order predates a
// camera or scene change): rendered in full by the per-lane Whitted loop
// (shade_levels, the mirror chains' path: the same answers as render_tile's
// packets, bit for bit, with a fraction of its registers), after the sky loop
// (sky_batch_wave), which so keeps only its own state live — with render_tile
// inside the sky loop the kernel had 152 VGPR / 163 SGPR spill slots and wrote
// 1.6x its sky pixels (round 5).  Not out of line: ROCm 7.2 miscompiles a
// callee's generic pointers to its private overflow stack (a GPU fault on the
// first stale tile, r07b/r07d; an "Illegal instruction ... src_private_base"
// compile error in other forms).  The tallies go to the counters directly.
// pos: the tile's position in the order.
template <bool Q4, bool BATCH>
__device__ __forceinline__ void sky_fallback(const SkyArgs<BATCH> &A, const rtt::Stack &st, int pos) {
    constexpr int FX = Q4 ? 2 : 0;
    const SceneDev &S = A.S;
    const FrameDev &H = head(A.P);
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    const int tile = __builtin_amdgcn_readfirstlane(rtt::cload(H.tile_order + pos));
    int ftile = tile;
    const FrameDev &F = frame_of(A.P, tile, ftile);
    const unsigned long long t0 = H.tile_cost ? __builtin_amdgcn_s_memtime() : 0ull;
    int px, ly, gy, s;
    const bool active = rts::slot_pixel<FX>(F, ftile, rtt::lane_id(), px, ly, gy, s);
    f3 color = mk(0.0f, 0.0f, 0.0f);
    if (active) {
        f3 o, d;
        rts::primary_ray<FX>(F, px, gy, s, o, d);
        color = shade_levels<false, false, true>(S, F, o, d, 0, st, cnt);
    }
    const f3 sum = rts::sample_sum(color, rtt::lane_id(), Q4 ? 4 : F.spp);
    if (active && s == 0) {
        f3 v = sum;
        if (Q4)
            v = v * 0.25f;
        else if (F.spp > 1)
            v = (F.spp & (F.spp - 1)) == 0 ? v * F.inv_spp : v / (float)F.spp;
        rts::store_pixel(F, (size_t)ly * F.res_x + px, v);
    }
    if (H.tile_cost && rtt::lane_id() == 0)
        H.tile_cost[tile] = max(1u, tile_cost_key(__builtin_amdgcn_s_memtime() - t0, -1, 4));
    rtt::flush_counts<false>(cnt, H.counters);
#ifdef RT_FETCH_COUNT
    const unsigned fb = rtt::wave_sum(cnt.fetch);
    if (rtt::lane_id() == 0 && fb) atomicAdd(rtt::counter_slot(H.counters) + 9, (unsigned long long)fb);
#endif
}

// The work a frame in flight has after its render_kernel / levels launch, in
// one launch on its stream (a second dependent launch per frame cost a 1/8
// share in flight 35 %): blocks [0, sky_blocks) the order's sky tail
// (kSkyBatch tiles a wave: each a sky test and a background store,
// sky_tile), the rest the launch's per-wave tallies (`waves` entries).  The
// tiles that stopped being sky are noted in a wave-uniform mask during the
// loop and rendered after it, out of line (sky_fallback).  BATCH: the tail of
// a batch's order, each tile with its own frame's constants.
// one-wave blocks: p0 is indexed by the block and wave_counts_part strides
// the lanes with threadIdx & 63
static_assert(kMkThreads == kWaveSize, "sky_batch_kernel runs one-wave blocks");
static_assert(rtk::kSkyBatch <= 32, "the stale-tile mask");
template <bool Q4, bool BATCH>
__device__ __forceinline__ void sky_batch_wave(const SkyArgs<BATCH> &A) {
    const FrameDev &H = head(A.P);
    const int sky_blocks = A.sky_blocks, waves = A.waves;
    if ((int)blockIdx.x >= sky_blocks) {  // wave-uniform
        wave_counts_part(H, waves, (int)blockIdx.x - sky_blocks, (int)gridDim.x - sky_blocks);
        return;
    }
    const int p0 = H.num_tiles - H.sky_batch_tiles + (int)blockIdx.x * rtk::kSkyBatch;
    const int n = min(rtk::kSkyBatch, H.num_tiles - p0);  // wave-uniform
    unsigned stale = 0u;                                 // wave-uniform: bit j, position p0 + j is not sky
#ifdef RT_FETCH_COUNT
    if (rtt::lane_id() == 0) atomicAdd(rtt::counter_slot(H.counters) + 9, (unsigned long long)(4 * n));  // the tile indices
#endif
    for (int j = 0; j < n; ++j) {
        const int tile = __builtin_amdgcn_readfirstlane(rtt::cload(H.tile_order + p0 + j));
        int ftile = tile;
        const FrameDev &F = frame_of(A.P, tile, ftile);
        if (sky_tile<Q4>(F, ftile)) {
            if (H.tile_cost && rtt::lane_id() == 0) H.tile_cost[tile] = 0u;  // still sky: dispatched last again
        } else {
            stale |= 1u << j;
        }
    }
    if (!stale) return;
    // (rare: a camera or scene change since the order's measurement) — after
    // the sky loop, so the loop keeps only its own state live
    __shared__ int stack_mem[kStackSize * kWaveSize];
    int ovf[kStackTotal - kStackSize];
    const rtt::Stack st{stack_mem, ovf, kStackSize};  // (+ lane per query: traverse)
    do {
        const int j = __builtin_ctz(stale);
        stale &= stale - 1u;
        sky_fallback<Q4, BATCH>(A, st, p0 + j);
    } while (stale);
}

template <bool Q4>
__global__ __launch_bounds__(kMkThreads, kSkyWaves) void sky_batch_kernel(SkyArgs<false> A) {
    sky_batch_wave<Q4, false>(A);
}

__global__ __launch_bounds__(kMkThreads, kSkyWaves) void sky_batch_batch_kernel(SkyArgs<true> A) {
    sky_batch_wave<true, true>(A);
}

// Per-wave tallies of a render_kernel launch (F.wave_counts) -> the frame's
// sharded counters: shadow, reflection and moot rays, plus the launch's
// camera samples (F.primary_total) once.
// Only entries carrying this launch's tag count (a stale entry of another
// launch never does).
__global__ __launch_bounds__(256) void wave_counts_kernel(const uint4 *wc, int n, unsigned tag,
                                                         unsigned long long primary_total,
                                                         unsigned long long *counters) {
    unsigned long long sh = 0, rf = 0, mo = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint4 v = wc[i];
        if (v.w != tag) continue;
        sh += v.x;
        rf += v.y;
        mo += v.z;
    }
    for (int off = 32; off > 0; off >>= 1) {
        sh += __shfl_xor(sh, off);
        rf += __shfl_xor(rf, off);
        mo += __shfl_xor(mo, off);
    }
    __shared__ unsigned long long part[4][3];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[w][0] = sh;
        part[w][1] = rf;
        part[w][2] = mo;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long *ctr = counters + (size_t)(blockIdx.x % kCounterSlots) * kCounterWords;
        const unsigned long long a = part[0][0] + part[1][0] + part[2][0] + part[3][0];
        const unsigned long long b = part[0][1] + part[1][1] + part[2][1] + part[3][1];
        const unsigned long long c = part[0][2] + part[1][2] + part[2][2] + part[3][2];
        if (blockIdx.x == 0 && primary_total) atomicAdd(ctr + 0, primary_total);
        if (a) atomicAdd(ctr + 1, a);
        if (b) atomicAdd(ctr + 2, b);
        if (c) atomicAdd(ctr + 8, c);
    }
}

// The frame's sharded counters summed into kCounterWords words (out: the
// context's page-locked host words), so a synchronous frame reads 128 B after
// its stream synchronisation instead of copying all 32 KB of slots.
__global__ __launch_bounds__(256) void fold_counters_kernel(const unsigned long long *counters,
                                                           unsigned long long *out) {
    static_assert(kCounterWords == 16 && kCounterSlots % 16 == 0, "16 words x 16 parts");
    const int w = threadIdx.x & 15, part = threadIdx.x >> 4;
    unsigned long long s = 0;
    for (int sl = part; sl < kCounterSlots; sl += 16) s += counters[(size_t)sl * kCounterWords + w];
    __shared__ unsigned long long acc[16][16];
    acc[part][w] = s;
    __syncthreads();
    if (threadIdx.x < 16) {
        unsigned long long t = 0;
        for (int p = 0; p < 16; ++p) t += acc[p][threadIdx.x];
        out[threadIdx.x] = t;
    }
}

// Wave-synchronous megakernel: the Whitted chain advances level by level for
// the whole wave; rays of levels < PACKET_LEVELS (camera rays and their shadow
// rays first of all) are traced as one packet per wave (packet.h), deeper
// mirror rays per lane (traverse.h).  Same arithmetic and results as
// render_kernel.
template <bool COUNT, int PACKET_LEVELS>
__global__ __launch_bounds__(kBlockThreads) void render_packet_kernel(SceneDev S, FrameDev F) {
    __shared__ int stack_mem[kWavesPerBlock * kStackSize * kWaveSize];
    __shared__ int wstack_mem[kWavesPerBlock * rtp::kWaveStack];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int ovf[kStackTotal - kStackSize];
    const rtt::Stack st{stack_mem + wave * kStackSize * kWaveSize, ovf};  // + lane per query (traverse)
    int *wstack = wstack_mem + wave * rtp::kWaveStack;
    const int tile = blockIdx.x * kWavesPerBlock + wave;
    if (tile >= F.num_tiles) return;  // wave-uniform
    int px, ly, gy, s;
    const bool active = rts::slot_pixel(F, tile, lane, px, ly, gy, s);
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    float fold_c[kMaxBounces][3];
    float fold_k[kMaxBounces][3];
    int depth = 0;
    f3 term = mk(0.0f, 0.0f, 0.0f);
    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    bool alive = active;
    if (active) {
        rts::primary_ray(F, px, gy, s, o, d);
        cnt.primary = 1;
    }
    for (int level = 0; __ballot(alive) != 0; ++level) {  // wave-uniform
        rtt::RayCtx r;
        rtt::setup_ray(r, o, d);
        float bt = FLT_MAX;
        int br = -1;
        if (level < PACKET_LEVELS) {
            rtp::PacketLane P;
            rtp::packet_trace<false, COUNT>(S, r, alive, 0.0f, 0.0f, P, wstack, cnt);
            bt = P.best_t;
            br = P.best_rank;
        } else if (alive) {
            rtt::traverse<false, COUNT>(S, r, 0.0f, 0.0f, bt, br, st, cnt);
        }
        const bool hit = alive && br >= 0;
        if (alive && !hit) term = rtt::ld3(F.bg255);  // :310-311
        rts::Surface sf;
        DevMaterial m;
        f3 col = mk(0.0f, 0.0f, 0.0f);
        if (hit) {
            if (COUNT) cnt.shading++;
            sf = rts::surface(S, o, d, bt, br);
            m = S.mats[sf.mat];
            col = rts::ambient(S, m);
        }
        for (int l = 0; l < S.num_lights; ++l) {  // :327-356, wave-uniform
            const DevLight L = S.lights[l];
            rts::ShadowRay sr;
            rtt::RayCtx rs;
            sr.o = o;
            sr.dir = d;
            sr.d2 = 0.0f;
            if (hit) {
                sr = rts::shadow_ray(sf, L);
                cnt.shadow++;
            }
            rtt::setup_ray(rs, sr.o, sr.dir);
            bool occ = false;
            if (level < PACKET_LEVELS) {
                rtp::PacketLane Q;
                rtp::packet_trace<true, COUNT>(S, rs, hit, sqrtf(sr.d2) * 1.001f, sr.d2, Q, wstack, cnt);
                occ = Q.best_rank == 1;
            } else if (hit) {
                float dt;
                int dr;
                occ = rtt::traverse<true, COUNT>(S, rs, sqrtf(sr.d2) * 1.001f, sr.d2, dt, dr, st, cnt);
            }
            if (hit && !occ) col = col + rts::light_term(S, sf, m, L, sr);
        }
        const bool mirror = hit && m.ka_mirror.w != 0.0f && level < F.max_bounces;  // :358
        if (mirror) {
            fold_c[depth][0] = col.x; fold_c[depth][1] = col.y; fold_c[depth][2] = col.z;
            fold_k[depth][0] = m.km.x; fold_k[depth][1] = m.km.y; fold_k[depth][2] = m.km.z;
            rts::reflect(sf, o, d);
            ++depth;
            cnt.reflection++;
        } else if (hit) {
            term = col;
        }
        alive = mirror;
    }
    for (int k = depth - 1; k >= 0; --k)
        term = mk(fold_c[k][0], fold_c[k][1], fold_c[k][2]) + mk(fold_k[k][0], fold_k[k][1], fold_k[k][2]) * term;
    const f3 color = term;
    const f3 sum = rts::sample_sum(color, lane, F.spp);
    if (active && s == 0) {
        f3 v = sum;
        if (F.spp > 1) v = v / (float)F.spp;
        rts::store_pixel(F, (size_t)ly * F.res_x + px, v);
    }
    rtt::flush_counts<COUNT>(cnt, F.counters);
}

__global__ __launch_bounds__(kBlockThreads) void intersect_kernel(SceneDev S, const float *rays, int n, int4 *out) {
    __shared__ int stack_mem[kWavesPerBlock * kStackSize * kWaveSize];
    const int wave = threadIdx.x >> 6;
    int ovf[kStackTotal - kStackSize];
    const rtt::Stack st{stack_mem + wave * kStackSize * kWaveSize, ovf};  // + lane per query (traverse)
    const int i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    const float *rr = rays + (size_t)i * 6;
    rtt::RayCtx r;
    rtt::setup_ray(r, mk(rr[0], rr[1], rr[2]), mk(rr[3], rr[4], rr[5]));
    float bt;
    int br;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    rtt::traverse<false, false>(S, r, 0.0f, 0.0f, bt, br, st, cnt);
    // ObjectId.MeshIndex: the reference sets it only when a mesh triangle
    // becomes the running closest hit and never resets it when a sphere or a
    // loose triangle wins later (Scene.cs:76-79 vs :94-97,:109-112), so for
    // such a winner it is the mesh of the closest mesh-triangle hit, if any.
    int mesh_rank = br >= 0 && br < S.mesh_tri_total ? br : -1;
    if (br >= S.mesh_tri_total && S.mesh_tri_total > 0) {
        float mt;
        rtt::traverse<false, false, true>(S, r, 0.0f, 0.0f, mt, mesh_rank, st, cnt);
    }
    out[i] = make_int4(br, __float_as_int(bt), mesh_rank, 0);
}

struct Px12 {  // float RGB pixel (RT_FLAG_OUT_RGB32F)
    float v[3];
};

template <typename Px>
__global__ void assemble_kernel(const Px *gathered, int res_x, int res_y, int band_count, int band_rows,
                                int local_rows, Px *image) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)res_x * res_y;
    if (i >= total) return;
    const int gy = (int)(i / res_x), x = (int)(i - (size_t)gy * res_x);
    const int blk = gy / band_rows;
    const int band = blk % band_count, slot = blk / band_count;
    const int ly = slot * band_rows + (gy - blk * band_rows);
    image[i] = gathered[((size_t)band * local_rows + ly) * res_x + x];
}

// The top-level cut of a 4-wide tree (rtd::CutTable): starting from the
// root's children, the internal entry with the largest box surface (the
// lowest entry among equals) is replaced by its children -- the first
// non-empty child in its place, the others appended -- while the cut has room
// for them.  One wave, entry i in lane i: a step is one wave-wide arg-max and
// one node fetch; every new entry fetches its own node's child count at once
// (a few tens of microseconds after each tree build or refit; the first,
// single-thread version spent 0.6 ms walking its arrays through scratch).
__global__ __launch_bounds__(64) void build_cut_kernel(const BvhNode4 *nodes, CutTable *out) {
    const int lane = threadIdx.x;
    int ref = 0, kids = 0;  // kids: the entry's own node's non-empty children (internal entries)
    int from = 0;           // the entry's parent node * 4 + child slot (refresh_cut_kernel)
    float lo0 = 0.0f, lo1 = 0.0f, lo2 = 0.0f, hi0 = 0.0f, hi1 = 0.0f, hi2 = 0.0f, area = -1.0f;
    int n = 0;  // wave-uniform
    // the children of `node` in place of entry `at` (the first) and appended
    auto expand = [&](int node, int at) {
        const BvhNode4 nd = nodes[node];
        const float lx[4] = {nd.lox.x, nd.lox.y, nd.lox.z, nd.lox.w}, hx[4] = {nd.hix.x, nd.hix.y, nd.hix.z, nd.hix.w};
        const float ly[4] = {nd.loy.x, nd.loy.y, nd.loy.z, nd.loy.w}, hy[4] = {nd.hiy.x, nd.hiy.y, nd.hiy.z, nd.hiy.w};
        const float lz[4] = {nd.loz.x, nd.loz.y, nd.loz.z, nd.loz.w}, hz[4] = {nd.hiz.x, nd.hiz.y, nd.hiz.z, nd.hiz.w};
        const int ch[4] = {nd.child.x, nd.child.y, nd.child.z, nd.child.w};
        bool mine = false;
        for (int c = 0; c < 4; ++c) {
            if (lx[c] == INFINITY && hx[c] == INFINITY) continue;  // empty slot
            const int k = at >= 0 ? at : n++;
            at = -1;
            if (lane != k) continue;
            mine = true;
            ref = ch[c];
            from = node * 4 + c;
            lo0 = lx[c]; lo1 = ly[c]; lo2 = lz[c];
            hi0 = hx[c]; hi1 = hy[c]; hi2 = hz[c];
            const float ex = hx[c] - lx[c], ey = hy[c] - ly[c], ez = hz[c] - lz[c];
            area = ch[c] >= 0 ? ex * ey + ey * ez + ez * ex : -1.0f;  // leaves never expand
            if (!(area >= 0.0f) && ch[c] >= 0) area = 0.0f;  // NaN box: expandable last
        }
        if (mine && ref >= 0) {
            const BvhNode4 own = nodes[ref];
            kids = (own.lox.x == INFINITY && own.hix.x == INFINITY ? 0 : 1) +
                   (own.lox.y == INFINITY && own.hix.y == INFINITY ? 0 : 1) +
                   (own.lox.z == INFINITY && own.hix.z == INFINITY ? 0 : 1) +
                   (own.lox.w == INFINITY && own.hix.w == INFINITY ? 0 : 1);
        }
    };
    expand(0, -1);
    while (true) {
        float m = area;
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        const unsigned long long at_max = __ballot(area >= 0.0f && area == m);
        if (!(m >= 0.0f) || at_max == 0) break;
        const int best = __ffsll((long long)at_max) - 1;
        const int bref = __shfl(ref, best), c = __shfl(kids, best);
        if (c == 0 || n - 1 + c > kCutMax) {
            if (lane == best) area = -1.0f;  // stays in the cut as it is
            continue;
        }
        expand(bref, best);
    }
    if (lane < n) {
        out->lo_x[lane] = lo0; out->lo_y[lane] = lo1; out->lo_z[lane] = lo2;
        out->hi_x[lane] = hi0; out->hi_y[lane] = hi1; out->hi_z[lane] = hi2;
        out->ref[lane] = ref;
        out->box[lane].lo = make_float4(lo0, lo1, lo2, __int_as_float(ref));
        out->box[lane].hi = make_float4(hi0, hi1, hi2, __int_as_float(from));
    }
    if (lane == 0) out->count = n;
}

// After a refit (same topology, new boxes: rt_abi.cpp refit_update) the cut
// keeps its subtrees and only takes their new padded boxes from their parents'
// child slots: one fetch per entry instead of the greedy selection's chain of
// dependent node fetches.  The subtrees still partition the leaves, so every
// camera ray's answer is unchanged (packet.h cut_select).
__global__ __launch_bounds__(64) void refresh_cut_kernel(const BvhNode4 *nodes, CutTable *out) {
    const int lane = threadIdx.x;
    if (lane >= out->count) return;
    const int from = __float_as_int(out->box[lane].hi.w);
    const BvhNode4 nd = nodes[from >> 2];
    const int c = from & 3;
    const float lo0 = c == 0 ? nd.lox.x : c == 1 ? nd.lox.y : c == 2 ? nd.lox.z : nd.lox.w;
    const float lo1 = c == 0 ? nd.loy.x : c == 1 ? nd.loy.y : c == 2 ? nd.loy.z : nd.loy.w;
    const float lo2 = c == 0 ? nd.loz.x : c == 1 ? nd.loz.y : c == 2 ? nd.loz.z : nd.loz.w;
    const float hi0 = c == 0 ? nd.hix.x : c == 1 ? nd.hix.y : c == 2 ? nd.hix.z : nd.hix.w;
    const float hi1 = c == 0 ? nd.hiy.x : c == 1 ? nd.hiy.y : c == 2 ? nd.hiy.z : nd.hiy.w;
    const float hi2 = c == 0 ? nd.hiz.x : c == 1 ? nd.hiz.y : c == 2 ? nd.hiz.z : nd.hiz.w;
    out->lo_x[lane] = lo0; out->lo_y[lane] = lo1; out->lo_z[lane] = lo2;
    out->hi_x[lane] = hi0; out->hi_y[lane] = hi1; out->hi_z[lane] = hi2;
    out->box[lane].lo = make_float4(lo0, lo1, lo2, out->box[lane].lo.w);
    out->box[lane].hi = make_float4(hi0, hi1, hi2, __int_as_float(from));
}

}  // namespace

namespace rtk {

hipError_t launch_build_cut(const BvhNode4 *nodes, CutTable *out, hipStream_t stream) {
    hipLaunchKernelGGL(build_cut_kernel, dim3(1), dim3(64), 0, stream, nodes, out);
    return hipGetLastError();
}

hipError_t launch_refresh_cut(const BvhNode4 *nodes, CutTable *out, hipStream_t stream) {
    hipLaunchKernelGGL(refresh_cut_kernel, dim3(1), dim3(64), 0, stream, nodes, out);
    return hipGetLastError();
}

// all-packet levels pay off where a wave's tile is small on screen (its
// mirror rays stay coherent): 16+ samples per pixel = at most 2x2 pixels
constexpr int kLevelsMinSpp = 16;


// one-wave tally blocks of sky_batch_kernel for `waves` entries (as many
// threads as wave_counts_kernel's up to 64 x 256)
static int tail_count_blocks(int waves) { return std::max(1, std::min(256, (waves + 255) / 256)); }

hipError_t launch_render_mega(const SceneDev &S, const FrameDev &F0, bool count_tests, hipStream_t stream,
                              const char **instance) {
    const char *dummy = nullptr;
    const char *&name = instance ? *instance : dummy;
    name = nullptr;
    if (F0.num_tiles <= 0) return hipSuccess;
    FrameDev F = F0;
    F.primary_total = active_samples(F.res_x, F.res_y, F.local_rows, F.row0, F.band_index, F.band_count, F.band_rows,
                                     F.spp);
    int blocks = (render_mega_waves(F) + kMkWaves - 1) / kMkWaves;
#ifdef RT_EXP_PERSIST
    if (F.persist_waves > 0 && !count_tests && F.split_tiles == 0 && F.split16_tiles == 0 && F.max_bounces <= kMaxBounces &&
        !(S.bvh4 && F.spp >= kLevelsMinSpp))
        blocks = std::min(blocks, F.persist_waves);
    else
        F.persist_waves = 0;
#endif
    const bool q4 = F.spp == 4 && F.tile_w == 4 && F.tile_h == 4;
    // a small frame: its slowest waves set its time (unless frames in flight hide them)
    const bool shard = F.num_tiles <= kShardTiles && !(F.in_flight && F.num_tiles > kShardW6InFlight);
    const bool split = F.split_tiles > 0 || F.split16_tiles > 0;
    constexpr int W5 = kMkMinWavesShard;
#if !defined(RT_EXP_MKWAVES) && !defined(RT_EXP_MKWSHARD)
    static_assert(kMkMinWaves == 6 && W5 == 5, "instance names below");
#endif
#define RT_LAUNCH(K, NAME)                                                                  \
    do {                                                                                    \
        if (blocks > 0) hipLaunchKernelGGL(K, dim3(blocks), dim3(kMkThreads), 0, stream, S, F); \
        name = NAME;                                                                        \
    } while (0)
    if (F.max_bounces > kMaxBounces) {  // mirror chains may outgrow the fold stack
        if (count_tests)
            RT_LAUNCH((render_kernel<true, false, true, false, W5>), "render_kernel<true, false, true, false, 5, false>");
        else
            RT_LAUNCH((render_kernel<false, false, true, false, W5>), "render_kernel<false, false, true, false, 5, false>");
    } else if (count_tests)
        RT_LAUNCH((render_kernel<true, false, false, false, W5>), "render_kernel<true, false, false, false, 5, false>");
    else if (split && q4 && shard && F.s16_shift == 0)
        RT_LAUNCH((render_kernel<false, true, false, true, W5, true>), "render_kernel<false, true, false, true, 5, true>");
    else if (split && q4 && shard)
        RT_LAUNCH((render_kernel<false, true, false, true, W5>), "render_kernel<false, true, false, true, 5, false>");
    else if (split && q4)
        RT_LAUNCH((render_kernel<false, true, false, true>), "render_kernel<false, true, false, true, 6, false>");
    else if (split && shard && F.s16_shift == 0)
        RT_LAUNCH((render_kernel<false, true, false, false, W5, true>),
                  "render_kernel<false, true, false, false, 5, true>");
    else if (split && shard)
        RT_LAUNCH((render_kernel<false, true, false, false, W5>), "render_kernel<false, true, false, false, 5, false>");
    else if (split)
        RT_LAUNCH((render_kernel<false, true>), "render_kernel<false, true, false, false, 6, false>");
    else if (S.bvh4 && F.spp >= kLevelsMinSpp) {
        const hipError_t e = launch_render_levels(S, F, stream);
        static const char *const lv[2][3] = {{"render_levels_kernel<6, 8, 4>", "render_levels_kernel<6, 16, 4>",
                                              "render_levels_kernel<6, 32, 4>"},
                                             {"render_levels_kernel<7, 8, 8>", "render_levels_kernel<7, 16, 8>",
                                              "render_levels_kernel<7, 32, 8>"}};
        name = F.spp > 16 && F.spp != 64 ? "render_levels_kernel<7, 32, 0>"
                                         : lv[F.spp <= 16 ? 0 : 1][F.max_bounces <= 8 ? 0 : F.max_bounces <= 16 ? 1 : 2];
        if (e != hipSuccess) return e;
        const int waves = F.num_tiles - F.sky_batch_tiles;  // one wave per position, no splits
        if (F.sky_batch_tiles > 0 && F.tile_order && F.wave_counts) {  // (16 spp in flight: the order's sky tail)
            const int sb = (F.sky_batch_tiles + rtk::kSkyBatch - 1) / rtk::kSkyBatch;
            hipLaunchKernelGGL(sky_batch_kernel<false>, dim3(sb + tail_count_blocks(waves)), dim3(kMkThreads), 0, stream,
                               SkyArgs<false>{S, F, sb, waves});
            return hipGetLastError();
        }
        if (!F.wave_counts) return hipGetLastError();
        hipLaunchKernelGGL(wave_counts_kernel, dim3(std::max(1, std::min(64, (waves + 1023) / 1024))), dim3(256), 0, stream,
                           (const uint4 *)F.wave_counts, waves, F.count_tag, F.primary_total, F.counters);
        return hipGetLastError();
    }
    else if (q4)
        RT_LAUNCH((render_kernel<false, false, false, true>), "render_kernel<false, false, false, true, 6, false>");
    else
        RT_LAUNCH(render_kernel<false>, "render_kernel<false, false, false, false, 6, false>");
#undef RT_LAUNCH
    if (!count_tests && F.sky_batch_tiles > 0 && F.tile_order && F.max_bounces <= kMaxBounces && F.wave_counts) {
        // the order's sky tail and the launch's tallies in one launch
        const int sb = (F.sky_batch_tiles + rtk::kSkyBatch - 1) / rtk::kSkyBatch;
        const int waves = render_mega_waves(F);
        const dim3 g(sb + tail_count_blocks(waves));
        if (q4)
            hipLaunchKernelGGL(sky_batch_kernel<true>, g, dim3(kMkThreads), 0, stream, SkyArgs<false>{S, F, sb, waves});
        else
            hipLaunchKernelGGL(sky_batch_kernel<false>, g, dim3(kMkThreads), 0, stream, SkyArgs<false>{S, F, sb, waves});
        return hipGetLastError();
    }
    if (!count_tests && F.wave_counts) {  // the launch's per-wave tallies -> counters
        const int waves = render_mega_waves(F);  // the entries lpt_prepare sized the buffer for
        hipLaunchKernelGGL(wave_counts_kernel, dim3(std::max(1, std::min(64, (waves + 1023) / 1024))), dim3(256), 0, stream,
                           (const uint4 *)F.wave_counts, waves, F.count_tag, F.primary_total, F.counters);
    }
    return hipGetLastError();
}

hipError_t launch_render_batch(const SceneDev &S, const FrameBatch &B0, hipStream_t stream, const char **instance) {
    const char *dummy = nullptr;
    const char *&name = instance ? *instance : dummy;
    name = nullptr;
    if (B0.frames < 1 || B0.frames > kMaxBatch || B0.f[0].num_tiles <= 0) return hipErrorInvalidValue;
    static thread_local FrameBatch B;
    B = B0;
    FrameDev &H = B.f[0];
    // the batch's camera samples: one frame's times the frames
    H.primary_total = active_samples(H.res_x, H.res_y, H.local_rows, H.row0, H.band_index, H.band_count,
                                     H.band_rows, H.spp) *
                      (unsigned long long)B.frames;
    const int blocks = render_mega_waves(H);
    if (H.split_tiles > 0 || H.split16_tiles > 0) {
        hipLaunchKernelGGL(render_batch_kernel<true>, dim3(blocks), dim3(kMkThreads), 0, stream, S, B);
        name = "render_batch_kernel<true>";
    } else {
        hipLaunchKernelGGL(render_batch_kernel<false>, dim3(blocks), dim3(kMkThreads), 0, stream, S, B);
        name = "render_batch_kernel<false>";
    }
    if (H.sky_batch_tiles > 0 && H.tile_order && H.wave_counts) {
        // the batch order's sky tail and the launch's tallies in one launch
        const int sb = (H.sky_batch_tiles + rtk::kSkyBatch - 1) / rtk::kSkyBatch;
        hipLaunchKernelGGL(sky_batch_batch_kernel, dim3(sb + tail_count_blocks(blocks)), dim3(kMkThreads), 0, stream,
                           SkyArgs<true>{S, B, sb, blocks});
    } else if (H.wave_counts) {
        hipLaunchKernelGGL(wave_counts_kernel, dim3(std::max(1, std::min(64, (blocks + 1023) / 1024))), dim3(256), 0,
                           stream, (const uint4 *)H.wave_counts, blocks, H.count_tag, H.primary_total, H.counters);
    }
    return hipGetLastError();
}

int render_mega_waves(const FrameDev &F) {
    // (the last F.sky_batch_tiles positions are sky_batch_kernel's; the counting launch's F has none)
    return F.num_tiles <= 0 ? 0
                            : F.num_tiles - F.sky_batch_tiles + ((64 >> F.s16_shift) - 1) * F.split16_tiles +
                                  3 * F.split_tiles;
}

__global__ __launch_bounds__(256) void sky_count_kernel(const unsigned *sorted, int n, unsigned seq,
                                                       unsigned long long *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    // sorted descending: the first 0 key, or n when none (exactly one thread
    // writes, one 64-bit vector store: the host never sees a torn pair)
    const bool zero = sorted[i] == 0u;
    if ((zero && (i == 0 || sorted[i - 1] != 0u)) || (!zero && i == n - 1))
        __hip_atomic_store(out, ((unsigned long long)seq << 32) | (unsigned)(zero ? i : n), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_sky_count(const unsigned *cost_sorted, int n, unsigned seq, unsigned long long *out,
                            hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sky_count_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, cost_sorted, n, seq, out);
    return hipGetLastError();
}

// Longest-first dispatch for the next frame: tiles sorted by the cost key this
// frame measured (descending, 9-bit log-scale keys).
size_t tile_sort_scratch_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr,
                                                        (const int *)nullptr, (int *)nullptr, n, 0, 9);
    return bytes;
}

__global__ void iota_kernel(int *p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

// The sort's identity payload, written on the device (a pageable host copy
// would block the host on the stream's first frame).
hipError_t launch_iota(int *p, int n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, p, n);
    return hipGetLastError();
}

hipError_t launch_fold_counters(const unsigned long long *counters, unsigned long long *out, hipStream_t stream) {
    hipLaunchKernelGGL(fold_counters_kernel, dim3(1), dim3(256), 0, stream, counters, out);
    return hipGetLastError();
}

hipError_t sort_tiles_by_cost(const unsigned *cost, unsigned *cost_sorted, const int *iota, int *order, int n,
                              void *scratch, size_t scratch_bytes, hipStream_t stream) {
    size_t bytes = scratch_bytes;
    return hipcub::DeviceRadixSort::SortPairsDescending(scratch, bytes, cost, cost_sorted, iota, order, n, 0, 9,
                                                        stream);
}


hipError_t launch_render_packet(const SceneDev &S, const FrameDev &F, bool count_tests, hipStream_t stream) {
    if (F.num_tiles <= 0) return hipSuccess;
    const int blocks = (F.num_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (count_tests)
        hipLaunchKernelGGL((render_packet_kernel<true, true>), dim3(blocks), dim3(kBlockThreads), 0,
                           stream, S, F);
    else
        hipLaunchKernelGGL((render_packet_kernel<false, true>), dim3(blocks), dim3(kBlockThreads), 0,
                           stream, S, F);
    return hipGetLastError();
}

hipError_t launch_intersect(const SceneDev &S, const float *rays, int n, int4 *out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int blocks = (n + kBlockThreads - 1) / kBlockThreads;
    hipLaunchKernelGGL(intersect_kernel, dim3(blocks), dim3(kBlockThreads), 0, stream, S, rays, n, out);
    return hipGetLastError();
}

hipError_t launch_assemble(const void *gathered, int res_x, int res_y, int band_count, int band_rows,
                           int local_rows, int pixel_bytes, void *image, hipStream_t stream) {
    const size_t total = (size_t)res_x * res_y;
    if (total == 0) return hipSuccess;
    const int threads = 256;
    const unsigned blocks = (unsigned)((total + threads - 1) / threads);
    if (pixel_bytes == 16)
        hipLaunchKernelGGL(assemble_kernel<float4>, dim3(blocks), dim3(threads), 0, stream, (const float4 *)gathered,
                           res_x, res_y, band_count, band_rows, local_rows, (float4 *)image);
    else if (pixel_bytes == 12)
        hipLaunchKernelGGL(assemble_kernel<Px12>, dim3(blocks), dim3(threads), 0, stream, (const Px12 *)gathered,
                           res_x, res_y, band_count, band_rows, local_rows, (Px12 *)image);
    else if (pixel_bytes == 8)
        hipLaunchKernelGGL(assemble_kernel<uint2>, dim3(blocks), dim3(threads), 0, stream, (const uint2 *)gathered,
                           res_x, res_y, band_count, band_rows, local_rows, (uint2 *)image);
    else if (pixel_bytes == 4)
        hipLaunchKernelGGL(assemble_kernel<unsigned>, dim3(blocks), dim3(threads), 0, stream,
                           (const unsigned *)gathered, res_x, res_y, band_count, band_rows, local_rows,
                           (unsigned *)image);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace rtk
