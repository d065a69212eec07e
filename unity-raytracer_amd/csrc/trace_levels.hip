// trace_levels.hip — the level-synchronous all-packet megakernel (the
// default non-counting path for >= 16 spp on a 4-wide BVH).  A file of its
// own so it is compiled with the default GCN machine scheduler (trace.hip
// uses the memory-clause strategy, which costs this kernel 4 % on C4).
// RayTracingSetup.Shade (Assets/RayTracer/Demo-RayTracing/
// RayTracingSetup.cs:304-366) per sample, exactly as render_kernel.
#include <float.h>

#include <hip/hip_runtime.h>

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

// The 16-spp order's non-sky tiles: keyed by their measured cost (longest
// first; default) or all keyed 1 (row order under the stable sort, the XCD
// stripes' locality kept; measuring builds -DRT_EXP_LVROWKEY=1).
#ifdef RT_EXP_LVROWKEY
constexpr bool kLvRowKeys = RT_EXP_LVROWKEY != 0;
#else
constexpr bool kLvRowKeys = false;
#endif

// Waves per SIMD the register budget must allow: 6 (80 VGPRs, fewer spills in
// the level loop) for up to 16 spp, 7 (72 VGPRs) above (8 until round 5).  Measured (round 3,
// interleaved A/B): C4 (16 spp, depth 8) 6 waves -5 % single frame / -8 %
// frames in flight against 7; C5 (64 spp, depth 16) 6 waves +2 %, 5 waves
// +6 % against 7; 8 waves -1.1 % against 7 (r04l).
#ifdef RT_EXP_LVLOW
constexpr int kLvWavesLowSpp = RT_EXP_LVLOW;  // measuring builds only
#else
constexpr int kLvWavesLowSpp = 6;
#endif
#ifdef RT_EXP_LVHIGH
constexpr int kLvWavesHighSpp = RT_EXP_LVHIGH;  // measuring builds only
#else
constexpr int kLvWavesHighSpp = 7;  // r05k, with the fixed 64-spp shape: C5 -1.9 % against 8
#endif

// Level-synchronous all-packet megakernel (the default non-counting path on
// a 4-wide BVH): one wave = one tile of 64 samples; the Whitted chain
// advances level by level for the whole wave, and every level's rays — the
// camera rays, the mirror rays of the lanes still bouncing, and each level's
// shadow rays — are traced as wave packets (packet.h).  Without a per-lane
// traversal the kernel needs no LDS lane stack and 64-80 VGPRs (8 or 6
// waves/SIMD, kLvWaves*); the mirror fold (c + km*(...), evaluated back to front as the
// recursion rounds) lives in scratch and is touched only by mirror lanes.
// Same arithmetic per sample as render_kernel.  The <= 16-spp instance's
// camera packets start below the top-level cut (below); round 3 measured that
// start +5 % on C4 before the LDS stash of the shadow-packet state freed the
// registers it needs.

// Lane state kept in LDS across a shadow packet (per instance): the 6-wave
// (<= 16 spp) instance stashes the hit (point, normal, view), the colour with
// and without the light and the mirror chain's term — 18 floats a lane, 4.5
// KB a wave — instead of spilling them around the packet loop: C4 HBM writes
// 4.40 -> 0.30 GB per launch, kernel -3 % single frame / -5 % frames in flight
// (profiles/r04/).  The 64-spp instance (8 waves/SIMD: 4.6 KB of LDS a wave
// fits 32 waves per CU) stashes 15 floats — all but the view vector: C5 HBM
// writes 19.6 -> 10.6 GB and reads 9.2 -> 3.4 GB per launch at the same time
// (r04n; 9 floats +1.3 %, 15 at 7 waves +2.4 %, 18 at 7 waves +6 %).
// Tile rows per XCD stripe (render_levels_kernel dispatch), per instance:
// <= 16 spp (2x2-pixel tiles) 1, 64 spp (one-pixel tiles) 4 — C4 -1.6 % with
// 1 against 4, C5 +0.5 % (2: +-0, 16: +2.6 %; r04ad).
#ifdef RT_EXP_XCDROWS
constexpr int kXcdStripeRowsLow = RT_EXP_XCDROWS, kXcdStripeRowsHigh = RT_EXP_XCDROWS;  // measuring builds
#else
constexpr int kXcdStripeRowsLow = 1, kXcdStripeRowsHigh = 4;
#endif

#ifdef RT_EXP_LVSTASH_HI
constexpr int kLvStashHigh = RT_EXP_LVSTASH_HI;  // measuring builds only (0, 9, 15 or 18)
#else
constexpr int kLvStashHigh = 15;
#endif
// RT_SEG_PROFILE (profiling builds only): per-wave shader-clock time of the
// setup, the camera packets (level 0), the shadow packets (every level, with
// their LDS stash), the mirror-ray packets (levels >= 1), the epilogue and the
// whole tile, summed into the (otherwise unused, non-counting) test-counter
// words 3-7 (tools/probe.py reads them); the rest is per-level shading.
#ifdef RT_SEG_PROFILE
#define RT_LSEG(...) __VA_ARGS__
#else
#define RT_LSEG(...)
#endif

// FD: mirror levels the fold stack holds, the frame's MaxReflectionBounces
// rounded up to 8, 16 or 32 (launch_render_levels; deeper frames take the
// megakernel's deep-chain instance): the private segment a wave slot
// reserves shrinks with it (C4, depth 8: 832 -> 256 B per lane).
// FIX: the frame shape fixed at compile time (shade.h rts::Fix): 4 for 16
// spp (2x2-pixel tiles), 8 for 64 spp (one-pixel tiles), 0 for 25 / 36 / 49
// spp — the slot -> sample mapping and the sub-pixel offsets by shifts
// instead of integer and float divisions (C4's per-wave setup was 30 % of
// its wave, seglv_r05h).
template <int MIN_WAVES, int FD = kMaxBounces, int FIX = 0>
__global__ __launch_bounds__(kWaveSize, MIN_WAVES) void render_levels_kernel(SceneDev S, FrameDev F) {
    __shared__ int wstack_mem[rtp::kWaveStack];
    constexpr bool LOW = FIX == 4;  // the 16-spp instance (2x2-pixel tiles)
    constexpr int STASH = LOW ? 18 : kLvStashHigh;  // floats per lane
    // (volatile: reloaded after the packet, so the register copies die at the store)
    __shared__ float stash_mem[(STASH > 0 ? STASH : 1) * kWaveSize];
    const int lane = threadIdx.x & 63;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    // XCD-aware dispatch (blocks b and b + 8 share an XCD, MI355X_MICROARCH.md
    // "Workgroup dispatch"; placement is a speed matter only): XCD group x
    // renders the stripes x, x + 8, ... of kXcdStripeRows* tile rows in row
    // order, so each XCD's L2 serves the geometry of one eighth of the screen
    // instead of all of it — C5 -3 %, C4 -2 % with frames in flight (r04g).
    // A frame's tiles are all here exactly once, whatever the placement.
    // (k / zs, k % zs by the launcher's magic multiplier: no scalar division)
    const int zs = F.lv_zs;
    const int k = blockIdx.x >> 3;
    unsigned q = __umulhi((unsigned)k, F.lv_zs_magic);
    int rk = k - (int)q * zs;
    if (rk >= zs) {
        ++q;
        rk -= zs;
    }
    const int wid = ((int)q * 8 + (blockIdx.x & 7)) * zs + rk;  // the tile itself
    // positions: the frame's tiles in row order, or (F.tile_order: whole 16-spp
    // frames in flight) the last measurement's non-sky tiles — longest first
    // (their measured cost keys), or in row order with kLvRowKeys (every
    // non-sky tile keyed 1: the stable sort keeps row order, so the stripes
    // above keep their locality over the compacted positions) — the sky tail
    // is trace.hip sky_batch_kernel's
    if (wid >= F.num_tiles - F.sky_batch_tiles) return;  // wave-uniform (the last stripes' padding)
    // the tile index in an SGPR (scalar slot -> pixel math, nothing spilled)
    int tile = __builtin_amdgcn_readfirstlane(F.tile_order ? rtt::cload(F.tile_order + wid) : wid);
    if (F.tile_order) RT_FETCH_WAVE(cnt, 4);
    const unsigned long long t0 = F.tile_cost ? __builtin_amdgcn_s_memtime() : 0ull;
    RT_LSEG(const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
            unsigned long long sg_cam = 0, sg_sh = 0, sg_mir = 0, sg_setup = 0;)
    static_assert(FD <= kMaxBounces, "the frame's depth bucket");
    float fold_c[FD][3];
    float fold_k[FD][3];
    int depth = 0;
    f3 term = mk(0.0f, 0.0f, 0.0f);
    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    bool alive;
    bool sky_wave = false;  // (the longest-first measurement's key 0: sky_batch_kernel's next time)
    {
        int px, ly, gy, s;
        alive = rts::slot_pixel<FIX>(F, tile, lane, px, ly, gy, s);
        // a wave whose samples all surely miss the padded Scene.AABB is
        // background without its exact rays (shade.h sky_maybe, as render_kernel)
        // (the <= 16-spp instance: C4 -8 %; at 64 spp, 1-pixel tiles, +1 %)
        const bool sky = LOW &&
                         __ballot(alive && (!F.sky_test || rts::sky_maybe<FIX>(F, px, gy, s))) == 0;
        if (alive) {
            if (!F.wave_counts) cnt.primary = 1;  // otherwise F.primary_total, once per launch
            if (sky)
                term = rtt::ld3(F.bg255);  // :310-311
            else
                rts::primary_ray<FIX>(F, px, gy, s, o, d);
        }
        if (sky) alive = false;
        sky_wave = sky;
    }
    // The <= 16-spp instance's camera packets start below the top-level cut
    // (packet.h cut_select, as render_kernel's): C4 -5.6 % single frame and
    // frames in flight (r04l).  Not at 64 spp: a one-pixel tile's frustum
    // touches most of C5's heavily overlapping top-level boxes, and every
    // waiting entry costs a scalar round trip when popped: C5 +43 %.
    constexpr bool CUT = LOW;
    rtp::CutStart cs = {0, 0, 0, -1};
    if (CUT && F.cut_test && __ballot(alive) != 0) {  // every lane executes here
        const rtp::CutLane cl = rtp::cut_load(S);
        RT_FETCH_WAVE(cnt, 7 * 4 * kCutMax + 4);  // the cut table's SoA entries and count
        cs = rtp::cut_select(S, F, rts::tile_rect<FIX>(F, tile), wstack_mem, &cl);
    }
    RT_LSEG(sg_setup = __builtin_amdgcn_s_memtime() - ts0;)
    for (int level = 0; __ballot(alive) != 0; ++level) {  // wave-uniform
        rtt::RayCtx r;
        rtt::setup_ray(r, o, d);
        rtp::PacketLane P;
        RT_LSEG(const unsigned long long tp0 = __builtin_amdgcn_s_memtime();)
        rtp::packet_trace<false, false, false, false>(S, r, alive, 0.0f, 0.0f, P, wstack_mem, cnt,
                                        CUT && level == 0 ? &cs : nullptr);
        RT_LSEG(const unsigned long long tp = __builtin_amdgcn_s_memtime() - tp0;
                if (level == 0) sg_cam += tp;
                else sg_mir += tp;)
        const bool hit = alive && P.best_rank >= 0;
        if (alive && !hit) term = rtt::ld3(F.bg255);  // :310-311
        rts::Surface sf;
        f3 col = mk(0.0f, 0.0f, 0.0f);
        int mat = 0;
        if (hit) {
            RT_FETCH_LANE(cnt, 16 + 64);  // the hit's shading record and material
            sf = rts::surface(S, o, d, P.best_t, P.best_rank);
            mat = sf.mat;
            col = rts::ambient(S, S.mats[mat]);
        } else {
            sf.p = sf.n = sf.view = mk(0.0f, 0.0f, 1.0f);
            sf.mat = 0;
        }
        for (int l = 0; l < S.num_lights; ++l) {  // :327-356, wave-uniform
            RT_FETCH_WAVE(cnt, 32);
            const DevLight Lt = S.lights[l];
            const rts::ShadowRay sr = rts::shadow_ray(sf, Lt);
            if (hit) cnt.shadow++;
            // a moot shadow ray (shade.h same_bits) is not traced
            f3 lit = col + rts::light_term(S, sf, S.mats[mat], Lt, sr);
            const bool trace = hit && !rts::same_bits(lit, col);
            cnt.moot += hit && !trace;
            rtt::RayCtx rs;
            rtt::setup_ray(rs, sr.o, sr.dir);
            rtp::PacketLane Q;
            RT_LSEG(const unsigned long long tq0 = __builtin_amdgcn_s_memtime();)
            if (STASH > 0) {
                volatile float *vs = stash_mem + rtt::lane_id();
                const float v[18] = {col.x, col.y, col.z, lit.x, lit.y, lit.z, term.x, term.y, term.z,
                                     sf.p.x, sf.p.y, sf.p.z, sf.n.x, sf.n.y, sf.n.z, sf.view.x, sf.view.y, sf.view.z};
#pragma unroll
                for (int i = 0; i < STASH; ++i) vs[i * kWaveSize] = v[i];
                rtp::packet_trace<true, false, false, false>(S, rs, trace, sqrtf(sr.d2) * 1.001f, sr.d2, Q, wstack_mem, cnt);
                vs = stash_mem + rtt::lane_id();
                col = mk(vs[0], vs[64], vs[128]);
                lit = mk(vs[192], vs[256], vs[320]);
                term = mk(vs[384], vs[448], vs[512]);
                if (STASH >= 15) {
                    sf.p = mk(vs[576], vs[640], vs[704]);
                    sf.n = mk(vs[768], vs[832], vs[896]);
                }
                if (STASH >= 18) sf.view = mk(vs[960], vs[1024], vs[1088]);
            } else {
                rtp::packet_trace<true, false, false, false>(S, rs, trace, sqrtf(sr.d2) * 1.001f, sr.d2, Q, wstack_mem, cnt);
            }
            RT_LSEG(sg_sh += __builtin_amdgcn_s_memtime() - tq0;)
            if (trace && Q.best_rank != 1) col = lit;
        }
        bool mirror = false;
        if (hit) {
            const DevMaterial m = S.mats[mat];
            mirror = m.ka_mirror.w != 0.0f && level < F.max_bounces;  // :358
            if (mirror) {
                fold_c[depth][0] = col.x; fold_c[depth][1] = col.y; fold_c[depth][2] = col.z;
                fold_k[depth][0] = m.km.x; fold_k[depth][1] = m.km.y; fold_k[depth][2] = m.km.z;
                rts::reflect(sf, o, d);
                ++depth;
                cnt.reflection++;
            } else {
                term = col;
            }
        }
        alive = mirror;
    }
    RT_LSEG(const unsigned long long te0 = __builtin_amdgcn_s_memtime();)
    for (int k = depth - 1; k >= 0; --k)
        term = mk(fold_c[k][0], fold_c[k][1], fold_c[k][2]) + mk(fold_k[k][0], fold_k[k][1], fold_k[k][2]) * term;
    // lane ids recomputed (rtt::lane_id), not kept live across the levels
    const int lane2 = rtt::lane_id();
    // A pixel's samples summed in sample order (row-major, ((s0 + s1) + s2)
    // + ...) through LDS: every lane writes its sample to the stash area (free
    // here) once, then each pixel's sample-0 lane reads its pixel's samples
    // back four at a time (three aligned float4 reads) and adds them in order
    // — the same sums as rts::sample_sum's (spp - 1) x 3 whole-wave lane
    // shuffles with a small fraction of their LDS traffic: C5 (64 spp)
    // -7.8 %, C4 (16 spp) -3.2 %, bit-identical (r05g).
    f3 sum = term;
    if (FIX != 0) {  // 16 or 64 spp (sample-0 lanes 16-aligned); 25 / 36 / 49 spp take the shuffles
        float *sm = stash_mem;
        sm[lane2 * 3 + 0] = term.x;
        sm[lane2 * 3 + 1] = term.y;
        sm[lane2 * 3 + 2] = term.z;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        constexpr int SPP = FIX * FIX;
        if ((lane2 & (SPP - 1)) == 0) {
            const float4 *q = reinterpret_cast<const float4 *>(sm + lane2 * 3);
            for (int k = 0; k < SPP; k += 4) {  // 4 samples = 12 floats
                const float4 a = q[0], b = q[1], c = q[2];
                q += 3;
                sum = k == 0 ? mk(a.x, a.y, a.z) : sum + mk(a.x, a.y, a.z);
                sum = sum + mk(a.w, b.x, b.y);
                sum = sum + mk(b.z, b.w, c.x);
                sum = sum + mk(c.y, c.z, c.w);
            }
        }
    } else {
        sum = rts::sample_sum(term, lane2, F.spp);
    }
    {
        int tile2 = __builtin_amdgcn_readfirstlane(tile);
        asm volatile("" : "+s"(tile2));
        int px, ly, gy, s;
        if (rts::slot_pixel<FIX>(F, tile2, lane2, px, ly, gy, s) && s == 0) {
            f3 v = sum;
            if (F.spp > 1) v = (F.spp & (F.spp - 1)) == 0 ? v * F.inv_spp : v / (float)F.spp;
            rts::store_pixel(F, (size_t)ly * F.res_x + px, v);
        }
    }
    if (F.tile_cost && lane2 == 0) {  // (16 spp: the sky flag is what the order is for)
        const unsigned c = (unsigned)min(__builtin_amdgcn_s_memtime() - t0, 0xffffffffull);
        const unsigned e = c ? 31u - __clz(c) : 0u;
        F.tile_cost[tile] = sky_wave ? 0u
                            : kLvRowKeys ? 1u
                                         : max(1u, e < 4 ? c : (((e - 3u) << 4) | ((c >> (e - 4u)) & 15u)));
    }
#ifdef RT_SEG_PROFILE
    if (lane2 == 0) {  // the clocks are wave-uniform
        const unsigned long long te1 = __builtin_amdgcn_s_memtime();
        unsigned long long *ctr = F.counters + (size_t)(blockIdx.x % kCounterSlots) * kCounterWords;
        // setup (slot, sky test, primary rays, cut) and epilogue (fold, sample sum, store) in 16-cycle units
        atomicAdd(ctr + 3, (sg_setup >> 4) | (((te1 - te0) >> 4) << 32));
        atomicAdd(ctr + 4, sg_cam);
        atomicAdd(ctr + 5, sg_sh);
        atomicAdd(ctr + 6, te1 - ts0);
        atomicAdd(ctr + 7, sg_mir);
    }
#endif
    if (F.wave_counts) {  // plain store, reduced after the launch (trace.hip wave_counts_kernel)
        unsigned sh = 0, rf = 0, mo = 0;
        if (__ballot((cnt.shadow | cnt.reflection | cnt.moot) != 0) != 0) {
            sh = rtt::wave_sum(cnt.shadow);
            rf = rtt::wave_sum(cnt.reflection);
            mo = rtt::wave_sum(cnt.moot);
        }
        if (lane2 == 0) F.wave_counts[wid] = make_uint4(sh, rf, mo, F.count_tag);
    } else {
        rtt::flush_counts<false>(cnt, F.counters);
    }
#ifdef RT_FETCH_COUNT
    {  // measuring builds: the wave's fetched bytes into counter word 9 (traverse.h RT_FETCH_*)
        const unsigned fb = rtt::wave_sum(cnt.fetch);
        if (lane2 == 0 && fb) atomicAdd(rtt::counter_slot(F.counters) + 9, (unsigned long long)fb);
    }
#endif
}

}  // namespace

namespace rtk {

hipError_t launch_render_levels(const SceneDev &S, const FrameDev &F0, hipStream_t stream) {
    if (F0.num_tiles <= 0) return hipSuccess;
    FrameDev F = F0;
    // whole groups of eight stripes (render_levels_kernel's XCD-aware dispatch)
    const long long rows = F.spp <= 16 ? kXcdStripeRowsLow : kXcdStripeRowsHigh;  // the instance launched below
    const long long zs = rows * F.tiles_x, ns = (F.num_tiles - F.sky_batch_tiles + zs - 1) / zs;
    F.lv_zs = (int)zs;
    F.lv_zs_magic = zs <= 1 ? 0xffffffffu : (unsigned)((1ull << 32) / (unsigned long long)zs);
    const long long grid = 8 * ((ns + 7) / 8) * zs;
    if (grid > 0x7fffffffll) return hipErrorInvalidValue;
    const dim3 g((unsigned)grid), b(kWaveSize);
    // the fold stack's depth bucket (render_levels_kernel FD); frames deeper
    // than kMaxBounces never come here (rt_frame.cpp frame_path)
    const int fd = F.max_bounces <= 8 ? 8 : F.max_bounces <= 16 ? 16 : kMaxBounces;
    if (F.spp <= 16) {  // 16 spp: FIX 4
        if (fd == 8)
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesLowSpp, 8, 4>), g, b, 0, stream, S, F);
        else if (fd == 16)
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesLowSpp, 16, 4>), g, b, 0, stream, S, F);
        else
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesLowSpp, kMaxBounces, 4>), g, b, 0, stream, S, F);
    } else if (F.spp == 64) {
        if (fd == 8)
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesHighSpp, 8, 8>), g, b, 0, stream, S, F);
        else if (fd == 16)
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesHighSpp, 16, 8>), g, b, 0, stream, S, F);
        else
            hipLaunchKernelGGL((render_levels_kernel<kLvWavesHighSpp, kMaxBounces, 8>), g, b, 0, stream, S, F);
    } else {  // 25 / 36 / 49 spp
        hipLaunchKernelGGL((render_levels_kernel<kLvWavesHighSpp, kMaxBounces, 0>), g, b, 0, stream, S, F);
    }
    return hipGetLastError();
}

}  // namespace rtk
