// trace_wf.hip — gfx950 wavefront render path (see wavefront.h for the pass
// structure).  Traversal passes are persistent: every wave keeps 64 lanes
// busy by fetching new rays from the level's queue (one atomic per wave,
// ballot + mbcnt to hand out slots) whenever a quarter of its lanes went idle,
// so the wave never waits on its slowest ray.  Shading passes are plain
// grid-stride loops.  Same arithmetic as the megakernel — results are
// bit-identical (tests/test_gpu_parity.py runs both).
#include <float.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "rt_device.h"
#include "rt_math.h"
#include "shade.h"
#include "traverse.h"
#include "wavefront.h"

using namespace rtd;
using rtm::f3;
using rtm::mk;
using rtt::Counts;

namespace {

constexpr int kRefill = 16;   // refill when at least this many lanes are idle
constexpr int kChunk = 1024;  // max slots per dynamic reservation

__device__ __forceinline__ int level_begin(const rtw::Counters *c, int level) {
    int b = 0;
    for (int j = 0; j < level; ++j) b += c->n[j];
    return b;
}

__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }

__device__ __forceinline__ unsigned long long lanes_below(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Persistent traversal over one queue.  ANY: shadow queue of level `level`;
// otherwise closest hits of level `level` (PRIMARY: level 0, rays regenerated).
//
// Work distribution: a wave owns a reservation of `chunk` consecutive queue
// slots (its first one static, later ones by ONE atomic on the level's head —
// a single dequeue word saturates near 88 atomics/us on MI355X, so fetching
// 64 rays per atomic would be atomic-bound).  Whenever kRefill lanes are
// idle they are refilled from the reservation with ballot + mbcnt, so lanes
// never wait for the wave's slowest ray.
template <bool ANY, bool PRIMARY, bool COUNT>
__global__ __launch_bounds__(kBlockThreads) void wf_trace(SceneDev S, FrameDev F, rtw::Args A, int level) {
    __shared__ int stack_mem[kWavesPerBlock * kStackSize * kWaveSize];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int ovf[kStackTotal - kStackSize];
    const rtt::Stack st{stack_mem + wave * kStackSize * kWaveSize + lane, ovf};
    const int n_level = PRIMARY ? A.n0 : A.ctr->n[level];
    const int count = ANY ? n_level * S.num_lights : n_level;
    const int base = (ANY || PRIMARY) ? 0 : level_begin(A.ctr, level);
    const int nwaves = gridDim.x * kWavesPerBlock;
    const int gw = blockIdx.x * kWavesPerBlock + wave;
    // reservation size: spread small queues over every wave, cap large ones
    int chunk = (count / nwaves + 63) & ~63;
    chunk = chunk < 64 ? 64 : (chunk > kChunk ? kChunk : chunk);
    int res = gw * chunk;  // static first reservation
    if (res >= count) return;  // wave-uniform: no work, no atomic
    int res_end = res + chunk < count ? res + chunk : count;
    int *head = ANY ? &A.ctr->head_a[level] : &A.ctr->head_c[level];
    const int dyn0 = nwaves * chunk;  // dynamic reservations start after the static ones
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    bool has = false, exhausted = false;
    int idx = 0;
    float d2 = 0.0f;
    rtt::RayCtx r;
    rtt::Trav t;
    while (true) {
        const unsigned long long idle = __ballot(!has);
        const int n_idle = __popcll(idle);
        if (!exhausted && n_idle >= kRefill) {
            if (res >= res_end) {  // reservation used up: reserve another chunk
                int b = 0;
                if (lane == 0) b = atomicAdd(head, chunk);
                b = __shfl(b, 0) + dyn0;
                res = b;
                res_end = b + chunk < count ? b + chunk : count;
            }
            if (res >= count) {
                exhausted = true;
            } else {
                const int my = res + __popcll(idle & lanes_below(lane));
                const int avail = res_end - res;
                res += n_idle < avail ? n_idle : avail;
                if (!has && my < res_end) {
                    idx = my;
                    f3 o, d;
                    bool live = true;
                    if (ANY) {
                        const float4 so = A.sh_o[my];
                        live = so.w != 0.0f;  // slot of a hit (shade wrote 1) or of a miss (0)
                        if (live) {
                            const float4 sd = A.sh_d[my];
                            o = xyz(so);
                            d = xyz(sd);
                            d2 = sd.w;
                        }
                    } else if (PRIMARY) {
                        int px, ly, gy, s;
                        live = rts::slot_pixel(F, A.tile0 + (my >> 6), my & 63, px, ly, gy, s);
                        if (live) rts::primary_ray(F, px, gy, s, o, d);
                    } else {
                        o = xyz(A.ray_o[base + my]);
                        d = xyz(A.ray_d[base + my]);
                    }
                    if (!live) {
                        if (!ANY) A.hit[my] = make_int4(-2, 0, -1, 0);
                    } else {
                        rtt::setup_ray(r, o, d);
                        const float tl = ANY ? sqrtf(d2) * 1.001f : 0.0f;
                        if (rtt::trav_begin<ANY, COUNT>(S, r, tl, t, cnt)) {
                            has = true;
                        } else if (ANY) {
                            A.occ[my] = 0;
                        } else {
                            A.hit[base + my] = make_int4(-1, __float_as_int(FLT_MAX), -1, 0);
                        }
                    }
                }
            }
        }
        if (__ballot(has) == 0) {
            if (exhausted) break;
            continue;
        }
        while (true) {
            if (has && rtt::trav_step<ANY, COUNT>(S, r, t, d2, st, cnt)) {
                has = false;
                if (ANY)
                    A.occ[idx] = t.best_rank == 1 ? 1 : 0;
                else
                    A.hit[base + idx] = make_int4(t.best_rank, __float_as_int(t.best_t), -1, 0);
            }
            const unsigned long long busy = __ballot(has);
            if (busy == 0) break;
            if (!exhausted && 64 - __popcll(busy) >= kRefill) break;
        }
    }
    if (COUNT) rtt::flush_counts<true>(cnt, F.counters);
}

// Wave-aggregated queue allocation: returns this lane's slot (if want).
__device__ __forceinline__ int wave_alloc(int *counter, bool want, int per_lane, int lane) {
    const unsigned long long m = __ballot(want);
    int b = 0;
    if (lane == 0 && m) b = atomicAdd(counter, __popcll(m) * per_lane);
    b = __shfl(b, 0);
    return b + __popcll(m & lanes_below(lane)) * per_lane;
}

template <bool PRIMARY>
__device__ __forceinline__ void entry_ray(const FrameDev &F, const rtw::Args &A, int e, f3 &o, f3 &d) {
    if (PRIMARY) {
        int px, ly, gy, s;
        rts::slot_pixel(F, A.tile0 + (e >> 6), e & 63, px, ly, gy, s);
        rts::primary_ray(F, px, gy, s, o, d);
    } else {
        o = xyz(A.ray_o[e]);
        d = xyz(A.ray_d[e]);
    }
}

// shade(k): misses get the background, hits emit one shadow ray per light
// (:329-333) and, on a mirror below the bounce limit, the reflection ray of
// level k+1 (:358-363, Reflect :368-373).
template <bool PRIMARY, bool COUNT>
__global__ __launch_bounds__(kBlockThreads) void wf_shade(SceneDev S, FrameDev F, rtw::Args A, int level) {
    const int lane = threadIdx.x & 63;
    const int count = PRIMARY ? A.n0 : A.ctr->n[level];
    const int base = PRIMARY ? 0 : level_begin(A.ctr, level);
    const int next_base = base + count;
    const int L = S.num_lights;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    const int nwaves = gridDim.x * kWavesPerBlock;
    for (int w = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); w * 64 < count; w += nwaves) {
        const int i = w * 64 + lane;
        const bool valid = i < count;
        const int e = base + i;
        int4 h = valid ? A.hit[e] : make_int4(-2, 0, -1, 0);
        const bool is_hit = valid && h.x >= 0;
        if (PRIMARY && valid && h.x != -2) cnt.primary++;
        rts::Surface sf;
        DevMaterial m;
        f3 o = mk(0, 0, 0), d = mk(0, 0, 0);
        bool mirror = false;
        if (is_hit) {
            entry_ray<PRIMARY>(F, A, e, o, d);
            sf = rts::surface(S, o, d, __int_as_float(h.y), h.x);
            m = S.mats[sf.mat];
            mirror = m.ka_mirror.w != 0.0f && level < A.max_level && level < F.max_bounces;
            if (COUNT) cnt.shading++;
        }
        // shadow rays of entry i live at slots i*L .. i*L+L-1 (no allocation);
        // .w of the origin marks a live slot
        const int sbase = i * L;
        if (is_hit) {
            for (int l = 0; l < L; ++l) {
                const rts::ShadowRay sr = rts::shadow_ray(sf, S.lights[l]);
                A.sh_o[sbase + l] = make_float4(sr.o.x, sr.o.y, sr.o.z, 1.0f);
                A.sh_d[sbase + l] = make_float4(sr.dir.x, sr.dir.y, sr.dir.z, sr.d2);
            }
            cnt.shadow += L;
        } else if (valid) {
            for (int l = 0; l < L; ++l) A.sh_o[sbase + l] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        const int slot = wave_alloc(&A.ctr->n[level + 1 < rtw::kMaxLevels ? level + 1 : level], mirror, 1, lane);
        int child = -1;
        if (mirror) {
            f3 ro, rd;
            rts::reflect(sf, ro, rd);
            child = next_base + slot;
            A.ray_o[child] = make_float4(ro.x, ro.y, ro.z, 0.0f);
            A.ray_d[child] = make_float4(rd.x, rd.y, rd.z, 0.0f);
            cnt.reflection++;
        }
        if (valid) {
            if (h.x == -2) {
                A.col[e] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
            } else if (h.x < 0) {  // miss: new Rgb(BackgroundColor), :310-311
                A.col[e] = make_float4(F.bg255[0], F.bg255[1], F.bg255[2], __int_as_float(-1));
            } else {
                A.hit[e].z = sbase;
                A.col[e].w = __int_as_float(child);
            }
        }
    }
    rtt::flush_counts<COUNT>(cnt, F.counters);
}

// finish(k): color = ambient; += diffuse + specular of every unoccluded
// light, in scene order (:324, :327-356).
template <bool PRIMARY>
__global__ __launch_bounds__(kBlockThreads) void wf_finish(SceneDev S, FrameDev F, rtw::Args A, int level) {
    const int count = PRIMARY ? A.n0 : A.ctr->n[level];
    const int base = PRIMARY ? 0 : level_begin(A.ctr, level);
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const int e = base + i;
        const int4 h = A.hit[e];
        if (h.x < 0) continue;
        f3 o, d;
        entry_ray<PRIMARY>(F, A, e, o, d);
        const rts::Surface sf = rts::surface(S, o, d, __int_as_float(h.y), h.x);
        const DevMaterial m = S.mats[sf.mat];
        f3 col = rts::ambient(S, m);
        for (int l = 0; l < S.num_lights; ++l) {
            if (A.occ[h.z + l]) continue;
            const DevLight Lt = S.lights[l];
            col = col + rts::light_term(S, sf, m, Lt, rts::shadow_ray(sf, Lt));
        }
        float4 c = A.col[e];
        c.x = col.x;
        c.y = col.y;
        c.z = col.z;
        A.col[e] = c;
    }
}

// fold(k): Shade's `color += new Rgb(mirrorReflectance * Shade(...).Value)`
// (:362) applied back to front: level k+1 is final when level k folds.
__global__ __launch_bounds__(kBlockThreads) void wf_fold(SceneDev S, rtw::Args A, int level) {
    const int count = level == 0 ? A.n0 : A.ctr->n[level];
    const int base = level == 0 ? 0 : level_begin(A.ctr, level);
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const int e = base + i;
        const float4 c = A.col[e];
        const int child = __float_as_int(c.w);
        if (child < 0) continue;
        const int rank = A.hit[e].x;
        const DevMaterial m = S.mats[__float_as_int(S.shade[rank].w)];
        const float4 r = A.col[child];
        const f3 res = xyz(c) + mk(m.km.x, m.km.y, m.km.z) * xyz(r);
        A.col[e] = make_float4(res.x, res.y, res.z, c.w);
    }
}

// resolve: ((s0 + s1) + s2) + ... per pixel, / spp, / 255 (Rgb.Color, Rgb.cs:13).
__global__ __launch_bounds__(kBlockThreads) void wf_resolve(FrameDev F, rtw::Args A) {
    const int ppw = F.tile_w * F.tile_h;
    const int total = (A.n0 >> 6) * ppw;
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int tl = i / ppw, pix = i - tl * ppw;
        const int lane0 = pix * F.spp;
        int px, ly, gy, s;
        if (!rts::slot_pixel(F, A.tile0 + tl, lane0, px, ly, gy, s)) continue;
        const int e0 = tl * 64 + lane0;
        f3 sum = xyz(A.col[e0]);
        for (int k = 1; k < F.spp; ++k) sum = sum + xyz(A.col[e0 + k]);
        if (F.spp > 1) sum = sum / (float)F.spp;
        rts::store_pixel(F, (size_t)ly * F.res_x + px, sum);
    }
}

__global__ void wf_reset(rtw::Args A) {
    const int i = threadIdx.x;
    if (i < rtw::kMaxLevels) {
        A.ctr->n[i] = i == 0 ? A.n0 : 0;
        A.ctr->shadow_n[i] = 0;
        A.ctr->head_c[i] = 0;
        A.ctr->head_a[i] = 0;
    }
}

// Grid of a persistent kernel: every CU filled to its occupancy limit.
template <typename K>
int persistent_blocks(K kernel) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1024;
        cus = prop.multiProcessorCount;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlockThreads, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    return cus * per_cu;
}

}  // namespace

namespace rtk {

hipError_t launch_render_wavefront(const SceneDev &S, const FrameDev &F, const rtw::Args &A0, int chunk_tiles,
                                   bool count, hipStream_t stream) {
    const int levels = (F.max_bounces > 0 ? F.max_bounces : 0) + 1;
    const int grid = 2048;
    for (int t0 = 0; t0 < F.num_tiles; t0 += chunk_tiles) {
        rtw::Args A = A0;
        A.tile0 = t0;
        A.n0 = (F.num_tiles - t0 < chunk_tiles ? F.num_tiles - t0 : chunk_tiles) * 64;
        A.max_level = levels - 1;
        hipLaunchKernelGGL(wf_reset, dim3(1), dim3(64), 0, stream, A);
        for (int k = 0; k < levels; ++k) {
            const bool p = k == 0;
#define RT_LAUNCH_TRACE(ANY, PRIM)                                                                              \
    do {                                                                                                        \
        if (count) {                                                                                            \
            auto kern = wf_trace<ANY, PRIM, true>;                                                              \
            hipLaunchKernelGGL(kern, dim3(persistent_blocks(kern)), dim3(kBlockThreads), 0, stream, S, F, A, k); \
        } else {                                                                                                \
            auto kern = wf_trace<ANY, PRIM, false>;                                                             \
            hipLaunchKernelGGL(kern, dim3(persistent_blocks(kern)), dim3(kBlockThreads), 0, stream, S, F, A, k); \
        }                                                                                                       \
    } while (0)
            if (p)
                RT_LAUNCH_TRACE(false, true);
            else
                RT_LAUNCH_TRACE(false, false);
            if (p) {
                if (count)
                    hipLaunchKernelGGL((wf_shade<true, true>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A, k);
                else
                    hipLaunchKernelGGL((wf_shade<true, false>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A, k);
            } else {
                if (count)
                    hipLaunchKernelGGL((wf_shade<false, true>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A, k);
                else
                    hipLaunchKernelGGL((wf_shade<false, false>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A,
                                       k);
            }
            if (S.num_lights > 0) RT_LAUNCH_TRACE(true, false);
#undef RT_LAUNCH_TRACE
            if (p)
                hipLaunchKernelGGL((wf_finish<true>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A, k);
            else
                hipLaunchKernelGGL((wf_finish<false>), dim3(grid), dim3(kBlockThreads), 0, stream, S, F, A, k);
        }
        for (int k = levels - 2; k >= 0; --k)
            hipLaunchKernelGGL(wf_fold, dim3(grid), dim3(kBlockThreads), 0, stream, S, A, k);
        hipLaunchKernelGGL(wf_resolve, dim3(grid), dim3(kBlockThreads), 0, stream, F, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace rtk
