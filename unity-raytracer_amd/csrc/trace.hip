// trace.hip — gfx950 kernels of the per-pixel trace path.
//
// Reference: RayTracingSetup.CastPixelRays/Shade (Assets/RayTracer/Demo-RayTracing/
// RayTracingSetup.cs:275-455), Scene.IntersectRay (Data/Objects/Scene.cs:43-122),
// RMath (Math/RMath.cs:12-108).  Brute-force scan → BVH2 traversal with an
// LDS stack; results are identical (rt_device.h: ranks, gates, padding).
//
// Execution shape: one wave64 = one tile of pixels x all their samples
// (spp lanes per pixel, consecutive), so a pixel's samples are summed in the
// documented fixed order with cross-lane moves and no atomics.  Branchy scalar
// FP32 — no MFMA.  Built with -ffp-contract=off and correctly rounded f32
// divide/sqrt so every reference operation rounds exactly once.
#include <float.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "rt_device.h"
#include "rt_math.h"

using namespace rtd;
using rtm::f3;
using rtm::mk;

namespace {

struct Counts {
    unsigned primary, shadow, reflection, box, tri, sph, shading;
};

struct RayCtx {
    f3 o, d;     // exact ray (reference semantics)
    f3 inv;      // rcp(dir) = 1.0f / dir, exact — reference AABB gates
    f3 ninv;     // node-test inverse (zero components nudged, approx rcp)
    f3 noi;      // o * ninv
};

__device__ __forceinline__ float nudge(float v) {
    return fabsf(v) > 1e-20f ? v : copysignf(1e-20f, v);
}

__device__ __forceinline__ void setup_ray(RayCtx &r, f3 o, f3 d) {
    r.o = o;
    r.d = d;
    r.inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    r.ninv = mk(__builtin_amdgcn_rcpf(nudge(d.x)), __builtin_amdgcn_rcpf(nudge(d.y)),
                __builtin_amdgcn_rcpf(nudge(d.z)));
    r.noi = mk(o.x * r.ninv.x, o.y * r.ninv.y, o.z * r.ninv.z);
}

__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

// Conservative slab test of both children of a node (padded boxes; FMA form).
__device__ __forceinline__ void test_children(const float4 a, const float4 b, const float4 c,
                                              const RayCtx &r, float tcull, bool &h0, bool &h1,
                                              float &tn0, float &tn1) {
    const float l0x = fmaf(a.x, r.ninv.x, -r.noi.x), u0x = fmaf(a.y, r.ninv.x, -r.noi.x);
    const float l0y = fmaf(a.z, r.ninv.y, -r.noi.y), u0y = fmaf(a.w, r.ninv.y, -r.noi.y);
    const float l0z = fmaf(c.x, r.ninv.z, -r.noi.z), u0z = fmaf(c.y, r.ninv.z, -r.noi.z);
    const float l1x = fmaf(b.x, r.ninv.x, -r.noi.x), u1x = fmaf(b.y, r.ninv.x, -r.noi.x);
    const float l1y = fmaf(b.z, r.ninv.y, -r.noi.y), u1y = fmaf(b.w, r.ninv.y, -r.noi.y);
    const float l1z = fmaf(c.z, r.ninv.z, -r.noi.z), u1z = fmaf(c.w, r.ninv.z, -r.noi.z);
    tn0 = fmaxf(fmaxf(fminf(l0x, u0x), fminf(l0y, u0y)), fmaxf(fminf(l0z, u0z), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(l0x, u0x), fmaxf(l0y, u0y)), fminf(fmaxf(l0z, u0z), tcull));
    tn1 = fmaxf(fmaxf(fminf(l1x, u1x), fminf(l1y, u1y)), fmaxf(fminf(l1z, u1z), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(l1x, u1x), fmaxf(l1y, u1y)), fminf(fmaxf(l1z, u1z), tcull));
    h0 = tn0 <= tf0;
    h1 = tn1 <= tf1;
}

// Scene.IntersectRay over the BVH.  ANY = shadow query: true as soon as a
// hit with t*t < d2 exists (≡ the reference's closest-hit-then-compare,
// RayTracingSetup.cs:333-345, because t >= 0 makes t -> t*t monotone).
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool traverse(const SceneDev &S, const RayCtx &r, float tlimit, float d2,
                                         float &best_t, int &best_rank, int *__restrict__ st,
                                         Counts &cnt) {
    if (COUNT) cnt.box++;
    if (!S.has_prims ||
        !rtm::ref_slab(r.o, r.inv, ld3(S.scene_lo), ld3(S.scene_hi)))  // Scene.cs:54
        return false;
    int sp = 0;
    int node = 0;
    int gate_cached = -1;
    bool gate_ok = false;
    float tcull = ANY ? tlimit : best_t;
    while (true) {
        if (node >= 0) {
            const BvhNode *np = S.nodes + node;
            const float4 a = np->a, b = np->b, c = np->c;
            const int4 ch = np->d;
            bool h0, h1;
            float tn0, tn1;
            test_children(a, b, c, r, tcull, h0, h1, tn0, tn1);
            if (COUNT) cnt.box += 2;
            if (h0 && h1) {
                const bool first0 = tn0 <= tn1;
                st[sp * kWaveSize] = first0 ? ch.y : ch.x;
                ++sp;
                node = first0 ? ch.x : ch.y;
                continue;
            }
            if (h0) { node = ch.x; continue; }
            if (h1) { node = ch.y; continue; }
        } else {
            const LeafDesc L = S.leaves[~node];
            bool ok = true;
            if (L.gate >= 0) {  // the reference's per-mesh AABB gate, Scene.cs:67
                if (L.gate != gate_cached) {
                    gate_cached = L.gate;
                    const MeshGate g = S.gates[L.gate];
                    gate_ok = rtm::ref_slab(r.o, r.inv, mk(g.lo.x, g.lo.y, g.lo.z),
                                            mk(g.hi.x, g.hi.y, g.hi.z));
                    if (COUNT) cnt.box++;
                }
                ok = gate_ok;
            }
            if (ok) {
                if (L.kind == kLeafTri) {
                    for (int i = 0; i < L.count; ++i) {
                        const TriRec tr = S.tris[L.first + i];
                        float t;
                        if (COUNT) cnt.tri++;
                        if (rtm::ref_triangle(r.o, r.d, mk(tr.p0.x, tr.p0.y, tr.p0.z),
                                              mk(tr.p0.w, tr.p1.x, tr.p1.y),
                                              mk(tr.p1.z, tr.p1.w, tr.p2.x), t)) {
                            const int rank = __float_as_int(tr.p2.y);
                            if (ANY) {
                                if (t * t < d2) return true;
                            } else if (t < best_t || (t == best_t && rank < best_rank)) {
                                best_t = t;
                                best_rank = rank;
                                tcull = t;
                            }
                        }
                    }
                } else {
                    for (int i = 0; i < L.count; ++i) {
                        const SphRec sr = S.sphs[L.first + i];
                        float t;
                        if (COUNT) cnt.sph++;
                        if (rtm::ref_sphere(r.o, r.d, mk(sr.cr.x, sr.cr.y, sr.cr.z), sr.cr.w, t)) {
                            const int rank = sr.misc.x;
                            if (ANY) {
                                if (t * t < d2) return true;
                            } else if (t < best_t || (t == best_t && rank < best_rank)) {
                                best_t = t;
                                best_rank = rank;
                                tcull = t;
                            }
                        }
                    }
                }
            }
        }
        if (sp == 0) break;
        --sp;
        node = st[sp * kWaveSize];
    }
    return ANY ? false : best_rank >= 0;
}

// Shade (RayTracingSetup.cs:304-366) with the mirror recursion unrolled into
// a loop; the recursion's results are folded back to front so
// c0 + km0*(c1 + km1*(...)) rounds exactly like the reference.
template <bool COUNT>
__device__ __forceinline__ f3 shade_path(const SceneDev &S, const FrameDev &F, f3 o, f3 d, int *st,
                                         Counts &cnt) {
    float fold_c[kMaxBounces][3];
    float fold_k[kMaxBounces][3];
    int depth = 0;
    f3 term;
    const f3 ambient = ld3(S.ambient);
    while (true) {
        RayCtx r;
        setup_ray(r, o, d);
        float bt = FLT_MAX;  // float.MaxValue, Scene.cs:45
        int br = -1;
        const bool hit = traverse<false, COUNT>(S, r, 0.0f, 0.0f, bt, br, st, cnt);
        if (!hit) {  // :310-311
            term = ld3(F.bg255);
            break;
        }
        if (COUNT) cnt.shading++;
        const f3 p = o + d * bt;  // Ray.GetPoint, Ray.cs:18-21
        const float4 sh = S.shade[br];
        const int mat_id = __float_as_int(sh.w);
        f3 n;
        if (br >= S.mesh_tri_total && br < S.mesh_tri_total + S.sphere_count)
            n = rtm::normalize(p - mk(sh.x, sh.y, sh.z));  // GetSphereNormal :402-407
        else
            n = mk(sh.x, sh.y, sh.z);                       // :422, :428
        const DevMaterial m = S.mats[mat_id];
        const f3 kd = mk(m.kd_phong.x, m.kd_phong.y, m.kd_phong.z);
        const f3 ks = mk(m.ks.x, m.ks.y, m.ks.z);
        f3 col = ambient * mk(m.ka_mirror.x, m.ka_mirror.y, m.ka_mirror.z);  // :438-441
        const f3 view = rtm::normalize(o - p);                                // :325
        for (int l = 0; l < S.num_lights; ++l) {                              // :327-356
            const DevLight L = S.lights[l];
            const f3 lp = mk(L.pos.x, L.pos.y, L.pos.z);
            const f3 lmp = lp - p;
            const f3 ldir = rtm::normalize(lmp);
            const f3 so = p + n * rtm::kShadowEpsilon;
            const float d2 = rtm::dot(lmp, lmp);  // distancesq(P, L) = lengthsq(L - P)
            cnt.shadow++;
            RayCtx sr;
            setup_ray(sr, so, ldir);
            float dt = 0.0f;
            int dr = -1;
            if (traverse<true, COUNT>(S, sr, sqrtf(d2) * 1.001f, d2, dt, dr, st, cnt)) continue;
            const f3 e = mk(L.intensity.x, L.intensity.y, L.intensity.z) / d2;  // :350
            const float ldn = rtm::dot(ldir, n);
            const f3 diffuse = (kd * rtm::umax(0.0f, ldn)) * e;  // CalculateDiffuse :443-455
            f3 spec = mk(0.0f, 0.0f, 0.0f);
            // CalculateSpecular :375-400; degrees(acos(ldn)) > 90f  <=>  ldn < threshold
            if (!(ldn < S.spec_threshold)) {
                const f3 v = ldir + view;
                const f3 h = v / rtm::length(v);
                const float cnh = rtm::umax(0.0f, rtm::dot(n, h));
                const float pw = (float)pow((double)cnh, (double)m.kd_phong.w);
                spec = (ks * pw) * e;
            }
            col = col + (diffuse + spec);
        }
        if (m.ka_mirror.w != 0.0f && depth < F.max_bounces) {  // :358-363
            fold_c[depth][0] = col.x; fold_c[depth][1] = col.y; fold_c[depth][2] = col.z;
            fold_k[depth][0] = m.km.x; fold_k[depth][1] = m.km.y; fold_k[depth][2] = m.km.z;
            o = p + n * rtm::kShadowEpsilon;                      // Reflect :368-373
            d = ((2.0f * n) * rtm::dot(view, n)) - view;
            ++depth;
            cnt.reflection++;
            continue;
        }
        term = col;
        break;
    }
    for (int k = depth - 1; k >= 0; --k) {
        term = mk(fold_c[k][0], fold_c[k][1], fold_c[k][2]) +
               mk(fold_k[k][0], fold_k[k][1], fold_k[k][2]) * term;
    }
    return term;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counts(const Counts &c, unsigned long long *ctr) {
    const unsigned p = wave_sum(c.primary), s = wave_sum(c.shadow), r = wave_sum(c.reflection);
    unsigned b = 0, t = 0, q = 0, h = 0;
    if (COUNT) {
        b = wave_sum(c.box);
        t = wave_sum(c.tri);
        q = wave_sum(c.sph);
        h = wave_sum(c.shading);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(ctr + 0, (unsigned long long)p);
        atomicAdd(ctr + 1, (unsigned long long)s);
        atomicAdd(ctr + 2, (unsigned long long)r);
        if (COUNT) {
            atomicAdd(ctr + 3, (unsigned long long)b);
            atomicAdd(ctr + 4, (unsigned long long)t);
            atomicAdd(ctr + 5, (unsigned long long)q);
            atomicAdd(ctr + 6, (unsigned long long)h);
        }
    }
}

template <bool COUNT>
__global__ __launch_bounds__(kBlockThreads) void render_kernel(SceneDev S, FrameDev F) {
    __shared__ int stack_mem[kWavesPerBlock * kStackSize * kWaveSize];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int *st = stack_mem + wave * kStackSize * kWaveSize + lane;
    const int tile = blockIdx.x * kWavesPerBlock + wave;
    if (tile >= F.num_tiles) return;  // wave-uniform

    const int spp = F.spp;
    const int pix = lane / spp;
    const int s = lane - pix * spp;
    const int tx = tile % F.tiles_x, ty = tile / F.tiles_x;
    const int px = tx * F.tile_w + pix % F.tile_w;
    const int ly = ty * F.tile_h + pix / F.tile_w;
    int gy = ly;
    if (F.band_count > 1) {
        const int blk = ly / F.band_rows;
        gy = (blk * F.band_count + F.band_index) * F.band_rows + (ly - blk * F.band_rows);
    }
    const bool active = pix < F.tile_w * F.tile_h && px < F.res_x && ly < F.local_rows && gy < F.res_y;

    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    f3 color = mk(0.0f, 0.0f, 0.0f);
    if (active) {
        // CastPixelRays :291-298 with n*n stratified offsets (n == 1: 0.5)
        const int n = F.spp_n;
        const int sj = s / n, si = s - sj * n;
        const float ox = ((float)si + 0.5f) / (float)n;
        const float oy = ((float)sj + 0.5f) / (float)n;
        const float rm = (((float)px + ox) * F.hl) / (float)F.res_x;
        const float dm = (((float)gy + oy) * F.vl) / (float)F.res_y;
        const f3 pp = (ld3(F.top_left) + rm * ld3(F.right)) - ld3(F.up) * dm;
        const f3 cam = ld3(F.cam_pos);
        const f3 dir = rtm::normalize(pp - cam);
        cnt.primary = 1;
        color = shade_path<COUNT>(S, F, cam, dir, st, cnt);
    }
    // Sum the pixel's samples in row-major sample order: ((s0 + s1) + s2) + ...
    f3 sum = color;
    for (int k = 1; k < spp; ++k) {
        const int src = lane + k;
        const float x = __shfl(color.x, src), y = __shfl(color.y, src), z = __shfl(color.z, src);
        sum = sum + mk(x, y, z);
    }
    if (active && s == 0) {
        f3 v = sum;
        if (spp > 1) v = v / (float)spp;
        // Rgb.Color, Rgb.cs:13
        F.out[(size_t)ly * F.res_x + px] = make_float4(v.x / 255.0f, v.y / 255.0f, v.z / 255.0f, 1.0f);
    }
    flush_counts<COUNT>(cnt, F.counters);
}

__global__ __launch_bounds__(kBlockThreads) void intersect_kernel(SceneDev S, const float *rays, int n,
                                                                  int4 *out) {
    __shared__ int stack_mem[kWavesPerBlock * kStackSize * kWaveSize];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int *st = stack_mem + wave * kStackSize * kWaveSize + lane;
    const int i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    const float *rr = rays + (size_t)i * 6;
    RayCtx r;
    setup_ray(r, mk(rr[0], rr[1], rr[2]), mk(rr[3], rr[4], rr[5]));
    float bt = FLT_MAX;
    int br = -1;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0};
    traverse<false, false>(S, r, 0.0f, 0.0f, bt, br, st, cnt);
    out[i] = make_int4(br, __float_as_int(bt), 0, 0);
}

__global__ void assemble_kernel(const float4 *gathered, int res_x, int res_y, int band_count,
                                int band_rows, int local_rows, float4 *image) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)res_x * res_y;
    if (i >= total) return;
    const int gy = (int)(i / res_x), x = (int)(i - (size_t)gy * res_x);
    const int blk = gy / band_rows;
    const int band = blk % band_count, slot = blk / band_count;
    const int ly = slot * band_rows + (gy - blk * band_rows);
    image[i] = gathered[((size_t)band * local_rows + ly) * res_x + x];
}

}  // namespace

namespace rtk {

hipError_t launch_render(const SceneDev &S, const FrameDev &F, bool count_tests, hipStream_t stream) {
    if (F.num_tiles <= 0) return hipSuccess;
    const int blocks = (F.num_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (count_tests)
        hipLaunchKernelGGL(render_kernel<true>, dim3(blocks), dim3(kBlockThreads), 0, stream, S, F);
    else
        hipLaunchKernelGGL(render_kernel<false>, dim3(blocks), dim3(kBlockThreads), 0, stream, S, F);
    return hipGetLastError();
}

hipError_t launch_intersect(const SceneDev &S, const float *rays, int n, int4 *out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int blocks = (n + kBlockThreads - 1) / kBlockThreads;
    hipLaunchKernelGGL(intersect_kernel, dim3(blocks), dim3(kBlockThreads), 0, stream, S, rays, n, out);
    return hipGetLastError();
}

hipError_t launch_assemble(const float4 *gathered, int res_x, int res_y, int band_count, int band_rows,
                           int local_rows, float4 *image, hipStream_t stream) {
    const size_t total = (size_t)res_x * res_y;
    if (total == 0) return hipSuccess;
    const int threads = 256;
    const unsigned blocks = (unsigned)((total + threads - 1) / threads);
    hipLaunchKernelGGL(assemble_kernel, dim3(blocks), dim3(threads), 0, stream, gathered, res_x, res_y,
                       band_count, band_rows, local_rows, image);
    return hipGetLastError();
}

}  // namespace rtk
