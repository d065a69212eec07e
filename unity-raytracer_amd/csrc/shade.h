// shade.h — Whitted shading of one hit, RayTracingSetup.cs:304-455, split
// into the pieces the megakernel and the wavefront kernels share.  Every
// function recomputes from (ray, t, rank) with the same operations, so the
// wavefront "shade" and "finish" passes see bit-identical P, N, V, L.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_math.h"
#include "packet.h"
#include "traverse.h"

namespace rts {

using rtm::f3;
using rtm::mk;

struct Surface {
    f3 p;     // surfacePoint = Ray.GetPoint(t), Ray.cs:18-21
    f3 n;     // GetSurfaceNormalAndMaterial, :409-436
    f3 view;  // rayDirection = normalize(rayOrigin - surfacePoint), :325
    int mat;
};

__device__ __forceinline__ Surface surface(const rtd::SceneDev &S, f3 o, f3 d, float t, int rank) {
    Surface s;
    s.p = o + d * t;
    const float4 sh = S.shade[rank];
    s.mat = __float_as_int(sh.w);
    if (rank >= S.mesh_tri_total && rank < S.mesh_tri_total + S.sphere_count)
        s.n = rtm::normalize(s.p - mk(sh.x, sh.y, sh.z));  // GetSphereNormal :402-407
    else
        s.n = mk(sh.x, sh.y, sh.z);  // TriangleData.Normals (:422) / Mesh.TriangleNormals (:428)
    s.view = rtm::normalize(o - s.p);
    return s;
}

// CalculateAmbient :438-441
__device__ __forceinline__ f3 ambient(const rtd::SceneDev &S, const rtd::DevMaterial &m) {
    return rtt::ld3(S.ambient) * mk(m.ka_mirror.x, m.ka_mirror.y, m.ka_mirror.z);
}

struct ShadowRay {
    f3 o, dir;
    float d2;  // lightDistanceSq = distancesq(P, L) = lengthsq(L - P)
};

// :329-334
__device__ __forceinline__ ShadowRay shadow_ray(const Surface &s, const rtd::DevLight &L) {
    ShadowRay r;
    const f3 lmp = mk(L.pos.x, L.pos.y, L.pos.z) - s.p;
    r.dir = rtm::normalize(lmp);
    r.o = s.p + s.n * rtm::kShadowEpsilon;
    r.d2 = rtm::dot(lmp, lmp);
    return r;
}

// (float)Math.Pow((double)x, (double)y).  Out of line by default: inlined,
// the double-precision polynomial constants are hoisted to the kernel entry
// and spilled to scratch for the whole frame (64 B per lane written, then
// reloaded serially in every light loop).
__device__ __attribute__((noinline)) float spec_pow(float x, float y) { return (float)pow((double)x, (double)y); }

// (float)Math.Pow((double)x, (double)y) for the Phong exponents scenes use:
// for an integer y in [1, 128], x^y by binary powering in double (relative
// error below 2y * 2^-53; no under-/overflow can matter since 0 <= x <= 1 and
// the float result of anything below 2^-1000 is 0), rounded to float when
// that error bound cannot straddle a float rounding boundary (Ziv's test):
// then the result is the float nearest the exact power — which is what the
// host's correctly rounded pow, rounded to float, also is.  Otherwise, and
// for any other exponent, the out-of-line double pow.
__device__ __forceinline__ float spec_pow_int(float x, float y) {
    const int n = (int)y;
    if ((float)n == y && n >= 1 && n <= 128) {
        double b = (double)x, r = (n & 1) ? b : 1.0;
        for (int e = n >> 1; e; e >>= 1) {
            b = b * b;
            if (e & 1) r = r * b;
        }
        const double err = fabs(r) * ((double)(2 * n) * 0x1p-53);
        const float lo = (float)(r - err), hi = (float)(r + err);
        if (lo == hi && (r != 0.0 || err == 0.0)) return (float)r;
    }
    return spec_pow(x, y);
}

// diffuseRgb + specularRgb of one unoccluded light (:350-355).
__device__ __forceinline__ f3 light_term(const rtd::SceneDev &S, const Surface &s, const rtd::DevMaterial &m,
                                         const rtd::DevLight &L, const ShadowRay &sr) {
    const f3 e = mk(L.intensity.x, L.intensity.y, L.intensity.z) / sr.d2;  // receivedIrradiance :350
    const float ldn = rtm::dot(sr.dir, s.n);
    const f3 kd = mk(m.kd_phong.x, m.kd_phong.y, m.kd_phong.z);
    const f3 diffuse = (kd * rtm::umax(0.0f, ldn)) * e;  // CalculateDiffuse :443-455
    f3 spec = mk(0.0f, 0.0f, 0.0f);
    // CalculateSpecular :375-400: degrees(acos(ldn)) > 90f  <=>  ldn < threshold
    if (!(ldn < S.spec_threshold)) {
        const f3 v = sr.dir + s.view;
        const f3 h = v / rtm::length(v);
        const float cnh = rtm::umax(0.0f, rtm::dot(s.n, h));
        // pow(float, float) = (float)System.Math.Pow((double)x, (double)y); a
        // material whose specular term is always a signed zero skips it
        // (ks.w, rt_abi.cpp to_dev): (ks * 0) * E has the same bits.
        const float pw = m.ks.w != 0.0f ? 0.0f : spec_pow_int(cnh, m.kd_phong.w);
        spec = (mk(m.ks.x, m.ks.y, m.ks.z) * pw) * e;
    }
    return diffuse + spec;
}

// A light whose unoccluded term leaves the running colour's bits unchanged
// (a light behind the surface: diffuse and specular are +0) yields the same
// colour whether its shadow ray (:332-343) is blocked or not, so the ray's
// answer is moot and it need not be traced.  Bitwise, so exact for every
// input (signed zeros, NaN, overflow included).
__device__ __forceinline__ bool same_bits(f3 a, f3 b) {
    return __float_as_uint(a.x) == __float_as_uint(b.x) && __float_as_uint(a.y) == __float_as_uint(b.y) &&
           __float_as_uint(a.z) == __float_as_uint(b.z);
}

// Reflect :368-373 (direction not re-normalised)
__device__ __forceinline__ void reflect(const Surface &s, f3 &o, f3 &d) {
    o = s.p + s.n * rtm::kShadowEpsilon;
    d = ((2.0f * s.n) * rtm::dot(s.view, s.n)) - s.view;
}

// A frame shape fixed at compile time (FIX = n, the samples per pixel edge):
// 0 reads it from F (any n x n spp); 2: 2x2 spp in 4x4-pixel tiles (Q4, the
// bench configurations); 4: 4x4 spp in 2x2-pixel tiles and 8: 8x8 spp in
// one-pixel tiles (the levels kernel's 16 and 64 spp).  The lane -> sample
// and pixel splits are then shifts and masks, and (i + 0.5) / n is an exact
// scaling by a power of two (the same value as the division).  The tile
// sizes are prepare_frame's (rt_frame.cpp): 64 / spp pixels per wave as a
// near-square 2^a x 2^b block.
template <int FIX>
struct Fix {
    static_assert(FIX == 0 || FIX == 2 || FIX == 4 || FIX == 8, "fixed frame shapes");
    static constexpr int lg_n = FIX == 2 ? 1 : FIX == 4 ? 2 : FIX == 8 ? 3 : 0;
    static constexpr int tw = FIX == 2 ? 4 : FIX == 4 ? 2 : 1;  // tile edge in pixels
    static constexpr int lg_tw = FIX == 2 ? 2 : FIX == 4 ? 1 : 0;
};

// Primary ray of sample (px, gy, sub-sample s): CastPixelRays :291-298 with
// n*n stratified offsets ((i + 0.5) / n; n == 1 gives the reference's 0.5).
template <int FIX = 0>
__device__ __forceinline__ void primary_ray(const rtd::FrameDev &F, int px, int gy, int s, f3 &o, f3 &d) {
    using X = Fix<FIX>;
    const int n = FIX ? FIX : F.spp_n;
    const int sj = FIX ? s >> X::lg_n : s / n, si = FIX ? s & (FIX - 1) : s - sj * n;
    const float ox = FIX ? ((float)si + 0.5f) * (1.0f / (float)FIX) : ((float)si + 0.5f) / (float)n;
    const float oy = FIX ? ((float)sj + 0.5f) * (1.0f / (float)FIX) : ((float)sj + 0.5f) / (float)n;
    const float rm = (((float)px + ox) * F.hl) / (float)F.res_x;
    const float dm = (((float)gy + oy) * F.vl) / (float)F.res_y;
    const f3 pp = (rtt::ld3(F.top_left) + rm * rtt::ld3(F.right)) - rtt::ld3(F.up) * dm;
    o = rtt::ld3(F.cam_pos);
    d = rtm::normalize(pp - o);
}

// The conservative sky test of one sample (FrameDev sky_*, rt_abi.cpp
// sky_setup): false only when the sample's ray, approximated with fast
// reciprocals (relative error ~1e-6, far inside the pad), surely misses the
// padded Scene.AABB — then the exact ray misses the exact gate (Scene.cs:54).
// A NaN anywhere leaves the answer "maybe" (fminf/fmaxf ignore NaN operands).
template <int FIX = 0>
__device__ __forceinline__ bool sky_maybe(const rtd::FrameDev &F, int px, int gy, int s) {
    using X = Fix<FIX>;
    const int n = FIX ? FIX : F.spp_n;
    const int sj = FIX ? s >> X::lg_n : s / n, si = FIX ? s & (FIX - 1) : s - sj * n;
    const float rn = FIX ? 1.0f / (float)FIX : __builtin_amdgcn_rcpf((float)n);
    const float ax = ((float)px + ((float)si + 0.5f) * rn) * F.sky_hx;
    const float ay = ((float)gy + ((float)sj + 0.5f) * rn) * F.sky_vy;
    const float dx = F.sky_tlc[0] + ax * F.right[0] - ay * F.up[0];
    const float dy = F.sky_tlc[1] + ax * F.right[1] - ay * F.up[1];
    const float dz = F.sky_tlc[2] + ax * F.right[2] - ay * F.up[2];
    const float ix = __builtin_amdgcn_rcpf(dx), iy = __builtin_amdgcn_rcpf(dy), iz = __builtin_amdgcn_rcpf(dz);
    const float lx = F.sky_lo[0] * ix, hx = F.sky_hi[0] * ix;
    const float ly = F.sky_lo[1] * iy, hy = F.sky_hi[1] * iy;
    const float lz = F.sky_lo[2] * iz, hz = F.sky_hi[2] * iz;
    const float tmin = fmaxf(fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fminf(lz, hz)), 0.0f);
    const float tmax = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fmaxf(lz, hz));
    return !(tmin > tmax);
}

// Sum of a pixel's samples in row-major sample order ((s0 + s1) + s2) + ...,
// valid at the pixel's sample-0 lane (samples sit in consecutive lanes).  4
// spp: DPP quad moves (no LDS round trip); otherwise lane shuffles.  Must be
// called with every lane of the wave active.
__device__ __forceinline__ rtm::f3 sample_sum(rtm::f3 c, int lane, int spp) {
    rtm::f3 sum = c;
    if (spp == 4) {
        // quad_perm [k,k,k,k]: every lane of a quad reads the quad's lane k
#define RT_QREAD(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (ctrl), 0xf, 0xf, false))
        sum = sum + rtm::mk(RT_QREAD(c.x, 0x55), RT_QREAD(c.y, 0x55), RT_QREAD(c.z, 0x55));
        sum = sum + rtm::mk(RT_QREAD(c.x, 0xAA), RT_QREAD(c.y, 0xAA), RT_QREAD(c.z, 0xAA));
        sum = sum + rtm::mk(RT_QREAD(c.x, 0xFF), RT_QREAD(c.y, 0xFF), RT_QREAD(c.z, 0xFF));
#undef RT_QREAD
        return sum;
    }
    for (int k = 1; k < spp; ++k) {
        const int src = lane + k;
        sum = sum + rtm::mk(__shfl(c.x, src), __shfl(c.y, src), __shfl(c.z, src));
    }
    return sum;
}

// Color -> Color32 (UnityEngine, restated): (byte)Mathf.Round(Mathf.Clamp01(c)
// * 255f); Mathf.Round rounds half to even (System.Math.Round).  A NaN
// channel encodes as 0.
__device__ __forceinline__ unsigned encode8(float c) {
    if (!(c == c)) return 0u;
    c = c < 0.0f ? 0.0f : (c > 1.0f ? 1.0f : c);
    return (unsigned)rintf(c * 255.0f);
}

__device__ __forceinline__ unsigned half_bits(float c) {
    return (unsigned)__builtin_bit_cast(unsigned short, (_Float16)c);  // round to nearest even
}

// Final pixel store: v is the sample mean in Rgb.Value units (0..255);
// Rgb.Color = Value / 255 (Rgb.cs:13), then the requested output format.
__device__ __forceinline__ void store_pixel(const rtd::FrameDev &F, size_t idx, rtm::f3 v) {
    const float r = v.x / 255.0f, g = v.y / 255.0f, b = v.z / 255.0f;
    if (F.out_format == rtd::kOutRGBA8) {
        ((unsigned *)F.out)[idx] = encode8(r) | (encode8(g) << 8) | (encode8(b) << 16) | (255u << 24);
    } else if (F.out_format == rtd::kOutRGB32F) {
        float *q = (float *)F.out + idx * 3;
        q[0] = r;
        q[1] = g;
        q[2] = b;
    } else if (F.out_format == rtd::kOutRGBA16F) {
        ((uint2 *)F.out)[idx] = make_uint2(half_bits(r) | (half_bits(g) << 16), half_bits(b) | (0x3C00u << 16));
    } else {
        ((float4 *)F.out)[idx] = make_float4(r, g, b, 1.0f);
    }
}

// tile -> (tx, ty) = (tile % tiles_x, tile / tiles_x) by the per-frame magic
// multiplier (FrameDev::tiles_x_magic = floor(2^32 / tiles_x)): the estimate
// is the quotient or one less, fixed by one compare — a few scalar
// instructions instead of an integer-division sequence on the tile's critical
// path.  Exact for every non-negative 32-bit tile.
__device__ __forceinline__ void tile_xy(const rtd::FrameDev &F, int tile, int &tx, int &ty) {
    unsigned q = __umulhi((unsigned)tile, F.tiles_x_magic);
    int r = tile - (int)q * F.tiles_x;
    if (r >= F.tiles_x) {
        ++q;
        r -= F.tiles_x;
    }
    tx = r;
    ty = (int)q;
}

// Local row -> (band block, row in the block), ly = blk * band_rows + r, by
// the per-frame magic multiplier (FrameDev::band_rows_magic = floor(2^32 /
// band_rows)) like tile_xy: exact for every non-negative row, without the
// integer-division sequence that cost each shard lane two of them per tile.
__device__ __forceinline__ void band_block(const rtd::FrameDev &F, int ly, int &blk, int &r) {
    unsigned q = __umulhi((unsigned)ly, F.band_rows_magic);
    int rr = ly - (int)q * F.band_rows;
    if (rr >= F.band_rows) {
        ++q;
        rr -= F.band_rows;
    }
    blk = (int)q;
    r = rr;
}

// The pixel rectangle of a tile (image rows; tile index wave-uniform) for the
// camera packet's frustum start (packet.h cut_start).  Valid when a tile's
// rows lie in one band block (rt_abi.cpp cut_setup checks band_rows).
template <int FIX = 0>
__device__ __forceinline__ rtp::TileRect tile_rect(const rtd::FrameDev &F, int tile) {
    const int tw = FIX ? Fix<FIX>::tw : F.tile_w, th = FIX ? Fix<FIX>::tw : F.tile_h;
    int tx, ty;
    tile_xy(F, tile, tx, ty);
    const int ly = ty * th;
    int gy = ly + F.row0;
    if (F.band_count > 1) {
        int blk, r;  // ly = blk * band_rows + r, by the magic multiplier (no division)
        band_block(F, ly, blk, r);
        gy = (blk * F.band_count + F.band_index) * F.band_rows + r;
    }
    return rtp::TileRect{tx * tw, gy, tw, th};
}

// Slot (tile, lane) -> pixel; false for lanes outside the image/shard.  A
// pixel's samples sit in consecutive lanes.
template <int FIX = 0>
__device__ __forceinline__ bool slot_pixel(const rtd::FrameDev &F, int tile, int lane, int &px, int &ly, int &gy,
                                           int &s) {
    using X = Fix<FIX>;
    const int spp = FIX ? FIX * FIX : F.spp;
    const int lp = FIX ? lane >> (2 * X::lg_n) : lane / spp;
    const int pix = lp;
    s = FIX ? lane & (FIX * FIX - 1) : lane - lp * spp;
    const int tw = FIX ? X::tw : F.tile_w, th = FIX ? X::tw : F.tile_h;
    int tx, ty;
    tile_xy(F, tile, tx, ty);
    px = tx * tw + (FIX ? pix & (X::tw - 1) : pix % tw);
    ly = ty * th + (FIX ? pix >> X::lg_tw : pix / tw);
    gy = ly + F.row0;
    if (F.band_count > 1) {
        int blk, r;  // ly = blk * band_rows + r, by the magic multiplier (no division)
        band_block(F, ly, blk, r);
        gy = (blk * F.band_count + F.band_index) * F.band_rows + r;
    }
    return lp < rtd::kWaveSize / spp && pix < tw * th && px < F.res_x && ly < F.local_rows && gy < F.res_y;
}

}  // namespace rts
