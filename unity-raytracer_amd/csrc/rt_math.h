// rt_math.h — float32 arithmetic with the reference's exact operation order.
//
// Unity.Mathematics 1.2.6 semantics (the reference's L0, not vendored;
// restated from its public source — DESIGN.md "Arithmetic contract"):
//   dot(x,y)      = x.x*y.x + x.y*y.y + x.z*y.z          (left to right)
//   cross(x,y)    = (x * y.yzx - x.yzx * y).yzx
//   normalize(x)  = rsqrt(dot(x,x)) * x,  rsqrt(v) = 1.0f / sqrt(v)
//   length(x)     = sqrt(dot(x,x))
//   min(x,y)      = isnan(y) || x < y ? x : y ;  max likewise with '>'
//   rcp(x)        = 1.0f / x
// Every file including this header is compiled with -ffp-contract=off and
// -fhip-fp32-correctly-rounded-divide-sqrt, so each + - * / sqrt below is a
// single IEEE-754 binary32 rounding on both the host and gfx950.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#define RT_HD __host__ __device__ __forceinline__

namespace rtm {

struct f3 {
    float x, y, z;
};

RT_HD f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RT_HD f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
RT_HD f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
RT_HD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }

// min/max inside the slab test.  Unity's min/max ignore a NaN operand, as
// fminf/fmaxf do; the two can differ only in which zero they return for
// (-0, +0), and a slab test's outcome (tmin <= tmax) cannot tell the zeros
// apart — so on the device the single-instruction v_min/v_max_f32 are used.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float slab_min(float x, float y) { return fminf(x, y); }
__device__ __forceinline__ float slab_max(float x, float y) { return fmaxf(x, y); }
#else
RT_HD float slab_min(float x, float y) { return (__builtin_isnan(y) || x < y) ? x : y; }
RT_HD float slab_max(float x, float y) { return (__builtin_isnan(y) || x > y) ? x : y; }
#endif

// Correctly rounded 1.0f / b: the IEEE division (the kernels are compiled
// with -fhip-fp32-correctly-rounded-divide-sqrt).
RT_HD float rcp_cr(float b) { return 1.0f / b; }

RT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD f3 cross(f3 x, f3 y) {
    return mk(x.y * y.z - x.z * y.y, x.z * y.x - x.x * y.z, x.x * y.y - x.y * y.x);
}
RT_HD float lengthsq(f3 a) { return dot(a, a); }
RT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
RT_HD f3 normalize(f3 a) {
    float r = rcp_cr(sqrtf(dot(a, a)));
    return r * a;
}
RT_HD float umin(float x, float y) { return (__builtin_isnan(y) || x < y) ? x : y; }
RT_HD float umax(float x, float y) { return (__builtin_isnan(y) || x > y) ? x : y; }



// RMath.Epsilon (RMath.cs:9) and RayTracingSetup.ShadowRayEpsilon (:42)
constexpr float kEpsilon = 0.00001f;
constexpr float kShadowEpsilon = 0.0001f;

// RMath.RayAABBIntersection (RMath.cs:12-26), exact form: inv = rcp(dir) is
// passed in (1.0f/dir per component, computed once per ray — the same value
// the reference recomputes on every call).
RT_HD bool ref_slab(f3 o, f3 inv, f3 lo, f3 hi) {
    float tmin = 0.0f, tmax = INFINITY;
    float t1, t2;
    t1 = (lo.x - o.x) * inv.x; t2 = (hi.x - o.x) * inv.x;
    tmin = slab_min(slab_max(t1, tmin), slab_max(t2, tmin));
    tmax = slab_max(slab_min(t1, tmax), slab_min(t2, tmax));
    t1 = (lo.y - o.y) * inv.y; t2 = (hi.y - o.y) * inv.y;
    tmin = slab_min(slab_max(t1, tmin), slab_max(t2, tmin));
    tmax = slab_max(slab_min(t1, tmax), slab_min(t2, tmax));
    t1 = (lo.z - o.z) * inv.z; t2 = (hi.z - o.z) * inv.z;
    tmin = slab_min(slab_max(t1, tmin), slab_max(t2, tmin));
    tmax = slab_max(slab_min(t1, tmax), slab_min(t2, tmax));
    return tmin <= tmax;
}

// RMath.RayTriangleIntersection (RMath.cs:29-73), with edge1 = v1 - v0 and
// edge2 = v2 - v0 precomputed on the host (the same two float subtractions).
RT_HD bool ref_triangle(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float &t_out) {
    f3 h = cross(d, e2);
    float a = dot(e1, h);
    if (a > -kEpsilon && a < kEpsilon) return false;
    f3 s = o - v0;
    const float sh = dot(s, h);
    float f = rcp_cr(a);
    float u = f * sh;
    if (u < 0.0f || u > 1.0f) return false;
    f3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot(e2, q);
    if (t > kEpsilon) { t_out = t; return true; }
    return false;
}

// RMath.RaySphereIntersection (RMath.cs:81-108)
RT_HD bool ref_sphere(f3 o, f3 d, f3 c, float r2, float &t_out) {
    f3 oc = o - c;
    float uoc = dot(d, oc);
    float disc = uoc * uoc - (lengthsq(oc) - r2);
    if (disc < 0) return false;
    float sq = sqrtf(disc);
    float big = -uoc + sq;
    if (big < 0) return false;
    float small = -uoc - sq;
    t_out = small < 0 ? big : small;
    return true;
}

}  // namespace rtm
