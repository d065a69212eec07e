// scene_xform.hip — device mesh extraction (see scene_xform.h).
#include "scene_xform.h"

#include <float.h>

#include "rt_math.h"

namespace rtx {
namespace {

using rtm::f3;
using rtm::mk;

constexpr int kThreads = 256;

// last mesh whose first element is <= i (empty meshes share their
// successor's start, so the owner is always the last such mesh)
template <int FIELD>
__device__ __forceinline__ int owner(const MeshSrcDev *m, int count, int i) {
    int a = 0, b = count - 1;
    while (a < b) {
        const int c = (a + b + 1) >> 1;
        const int first = FIELD == 0 ? m[c].vertex_first : m[c].tri_first;
        if (first <= i) a = c; else b = c - 1;
    }
    return a;
}

// Matrix4x4.MultiplyPoint3x4 (UnityEngine; restated in scene.py
// multiply_point3x4): per row ((m0*x + m1*y) + m2*z) + m3, unfused.
__global__ void k_vertices(XformArgs a) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= a.vertex_total) return;
    const int m = owner<0>(a.meshes, a.mesh_count, v);
    const float *M = a.matrices + (size_t)m * 16;
    const float x = a.local[3 * (size_t)v], y = a.local[3 * (size_t)v + 1], z = a.local[3 * (size_t)v + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) a.world[3 * (size_t)v + r] = ((M[4 * r] * x + M[4 * r + 1] * y) + M[4 * r + 2] * z) + M[4 * r + 3];
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = rtm::umin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = rtm::umax(v, __shfl_xor(v, o));
    return v;
}

// Mesh.AABB: Min = float.MaxValue, Max = float.MinValue (= -FLT_MAX), then
// Encapsulate(point) = min(point, Min) / max(point, Max) for every vertex
// (AABB.cs:10-14).  A NaN coordinate never enters (Unity's min(x, y) keeps y
// unless y is NaN or x < y), so partial results are NaN-free and their
// combination order does not matter.  Two passes, so one big mesh does not
// fall to a single wave (C3's knot: 35k vertices, 158 us): one wave per part
// of kAabbPart vertices of a mesh, then one thread per mesh over its parts.
__global__ void k_aabb_parts(XformArgs a) {
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) / rtd::kWaveSize;
    const int lane = threadIdx.x % rtd::kWaveSize;
    if (w >= a.part_total) return;
    int lo_m = 0, hi_m = a.mesh_count - 1;  // last mesh with part_first <= w
    while (lo_m < hi_m) {
        const int c = (lo_m + hi_m + 1) >> 1;
        if (a.meshes[c].part_first <= w) lo_m = c; else hi_m = c - 1;
    }
    const MeshSrcDev M = a.meshes[lo_m];
    const int v0 = (w - M.part_first) * kAabbPart, v1 = min(M.vertex_count, v0 + kAabbPart);
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int v = v0 + lane; v < v1; v += rtd::kWaveSize) {
        const float *p = a.world + 3 * (size_t)(M.vertex_first + v);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lo[c] = rtm::umin(p[c], lo[c]);
            hi[c] = rtm::umax(p[c], hi[c]);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = wave_min(lo[c]);
        hi[c] = wave_max(hi[c]);
    }
    if (lane == 0) {
        a.parts[w].lo = make_float4(lo[0], lo[1], lo[2], 0.0f);
        a.parts[w].hi = make_float4(hi[0], hi[1], hi[2], 0.0f);
    }
}

__global__ void k_aabbs(XformArgs a) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= a.mesh_count) return;
    const int p0 = a.meshes[m].part_first, p1 = m + 1 < a.mesh_count ? a.meshes[m + 1].part_first : a.part_total;
    float4 lo = a.parts[p0].lo, hi = a.parts[p0].hi;
    for (int p = p0 + 1; p < p1; ++p) {
        const float4 l = a.parts[p].lo, h = a.parts[p].hi;
        lo = make_float4(rtm::umin(l.x, lo.x), rtm::umin(l.y, lo.y), rtm::umin(l.z, lo.z), 0.0f);
        hi = make_float4(rtm::umax(h.x, hi.x), rtm::umax(h.y, hi.y), rtm::umax(h.z, hi.z), 0.0f);
    }
    a.aabbs[m].lo = lo;
    a.aabbs[m].hi = hi;
}

// Triangles from the index buffer in order; mesh normal = -Triangle.Normal.
__global__ void k_triangles(XformArgs a) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.tri_total) return;
    const int *ix = a.indices + 3 * (size_t)t;
    const float *w0 = a.world + 3 * (size_t)ix[0], *w1 = a.world + 3 * (size_t)ix[1],
                *w2 = a.world + 3 * (size_t)ix[2];
    const f3 v0 = mk(w0[0], w0[1], w0[2]), v1 = mk(w1[0], w1[1], w1[2]), v2 = mk(w2[0], w2[1], w2[2]);
    float *o = a.tris + 9 * (size_t)t;
    o[0] = v0.x; o[1] = v0.y; o[2] = v0.z;
    o[3] = v1.x; o[4] = v1.y; o[5] = v1.z;
    o[6] = v2.x; o[7] = v2.y; o[8] = v2.z;
    const f3 v = rtm::cross(v2 - v0, v1 - v0);
    const float len = sqrtf(rtm::dot(v, v));
    float *n = a.normals + 3 * (size_t)t;
    n[0] = -(v.x / len);
    n[1] = -(v.y / len);
    n[2] = -(v.z / len);
}

// One block.  The host folds acc = umin(acc, lo_m) over the meshes in order
// (ties keep the later operand: the sign of a zero follows the last mesh that
// attains the minimum); on NaN-free operands — mesh AABBs are (k_aabb_parts)
// — that fold is associative, so contiguous chunks folded per thread and the
// chunk results then combined pairwise in order (left operand first) give
// the same bits.
constexpr int kBoxThreads = 256;
__device__ __forceinline__ void box_fold(float *a, const float *b) {  // a = a (earlier) folded with b (later)
    for (int c = 0; c < 3; ++c) {
        a[c] = rtm::umin(a[c], b[c]);
        a[3 + c] = rtm::umax(a[3 + c], b[3 + c]);
    }
}
__global__ __launch_bounds__(kBoxThreads) void k_scene_box(const rtd::MeshGate *aabbs, int mesh_count, float rlx,
                                                           float rly, float rlz, float rhx, float rhy, float rhz,
                                                           float *box, float *host_box) {
    __shared__ float part[kBoxThreads][6];
    const int t = threadIdx.x;
    const int per = (mesh_count + kBoxThreads - 1) / kBoxThreads;
    const int m0 = min(mesh_count, t * per), m1 = min(mesh_count, m0 + per);
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int m = m0; m < m1; ++m) {
        const float4 l = aabbs[m].lo, h = aabbs[m].hi;
        const float b[6] = {l.x, l.y, l.z, h.x, h.y, h.z};
        box_fold(v, b);
    }
    for (int c = 0; c < 6; ++c) part[t][c] = v[c];
    __syncthreads();
    for (int o = 1; o < kBoxThreads; o <<= 1) {  // ordered pairwise tree: t absorbs t + o
        if ((t & (2 * o - 1)) == 0) box_fold(part[t], part[t + o]);
        __syncthreads();
    }
    if (t != 0) return;
    for (int c = 0; c < 6; ++c) v[c] = part[0][c];
    const float rest[6] = {rlx, rly, rlz, rhx, rhy, rhz};
    box_fold(v, rest);
    float scale = 1.0f;  // pad_abs_of: 2^-13 of the largest finite coordinate magnitude, at least 1
    for (int c = 0; c < 6; ++c)
        if (__builtin_isfinite(v[c])) scale = scale < fabsf(v[c]) ? fabsf(v[c]) : scale;
    for (int c = 0; c < 6; ++c) {
        box[c] = v[c];
        host_box[c] = v[c];
    }
    box[6] = scale * 0x1p-13f;
    host_box[6] = scale * 0x1p-13f;
}

// ---- refit (RefitArgs) ----------------------------------------------------

typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void st_wt(float *p, float v) {  // write-through (sc1), see lbvh.hip
    __hip_atomic_store((gu32 *)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float *p) {
    return __uint_as_float(__hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// padded triangle box, the builders' rule (rt_abi.cpp add_tri_prim, lbvh.hip k_prims)
__device__ __forceinline__ void tri_box(const float *v, float pad_abs, float4 &lo, float4 &hi) {
    float l[3], h[3], ext = 0.0f;
    for (int c = 0; c < 3; ++c) {
        l[c] = fminf(v[c], fminf(v[3 + c], v[6 + c]));
        h[c] = fmaxf(v[c], fmaxf(v[3 + c], v[6 + c]));
        ext = fmaxf(ext, h[c] - l[c]);
    }
    const float pad = pad_abs + ext * 1e-4f;
    lo = make_float4(l[0] - pad, l[1] - pad, l[2] - pad, 0.0f);
    hi = make_float4(h[0] + pad, h[1] + pad, h[2] + pad, 0.0f);
}

__global__ void k_refit_prims(RefitArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float pad_abs = a.box[6];
    if (i < a.ntri) {
        rtd::TriRec t = a.tris[i];
        const int rank = __float_as_int(t.p2.y);
        const float *v;
        if (rank < a.mt) {
            int lo_m = 0, hi_m = a.mesh_count - 1;  // last mesh with rank_first <= rank
            while (lo_m < hi_m) {
                const int c = (lo_m + hi_m + 1) >> 1;
                if (a.mesh_rank_first[c] <= rank) lo_m = c; else hi_m = c - 1;
            }
            const int g = a.mesh_geom_first[lo_m] + (rank - a.mesh_rank_first[lo_m]);
            v = a.mesh_tris + 9 * (size_t)g;
            const f3 v0 = mk(v[0], v[1], v[2]), v1 = mk(v[3], v[4], v[5]), v2 = mk(v[6], v[7], v[8]);
            const f3 e1 = v1 - v0, e2 = v2 - v0;  // RMath.cs:34-35
            t.p0 = make_float4(v0.x, v0.y, v0.z, e1.x);
            t.p1 = make_float4(e1.y, e1.z, e2.x, e2.y);
            t.p2.x = e2.z;
            a.tris[i] = t;
            const float *n = a.mesh_normals + 3 * (size_t)g;
            a.shade[rank] = make_float4(n[0], n[1], n[2], a.shade[rank].w);
        } else {
            v = a.loose_tris + 9 * (size_t)(rank - a.mt - a.ns);
        }
        tri_box(v, pad_abs, a.prim_lo[i], a.prim_hi[i]);
    } else if (i < a.ntri + a.nsph) {
        const float4 cr = a.sphs[i - a.ntri].cr;
        const float r = sqrtf(cr.w), pad = pad_abs + r * 1e-4f;
        a.prim_lo[i] = make_float4(cr.x - r - pad, cr.y - r - pad, cr.z - r - pad, 0.0f);
        a.prim_hi[i] = make_float4(cr.x + r + pad, cr.y + r + pad, cr.z + r + pad, 0.0f);
    }
}

__device__ __forceinline__ float half_area3(float4 lo, float4 hi) {
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return dx * dy + dy * dz + dz * dx;
}

// The tree-quality sum (RefitArgs::quality) in fixed point: each internal
// slot's half area in units of 2^-24 of the scene box's, added as a 64-bit
// integer — an order-free, hence reproducible, sum (a float atomic sum in
// arrival order could flip the rebuild decision from run to run).  0 when
// the scene box is degenerate or not finite (the root then reports NaN).
__device__ __forceinline__ double quality_scale(const float *box) {
    const double dx = (double)box[3] - box[0], dy = (double)box[4] - box[1], dz = (double)box[5] - box[2];
    const double sa = dx * dy + dy * dz + dz * dx;
    return sa > 1e-30 && sa < 1e30 ? 0x1p24 / sa : 0.0;
}

__global__ void k_refit_nodes(RefitArgs a) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= a.nnodes || a.internal_children[v] != 0) return;
    const double qscale = quality_scale(a.box);
    unsigned long long *const qsum = reinterpret_cast<unsigned long long *>(a.quality + 2);
    for (;;) {
        rtd::BvhNode4 *nd = a.nodes + v;
        const int4 ch = nd->child;
        const int refs[4] = {ch.x, ch.y, ch.z, ch.w};
        float4 ulo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), uhi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        float inner_area = 0.0f;
        float *lox = &nd->lox.x, *hix = &nd->hix.x, *loy = &nd->loy.x, *hiy = &nd->hiy.x, *loz = &nd->loz.x,
              *hiz = &nd->hiz.x;
        for (int k = 0; k < 4; ++k) {
            const int ref = refs[k];
            if (ref == a.empty_ref) continue;
            float4 lo, hi;
            if (ref >= 0) {  // the child's thread wrote this slot
                lo = make_float4(ld_wt(lox + k), ld_wt(loy + k), ld_wt(loz + k), 0.0f);
                hi = make_float4(ld_wt(hix + k), ld_wt(hiy + k), ld_wt(hiz + k), 0.0f);
                inner_area += half_area3(lo, hi);
            } else {
                const int d = ~ref, first = d & ((1 << rtd::kLeafFirstBits) - 1);
                const int count = ((d >> rtd::kLeafFirstBits) & 3) + 1, kind = (d >> (rtd::kLeafFirstBits + 2)) & 1;
                const int base = kind == rtd::kLeafSphere ? a.ntri + first : first;
                lo = a.prim_lo[base];
                hi = a.prim_hi[base];
                for (int p = 1; p < count; ++p) {
                    const float4 l = a.prim_lo[base + p], h = a.prim_hi[base + p];
                    lo = make_float4(fminf(lo.x, l.x), fminf(lo.y, l.y), fminf(lo.z, l.z), 0.0f);
                    hi = make_float4(fmaxf(hi.x, h.x), fmaxf(hi.y, h.y), fmaxf(hi.z, h.z), 0.0f);
                }
                st_wt(lox + k, lo.x); st_wt(hix + k, hi.x);
                st_wt(loy + k, lo.y); st_wt(hiy + k, hi.y);
                st_wt(loz + k, lo.z); st_wt(hiz + k, hi.z);
            }
            ulo = make_float4(fminf(ulo.x, lo.x), fminf(ulo.y, lo.y), fminf(ulo.z, lo.z), 0.0f);
            uhi = make_float4(fmaxf(uhi.x, hi.x), fmaxf(uhi.y, hi.y), fmaxf(uhi.z, hi.z), 0.0f);
        }
        if (inner_area > 0.0f && qscale > 0.0)  // one term < 2^34, at most 2^27 nodes: no overflow
            atomicAdd(qsum, __double2ull_rn(fmin((double)inner_area * qscale, 0x1p34)));
        const int ps = a.parent_slot[v];
        if (ps < 0) {  // the root: every other node's term was added before its arrival count
            const unsigned long long sum = __hip_atomic_load(qsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.quality[0] = qscale > 0.0 ? (float)((double)sum / qscale) : __int_as_float(0x7fc00000);
            a.quality[1] = half_area3(ulo, uhi);
            return;
        }
        const int p = ps >> 2, k = ps & 3;
        rtd::BvhNode4 *pn = a.nodes + p;
        st_wt(&pn->lox.x + k, ulo.x); st_wt(&pn->hix.x + k, uhi.x);
        st_wt(&pn->loy.x + k, ulo.y); st_wt(&pn->hiy.x + k, uhi.y);
        st_wt(&pn->loz.x + k, ulo.z); st_wt(&pn->hiz.x + k, uhi.z);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot is visible before the count
        const int arrived = __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)&a.arrivals[p], 1,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (arrived != a.internal_children[p]) return;  // a sibling subtree is still refitting
        v = p;
    }
}

// the tree's links: each node's parent slot (4 * parent + slot; the root
// keeps the -1 of the memset) and its number of internal children
__global__ void k_refit_links(rtd::BvhNode4 *nodes, int nnodes, int *parent_slot, int *internal_children) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nnodes) return;
    const int4 ch = nodes[v].child;
    const int c[4] = {ch.x, ch.y, ch.z, ch.w};
    int n = 0;
    for (int k = 0; k < 4; ++k)
        if (c[k] >= 0) {
            parent_slot[c[k]] = 4 * v + k;
            ++n;
        }
    internal_children[v] = n;
}

}  // namespace

hipError_t refit_links(const RefitArgs &a, int *parent_slot, int *internal_children, hipStream_t stream) {
    if (a.nnodes <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(parent_slot, 0xff, sizeof(int) * (size_t)a.nnodes, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_refit_links, dim3((a.nnodes + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, a.nodes,
                       a.nnodes, parent_slot, internal_children);
    return hipGetLastError();
}

hipError_t refit_tree(const RefitArgs &a, hipStream_t stream) {
    if (a.nnodes <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.arrivals, 0, sizeof(int) * (size_t)a.nnodes, stream);
    if (e == hipSuccess) e = hipMemsetAsync(a.quality, 0, 4 * sizeof(float), stream);
    if (e != hipSuccess) return e;
    const int np = a.ntri + a.nsph;
    if (np > 0) hipLaunchKernelGGL(k_refit_prims, dim3((np + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, a);
    hipLaunchKernelGGL(k_refit_nodes, dim3((a.nnodes + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t scene_box(const rtd::MeshGate *aabbs, int mesh_count, const float rest_lo[3], const float rest_hi[3],
                     float *box, float *host_box, hipStream_t stream) {
    hipLaunchKernelGGL(k_scene_box, dim3(1), dim3(kBoxThreads), 0, stream, aabbs, mesh_count, rest_lo[0], rest_lo[1],
                       rest_lo[2], rest_hi[0], rest_hi[1], rest_hi[2], box, host_box);
    return hipGetLastError();
}

hipError_t transform_meshes(const XformArgs &a, hipStream_t stream) {
    if (a.mesh_count <= 0) return hipSuccess;
    if (a.vertex_total > 0)
        hipLaunchKernelGGL(k_vertices, dim3((a.vertex_total + kThreads - 1) / kThreads), dim3(kThreads), 0, stream,
                           a);
    const int waves_per_block = kThreads / rtd::kWaveSize;
    hipLaunchKernelGGL(k_aabb_parts, dim3((a.part_total + waves_per_block - 1) / waves_per_block), dim3(kThreads), 0,
                       stream, a);
    hipLaunchKernelGGL(k_aabbs, dim3((a.mesh_count + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, a);
    if (a.tri_total > 0)
        hipLaunchKernelGGL(k_triangles, dim3((a.tri_total + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace rtx
