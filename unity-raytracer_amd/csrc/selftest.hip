// selftest.hip — device-math self-checks behind librt_selftest.so (test
// infrastructure; not part of the product ABI in include/rt_mi355.h).
// The kernels' shortcuts for IEEE operations must give bit-identical results:
//   rt_selftest_pow  rts::spec_pow_int(x, y) on host-given arguments (the test
//                    compares with the host's correctly rounded pow).
//   rt_selftest_deep_stack  rtt::traverse over a "comb" tree whose every
//                    pending sibling stays on the lane stack, so the stack
//                    reaches 3 x depth entries (the builders accept 3 x
//                    (depth + 1) <= kStackTotal) across the LDS / private
//                    overflow boundary of both render_kernel shapes (16 LDS
//                    entries at six waves, kStackShard at five).
#include <stdint.h>

#include <vector>

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_math.h"
#include "shade.h"
#include "traverse.h"

namespace {

__global__ void pow_eval(const float *x, const float *y, float *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rts::spec_pow_int(x[i], y[i]);
}

// One query per lane (all lanes the same ray) with the lane stack shaped as
// render_kernel's: SS entries in LDS, kStackTotal - SS in the private array.
template <int SS>
__global__ __launch_bounds__(64) void deep_stack_eval(rtd::SceneDev S, int *out) {
    __shared__ int lds[SS * rtd::kWaveSize];
    int ovf[rtd::kStackTotal - SS];
    const rtt::Stack st{lds, ovf, SS};
    rtt::RayCtx r;
    rtt::setup_ray(r, rtm::mk(0.0f, 0.0f, 0.0f), rtm::mk(0.0f, 0.0f, 1.0f));
    float bt;
    int br;
    rtt::Counts cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    (void)rtt::traverse<false, true>(S, r, 0.0f, 0.0f, bt, br, st, cnt);
    if (threadIdx.x == 0) {
        out[0] = br;
        out[1] = __float_as_int(bt);
        out[2] = (int)cnt.tri;
        out[3] = (int)cnt.box;
    }
}

}  // namespace

extern "C" {

// The comb: internal node i (< depth) has child 0 = node i + 1 and leaves in
// children 1..3 (the last node: four leaves); every child box holds the ray
// origin, so every child is entered and, with equal entry distances, the
// internal child is descended first and the three leaves wait on the stack:
// 3 x depth entries at the deepest node.  Leaf j holds one triangle across the
// ray (+z from the origin) at t = 2 + j / 64, except the leaf pushed first
// (node 0's child 3, the stack bottom), at t = 1: the closest hit, found last.
// out = {rank, t bits, triangle tests, box tests}; 0 ok, -1 HIP error,
// -2 bad arguments.
int rt_selftest_deep_stack(int depth, int lds_entries, int *out4) {
    if (depth < 1 || 3 * depth > rtd::kStackTotal || (lds_entries != 16 && lds_entries != 24)) return -2;
    std::vector<rtd::BvhNode4> nodes((size_t)depth);
    std::vector<rtd::TriRec> tris;
    const float B = 1000.0f;
    for (int i = 0; i < depth; ++i) {
        rtd::BvhNode4 &n = nodes[(size_t)i];
        n.lox = n.loy = n.loz = make_float4(-B, -B, -B, -B);
        n.hix = n.hiy = n.hiz = make_float4(B, B, B, B);
        int ch[4];
        for (int c = 0; c < 4; ++c) {
            if (c == 0 && i + 1 < depth) {
                ch[c] = i + 1;
                continue;
            }
            const int j = (int)tris.size();
            const float t = (i == 0 && c == 3) ? 1.0f : 2.0f + (float)j / 64.0f;
            rtd::TriRec tr;
            const int gate = -1;
            float rb, gb;
            __builtin_memcpy(&rb, &j, 4);
            __builtin_memcpy(&gb, &gate, 4);
            tr.p0 = make_float4(-1.0f, -1.0f, t, 4.0f);  // v0, e1 = (4, 0, 0)
            tr.p1 = make_float4(0.0f, 0.0f, 0.0f, 4.0f);  // e2 = (0, 4, 0)
            tr.p2 = make_float4(0.0f, rb, gb, 0.0f);
            tris.push_back(tr);
            ch[c] = rtd::encode_leaf(j, 1, rtd::kLeafTri);
        }
        n.child = make_int4(ch[0], ch[1], ch[2], ch[3]);
        n.pad = make_int4(0, 0, 0, 0);
    }
    tris.push_back(rtd::sentinel_tri());
    rtd::BvhNode4 *dn = nullptr;
    rtd::TriRec *dt = nullptr;
    int *dout = nullptr;
    bool ok = hipMalloc(&dn, nodes.size() * sizeof nodes[0]) == hipSuccess &&
              hipMalloc(&dt, tris.size() * sizeof tris[0]) == hipSuccess &&
              hipMalloc(&dout, 4 * sizeof(int)) == hipSuccess &&
              hipMemcpy(dn, nodes.data(), nodes.size() * sizeof nodes[0], hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dt, tris.data(), tris.size() * sizeof tris[0], hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        rtd::SceneDev S{};
        S.nodes4 = dn;
        S.tris = dt;
        S.has_prims = 1;
        S.bvh4 = 1;
        for (int a = 0; a < 3; ++a) {
            S.scene_lo[a] = -B;
            S.scene_hi[a] = B;
        }
        if (lds_entries == 24)
            hipLaunchKernelGGL(deep_stack_eval<24>, dim3(1), dim3(64), 0, 0, S, dout);
        else
            hipLaunchKernelGGL(deep_stack_eval<16>, dim3(1), dim3(64), 0, 0, S, dout);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(out4, dout, 4 * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (dn) (void)hipFree(dn);
    if (dt) (void)hipFree(dt);
    if (dout) (void)hipFree(dout);
    return ok ? 0 : -1;
}

// out[i] = spec_pow_int(x[i], y[i]) on the device (host arrays); 0 ok, -1 HIP error.
int rt_selftest_pow(const float *x, const float *y, float *out, int n) {
    if (n <= 0) return 0;
    float *d = nullptr;
    const size_t b = (size_t)n * sizeof(float);
    if (hipMalloc(&d, 3 * b) != hipSuccess) return -1;
    bool ok = hipMemcpy(d, x, b, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d + n, y, b, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(pow_eval, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, d + 2 * n, n);
        ok = hipDeviceSynchronize() == hipSuccess && hipMemcpy(out, d + 2 * n, b, hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    return ok ? 0 : -1;
}

}  // extern "C"
