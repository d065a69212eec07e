// selftest.hip — device-math self-checks behind librt_selftest.so (test
// infrastructure; not part of the product ABI in include/rt_mi355.h).
// The kernels' shortcuts for IEEE operations must give bit-identical results:
//   rt_selftest_rcp  rtm::rcp_cr(b) vs IEEE 1.0f / b over a range of float bit
//                    patterns (both signs), counted on the device;
//   rt_selftest_pow  rts::spec_pow_int(x, y) on host-given arguments (the test
//                    compares with the host's correctly rounded pow).
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "rt_math.h"
#include "shade.h"

namespace {

__global__ void rcp_check(uint32_t lo, uint32_t hi, unsigned long long *bad, uint32_t *first) {
    const uint64_t span = (uint64_t)hi - lo;
    unsigned long long local = 0;
    uint32_t fb = 0xffffffffu;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t bits = lo + (uint32_t)i;
#pragma unroll
        for (int sgn = 0; sgn < 2; ++sgn) {
            const float b = __uint_as_float(bits | (sgn ? 0x80000000u : 0u));
            const float want = 1.0f / b;  // IEEE division (-fhip-fp32-correctly-rounded-divide-sqrt)
            const float got = rtm::rcp_cr(b);
            if (__float_as_uint(want) != __float_as_uint(got)) {
                ++local;
                fb = min(fb, bits);
            }
        }
    }
    if (local) {
        atomicAdd(bad, local);
        atomicMin(first, fb);
    }
}

__global__ void pow_eval(const float *x, const float *y, float *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rts::spec_pow_int(x[i], y[i]);
}

}  // namespace

extern "C" {

// Mismatch count of rcp_cr over bit patterns [lo, hi) of both signs; -1 on a HIP error.
long long rt_selftest_rcp(uint32_t lo, uint32_t hi, uint32_t *first_bad) {
    unsigned long long *d_bad = nullptr;
    uint32_t *d_first = nullptr;
    if (hipMalloc(&d_bad, sizeof *d_bad) != hipSuccess || hipMalloc(&d_first, sizeof *d_first) != hipSuccess)
        return -1;
    const uint32_t init = 0xffffffffu;
    (void)hipMemset(d_bad, 0, sizeof *d_bad);
    (void)hipMemcpy(d_first, &init, sizeof init, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(rcp_check, dim3(8192), dim3(256), 0, 0, lo, hi, d_bad, d_first);
    unsigned long long bad = 0;
    uint32_t fb = init;
    const bool ok = hipDeviceSynchronize() == hipSuccess &&
                    hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(&fb, d_first, sizeof fb, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    if (first_bad) *first_bad = fb;
    return ok ? (long long)bad : -1;
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
