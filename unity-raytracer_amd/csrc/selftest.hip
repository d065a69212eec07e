// selftest.hip — device-math self-checks behind librt_selftest.so (test
// infrastructure; not part of the product ABI in include/rt_mi355.h).
// The kernels' shortcuts for IEEE operations must give bit-identical results:
//   rt_selftest_pow  rts::spec_pow_int(x, y) on host-given arguments (the test
//                    compares with the host's correctly rounded pow).
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "rt_math.h"
#include "shade.h"

namespace {

__global__ void pow_eval(const float *x, const float *y, float *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rts::spec_pow_int(x[i], y[i]);
}

}  // namespace

extern "C" {

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
