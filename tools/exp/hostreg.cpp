// Cost of pinning a pageable host frame per call (hipHostRegister) vs the
// staged pageable copy: 33 MB (1080p float RGBA) and 8 MB (RGBA8).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    for (size_t bytes : {(size_t)33177600, (size_t)8294400}) {
        void *d; hipMalloc(&d, bytes); hipMemset(d, 1, bytes);
        std::vector<unsigned char> h(bytes);
        std::memset(h.data(), 0, bytes);
        hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        for (int rep = 0; rep < 5; ++rep) {
            double t0 = now();
            hipMemcpyAsync(h.data(), d, bytes, hipMemcpyDeviceToHost, s); hipStreamSynchronize(s);
            double t1 = now();
            hipHostRegister(h.data(), bytes, hipHostRegisterDefault);
            double t2 = now();
            for (int k = 0; k < 6; ++k)
                hipMemcpyAsync(h.data() + bytes / 6 * k, (char *)d + bytes / 6 * k, bytes / 6, hipMemcpyDeviceToHost, s);
            double t3 = now();
            hipStreamSynchronize(s);
            double t4 = now();
            hipHostUnregister(h.data());
            double t5 = now();
            printf("%zu MB pageable copy %.3f ms | register %.3f, 6 async copies issue %.3f, complete %.3f, unregister %.3f ms\n",
                   bytes >> 20, t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4);
        }
        hipFree(d);
    }
    return 0;
}
