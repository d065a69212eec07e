// Steady-state D2H copy rate into a caller buffer registered ONCE
// (hipHostRegister with various flags) vs hipHostMalloc'd and pageable
// memory: 33 MB (1080p float RGBA) in 1 and 8 async chunks.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static void bench(const char *name, void *h, void *d, size_t bytes, hipStream_t s) {
    for (int chunks : {1, 8}) {
        double best = 1e9, sum = 0;
        for (int rep = 0; rep < 8; ++rep) {
            double t0 = now();
            for (int k = 0; k < chunks; ++k)
                hipMemcpyAsync((char *)h + bytes / chunks * k, (char *)d + bytes / chunks * k, bytes / chunks,
                               hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
            double t = now() - t0;
            if (rep >= 2) { best = t < best ? t : best; sum += t; }
        }
        printf("%-22s chunks %d: best %.3f avg %.3f ms\n", name, chunks, best, sum / 6);
    }
}
int main() {
    const size_t bytes = 33177600;
    void *d; hipMalloc(&d, bytes); hipMemset(d, 1, bytes);
    hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<unsigned char> pg(bytes, 0);
    bench("pageable", pg.data(), d, bytes, s);
    void *pm; hipHostMalloc(&pm, bytes, hipHostMallocDefault); std::memset(pm, 0, bytes);
    bench("hipHostMalloc", pm, d, bytes, s);
    struct { const char *n; unsigned f; } fl[] = {{"register default", hipHostRegisterDefault},
                                                  {"register mapped", hipHostRegisterMapped},
                                                  {"register portable", hipHostRegisterPortable}};
    for (auto &f : fl) {
        std::vector<unsigned char> h(bytes, 0);
        double t0 = now();
        hipError_t e = hipHostRegister(h.data(), bytes, f.f);
        printf("%s: register %.3f ms (%s)\n", f.n, now() - t0, hipGetErrorString(e));
        bench(f.n, h.data(), d, bytes, s);
        t0 = now();
        hipHostUnregister(h.data());
        printf("%s: unregister %.3f ms\n", f.n, now() - t0);
    }
    // pageable again after registrations
    bench("pageable again", pg.data(), d, bytes, s);
    return 0;
}
