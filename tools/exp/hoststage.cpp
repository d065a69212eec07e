// D2H into a pinned staging buffer (hipHostMalloc) + threaded memcpy into a
// pageable frame, against the staged pageable copy: 33 MB and 8 MB frames.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    for (size_t bytes : {(size_t)33177600, (size_t)8294400}) {
        void *d; (void)hipMalloc(&d, bytes); (void)hipMemset(d, 1, bytes);
        void *pin; (void)hipHostMalloc(&pin, bytes, hipHostMallocDefault);
        for (int thp = 0; thp < 2; ++thp) {
            unsigned char *h = (unsigned char *)aligned_alloc(2 << 20, (bytes + (2 << 20) - 1) & ~(size_t)((2 << 20) - 1));
            if (thp) madvise(h, bytes, MADV_HUGEPAGE);
            std::memset(h, 0, bytes);
            hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            for (int rep = 0; rep < 4; ++rep) {
                double t0 = now();
                (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s); (void)hipStreamSynchronize(s);
                double t1 = now();
                (void)hipMemcpyAsync(pin, d, bytes, hipMemcpyDeviceToHost, s); (void)hipStreamSynchronize(s);
                double t2 = now();
                double tm[4];
                int ti = 0;
                for (int nt : {1, 4, 8, 16}) {
                    double a = now();
                    std::vector<std::thread> th;
                    for (int i = 0; i < nt; ++i)
                        th.emplace_back([=] { size_t c = bytes / nt; std::memcpy(h + c * i, (char *)pin + c * i, i == nt - 1 ? bytes - c * i : c); });
                    for (auto &x : th) x.join();
                    tm[ti++] = now() - a;
                }
                printf("%zu MB thp %d: pageable copy %.3f ms | pinned D2H %.3f ms, memcpy 1/4/8/16 thr %.3f %.3f %.3f %.3f ms\n",
                       bytes >> 20, thp, t1 - t0, t2 - t1, tm[0], tm[1], tm[2], tm[3]);
            }
            free(h);
        }
        (void)hipHostFree(pin);
        (void)hipFree(d);
    }
    return 0;
}
