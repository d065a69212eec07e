// rt_util.cpp — error reporting, roctx ranges and grow-only device buffers
// shared by the host modules (rt_host.h).
#include "rt_host.h"

namespace rti {

thread_local std::string g_create_error;

int fail(rt_ctx *ctx, int status, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx)
        ctx->err = buf;
    else
        g_create_error = buf;
    return status;
}

const Roctx &roctx() {
    static const Roctx r = [] {
        Roctx x;
        void *h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            x.push = (decltype(x.push))dlsym(h, "roctxRangePushA");
            x.pop = (decltype(x.pop))dlsym(h, "roctxRangePop");
            if (!x.push || !x.pop) x.push = nullptr, x.pop = nullptr;
        }
        return x;
    }();
    return r;
}

// Grow-only device buffer (per-frame rebuilds reuse their memory).
hipError_t ensure(rt_ctx *ctx, GrowBuf &b, size_t bytes) {
    (void)ctx;
    if (bytes <= b.cap) return hipSuccess;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        if (e != hipSuccess) return e;
    }
    b.p = nullptr;
    b.cap = 0;
    hipError_t e = hipMalloc(&b.p, bytes < 256 ? 256 : bytes);
    if (e == hipSuccess) b.cap = bytes < 256 ? 256 : bytes;
    return e;
}

hipError_t ensure_out(rt_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->d_out_cap) return hipSuccess;
    if (ctx->d_out) {
        hipError_t e = hipFree(ctx->d_out);
        if (e != hipSuccess) return e;
    }
    ctx->d_out = nullptr;
    ctx->d_out_cap = 0;
    hipError_t e = hipMalloc(&ctx->d_out, bytes);
    if (e == hipSuccess) ctx->d_out_cap = bytes;
    return e;
}

int32_t band_local_rows(int32_t res_y, int32_t band_count, int32_t band_rows) {
    if (res_y <= 0) return 0;
    if (band_count <= 1) return res_y;
    const int32_t blocks = (res_y + band_rows - 1) / band_rows;
    const int32_t slots = (blocks + band_count - 1) / band_count;
    return slots * band_rows;
}

}  // namespace rti
