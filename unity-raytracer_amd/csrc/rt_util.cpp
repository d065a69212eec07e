// rt_util.cpp — error reporting, roctx ranges and grow-only device buffers
// shared by the host modules (rt_host.h).
#include "rt_host.h"

#include <atomic>
#include <unordered_set>

#include <sys/syscall.h>
#include <unistd.h>

namespace rti {

// ---- host waits (rt_debug_read RT_DEBUG_HOST_WAITS)
// One slot per live host thread that has entered a blocking call of the
// library; a thread keeps its slot until it exits.  Plain atomics: the
// report may run on another thread while the owner is blocked.
namespace {
constexpr int kWaitSlots = 256;
struct WaitSlot {
    std::atomic<long> tid{0};  // 0: free
    std::atomic<const char *> what{nullptr};
    std::atomic<int> device{-1};
    std::atomic<long long> since_ns{0};
};
WaitSlot g_waits[kWaitSlots];

long long now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct SlotOwner {
    int slot = -1;
    ~SlotOwner() {
        if (slot >= 0) {
            g_waits[slot].what.store(nullptr);
            g_waits[slot].tid.store(0);
        }
    }
    int get() {
        if (slot != -1) return slot;
        slot = -2;  // table full: this thread is not tracked
        const long tid = (long)syscall(SYS_gettid);
        for (int i = 0; i < kWaitSlots; ++i) {
            long free = 0;
            if (g_waits[i].tid.compare_exchange_strong(free, tid)) {
                slot = i;
                break;
            }
        }
        return slot;
    }
};
thread_local SlotOwner t_wait_slot;
}  // namespace

Wait::Wait(const char *what) : slot_(t_wait_slot.get()), prev_what_(nullptr), prev_since_(0) {
    if (slot_ < 0) return;
    WaitSlot &w = g_waits[slot_];
    prev_what_ = w.what.load(std::memory_order_relaxed);
    prev_since_ = w.since_ns.load(std::memory_order_relaxed);
    int dev = -1;
    (void)hipGetDevice(&dev);
    w.device.store(dev, std::memory_order_relaxed);
    w.since_ns.store(now_ns(), std::memory_order_relaxed);
    w.what.store(what, std::memory_order_release);
}

Wait::~Wait() {
    if (slot_ < 0) return;
    WaitSlot &w = g_waits[slot_];
    w.since_ns.store(prev_since_, std::memory_order_relaxed);
    w.what.store(prev_what_, std::memory_order_release);
}

namespace {
void stream_line(std::string &o, const char *who, int member, int dev, hipStream_t s) {
    if (!s) return;
    (void)hipSetDevice(dev);
    const hipError_t e = hipStreamQuery(s);
    char b[160];
    snprintf(b, sizeof b, "  member %d device %d %s stream %p: %s\n", member, dev, who, (void *)s,
             e == hipSuccess ? "idle" : e == hipErrorNotReady ? "work pending" : hipGetErrorString(e));
    o += b;
}
}  // namespace

// ---- live contexts: the report reads a context only while it is registered,
// under the registry's lock, and rt_destroy unregisters it (taking the same
// lock) before any teardown — so a report from another thread never reads a
// context being destroyed or freed (it only compares the pointer value).
namespace {
std::mutex g_live_mu;
std::unordered_set<const rt_ctx *> g_live;
}  // namespace

void register_ctx(const rt_ctx *ctx) {
    if (!ctx) return;
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.insert(ctx);
}

void unregister_ctx(const rt_ctx *ctx) {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.erase(ctx);
}

std::string host_waits_report(rt_ctx *ctx) {
    std::string o = "host threads inside blocking library calls:\n";
    const long long t = now_ns();
    int n = 0;
    for (int i = 0; i < kWaitSlots; ++i) {
        const long tid = g_waits[i].tid.load();
        const char *what = g_waits[i].what.load(std::memory_order_acquire);
        if (!tid || !what) continue;
        char b[320];
        snprintf(b, sizeof b, "  thread %ld device %d: %s for %.1f ms\n", tid, g_waits[i].device.load(), what,
                 (double)(t - g_waits[i].since_ns.load()) * 1e-6);
        o += b;
        ++n;
    }
    if (!n) o += "  (none)\n";
    if (!ctx) return o;
    std::lock_guard<std::mutex> live(g_live_mu);  // held while the context is read
    if (!g_live.count(ctx) || ctx->destroying.load())
        return o + "context: not live (destroyed or being destroyed by rt_destroy), not read\n";
    DeviceGuard guard;
    o += "streams of the context:\n";
    for (int m = 0; m < nmembers(ctx); ++m) {
        rt_ctx *c = member(ctx, m);
        stream_line(o, "current", m, c->device, c->stream);
        if (c->own_stream != c->stream) stream_line(o, "own", m, c->device, c->own_stream);
        stream_line(o, "slab", m, c->device, c->slab_stream2);
        stream_line(o, "copy", m, c->device, c->copy_stream);
        std::unique_lock<std::mutex> lk(c->copier.mu, std::try_to_lock);
        if (lk.owns_lock()) {
            char b[128];
            snprintf(b, sizeof b, "  member %d copier: %zu queued, %s\n", m, c->copier.jobs.size(),
                     c->copier.busy ? "copying" : "idle");
            o += b;
        } else {
            o += "  copier lock held\n";
        }
    }
    for (const GroupSlot &g : ctx->gslots) {
        if (!g.used) continue;
        for (size_t i = 0; i < g.member_stream.size(); ++i)
            stream_line(o, "group band", (int)i, member(ctx, (int)i)->device, g.member_stream[i]);
    }
    return o;
}

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
    const Wait w("ensure: hipFree + hipMalloc (device buffer growth)");
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
    const Wait w("ensure_out: hipFree + hipMalloc");
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
