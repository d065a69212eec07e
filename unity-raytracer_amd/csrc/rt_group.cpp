// rt_group.cpp — contexts: single-device creation / destruction and the
// multi-device context that renders block-cyclic row bands on N GPUs from one
// host thread and gathers them to device 0 over RCCL (or peer copies);
// SURVEY §8(e), RayTracingSetup.cs:288-301.
#include "rt_host.h"

namespace rti {

// RCCL, resolved at run time (only a multi-device context with an RCCL gather
// needs it; a single-GPU host never loads it).
struct Rccl {
    bool tried = false, ok = false;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    // the process's RCCL when one is loaded (PyTorch's has this soname), else ROCm's
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.send = (decltype(r.send))dlsym(h, "ncclSend");
    r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv && r.error_string;
    return r;
}

// A single-device context on device `dev` (made current).
int create_one(int dev, rt_ctx **out) {
    *out = nullptr;
    if (hipSetDevice(dev) != hipSuccess) return fail(nullptr, RT_E_NO_DEVICE, "hipSetDevice(%d) failed", dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return fail(nullptr, RT_E_NO_DEVICE, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, RT_E_NO_DEVICE, "device %d is %s; this library is built for gfx950 (MI355X)", dev,
                    prop.gcnArchName);
    rt_ctx *c = new rt_ctx();
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev_a0) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_slab0, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c->d_counters, rtd::kCounterSlots * rtd::kCounterWords * sizeof(unsigned long long)) !=
            hipSuccess ||
        hipHostMalloc((void **)&c->h_counts, rtd::kCounterWords * sizeof(unsigned long long),
                      hipHostMallocCoherent) != hipSuccess) {
        rt_destroy(c);
        return fail(nullptr, RT_E_HIP, "stream/event/counter allocation failed");
    }
    c->stream = c->own_stream;
    *out = c;
    return RT_OK;
}

void destroy_one(rt_ctx *ctx) {
    (void)hipSetDevice(ctx->device);
    {
        const Wait w("destroy: copier thread stop (join)");
        ctx->copier.stop();
    }
    {
        // only the context's own streams: its current stream may be a caller's
        // (rt_set_stream) that no longer exists — the frees below wait for
        // the device anyway
        const Wait w("destroy: hipStreamSynchronize (own, copy and slab streams)");
        if (ctx->own_stream) (void)hipStreamSynchronize(ctx->own_stream);
        if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
        if (ctx->slab_stream2) (void)hipStreamSynchronize(ctx->slab_stream2);
    }
    {
        const Wait w("destroy: hipFree of scene, LBVH, refit and longest-first buffers");
        free_scene(ctx);
        free_wavefront(ctx);
        ctx->lb.release();
        ctx->src.refit.release();
        for (LptSlot &l : ctx->lpt) l.release();
        if (ctx->wf_ctr) (void)hipFree(ctx->wf_ctr);
        if (ctx->d_out) (void)hipFree(ctx->d_out);
        if (ctx->d_counters) (void)hipFree(ctx->d_counters);
        if (ctx->d_cut) (void)hipFree(ctx->d_cut);
        if (ctx->wave_clock.p) (void)hipFree(ctx->wave_clock.p);
        if (ctx->d_rays) (void)hipFree(ctx->d_rays);
        if (ctx->d_hits) (void)hipFree(ctx->d_hits);
    }
    {
        const Wait w("destroy: hipHostFree (counter and update words)");
        if (ctx->h_counts) (void)hipHostFree(ctx->h_counts);
        if (ctx->h_update) (void)hipHostFree(ctx->h_update);
    }
    {
        const Wait w("destroy: hipEventDestroy");
        if (ctx->ev_x) (void)hipEventDestroy(ctx->ev_x);
        if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
        if (ctx->ev_a0) (void)hipEventDestroy(ctx->ev_a0);
        if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
        if (ctx->ev_slab0) (void)hipEventDestroy(ctx->ev_slab0);
        for (auto &se : ctx->async_end) (void)hipEventDestroy(se.second);
        for (hipEvent_t e : ctx->slab_done) (void)hipEventDestroy(e);
    }
    {
        const Wait w("destroy: hipStreamDestroy");
        if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
        if (ctx->slab_stream2) (void)hipStreamDestroy(ctx->slab_stream2);
        if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    }
    delete ctx;
}

void release_group(rt_ctx *ctx) {
    if (!ctx->comms.empty()) {  // only an RCCL group ever loaded the library
        const Wait w("destroy: ncclCommDestroy");
        Rccl &R = rccl();
        for (ncclComm_t c : ctx->comms)
            if (c && R.ok) (void)R.comm_destroy(c);
        ctx->comms.clear();
    }
    const int n = nmembers(ctx);
    for (GroupSlot &g : ctx->gslots) {
        if (!g.used) continue;
        for (int i = 0; i < n && i < (int)g.member_stream.size(); ++i) {
            rt_ctx *m = member(ctx, i);
            (void)hipSetDevice(m->device);
            // a member's frames ran on this stream (group_frame), and it is
            // still the member's current stream: back to its own before the
            // stream is destroyed — destroy_one synchronises the current
            // stream, and was handed this one's dangling handle until round 5
            // (whose one caught stall, r05c, had the host inside rt_destroy
            // of an 8-member group)
            if (m->stream == g.member_stream[(size_t)i]) m->stream = m->own_stream;
            if (g.member_stream[(size_t)i]) {
                {
                    const Wait w("destroy: hipStreamSynchronize (a group band stream)");
                    (void)hipStreamSynchronize(g.member_stream[(size_t)i]);
                }
                const Wait w("destroy: hipStreamDestroy (a group band stream)");
                (void)hipStreamDestroy(g.member_stream[(size_t)i]);
            }
            const Wait w("destroy: hipEventDestroy / hipFree (a group band's event and buffer)");
            if (g.member_done[(size_t)i]) (void)hipEventDestroy(g.member_done[(size_t)i]);
            if (g.member_out[(size_t)i].p) (void)hipFree(g.member_out[(size_t)i].p);
        }
        (void)hipSetDevice(ctx->device);
        const Wait w("destroy: hipFree / hipEventDestroy (the group's gather buffer and event)");
        if (g.gather.p) (void)hipFree(g.gather.p);
        if (g.gather_free) (void)hipEventDestroy(g.gather_free);
        g = GroupSlot{};
    }
    for (rt_ctx *p : ctx->peers) destroy_one(p);
    ctx->peers.clear();
}

// A context over `devices` (devices[0] = root; repeats = logical shards).
int create_group(const int32_t *devices, int32_t n, int32_t gather, rt_ctx **out_ctx) {
    DeviceGuard guard;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(nullptr, RT_E_NO_DEVICE, "no HIP device visible");
    bool distinct = true;
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= count)
            return fail(nullptr, RT_E_NO_DEVICE, "device %d not visible (%d devices)", devices[i], count);
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) distinct = false;
    }
    if (gather == 0) gather = n > 1 ? (distinct ? RT_GATHER_RCCL : RT_GATHER_PEER_COPY) : RT_GATHER_NONE;
    if (gather == RT_GATHER_NONE && n > 1)
        return fail(nullptr, RT_E_INVALID, "a %d-device context needs a gather transport", n);
    if (gather == RT_GATHER_RCCL && !distinct)
        return fail(nullptr, RT_E_INVALID, "RT_GATHER_RCCL needs distinct devices (one RCCL rank per GPU)");
    if (gather != RT_GATHER_NONE && gather != RT_GATHER_PEER_COPY && gather != RT_GATHER_RCCL)
        return fail(nullptr, RT_E_INVALID, "unknown gather transport %d", gather);
    rt_ctx *root = nullptr;
    int st = create_one(devices[0], &root);
    if (st) return st;
    for (int i = 1; i < n; ++i) {
        rt_ctx *p = nullptr;
        st = create_one(devices[i], &p);
        if (st) {
            release_group(root);
            destroy_one(root);
            return st;
        }
        root->peers.push_back(p);
    }
    root->gather = gather;
    if (gather == RT_GATHER_PEER_COPY && distinct) {
        // direct xGMI copies between the root and every other device
        for (int i = 1; i < n; ++i) {
            (void)hipSetDevice(devices[0]);
            hipError_t e = hipDeviceEnablePeerAccess(devices[i], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            (void)hipSetDevice(devices[i]);
            e = hipDeviceEnablePeerAccess(devices[0], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
    }
    if (gather == RT_GATHER_RCCL) {
        Rccl &R = rccl();
        if (!R.ok) {
            release_group(root);
            destroy_one(root);
            return fail(nullptr, RT_E_NO_DEVICE, "RT_GATHER_RCCL: librccl.so.1 not loadable");
        }
        root->comms.assign((size_t)n, nullptr);
        ncclResult_t r;
        {
            const Wait w("ncclCommInitAll");
            r = R.comm_init_all(root->comms.data(), n, devices);
        }
        if (r != ncclSuccess) {
            root->comms.clear();
            release_group(root);
            destroy_one(root);
            return fail(nullptr, RT_E_HIP, "ncclCommInitAll(%d devices): %s", n, R.error_string(r));
        }
    }
    *out_ctx = root;
    return RT_OK;
}

// The frame buffers of the root stream the next multi-device frame runs on.
int group_slot(rt_ctx *ctx, GroupSlot *&gs) {
    gs = nullptr;
    for (GroupSlot &g : ctx->gslots)
        if (g.used && g.root_stream == ctx->stream) gs = &g;
    if (gs) return RT_OK;
    for (GroupSlot &g : ctx->gslots)
        if (!g.used && !gs) gs = &g;
    if (!gs) return fail(ctx, RT_E_STATE, "more than %d streams in flight on a multi-device context", kGroupSlots);
    const int n = nmembers(ctx);
    gs->used = true;
    gs->root_stream = ctx->stream;
    gs->member_stream.assign((size_t)n, nullptr);
    gs->member_done.assign((size_t)n, nullptr);
    gs->member_out.assign((size_t)n, GrowBuf{});
    for (int i = 0; i < n; ++i) {
        HIP_OR_FAIL(ctx, hipSetDevice(member(ctx, i)->device));
        HIP_OR_FAIL(ctx, hipStreamCreateWithFlags(&gs->member_stream[(size_t)i], hipStreamNonBlocking));
        HIP_OR_FAIL(ctx, hipEventCreateWithFlags(&gs->member_done[(size_t)i], hipEventDisableTiming));
    }
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_OR_FAIL(ctx, hipEventCreateWithFlags(&gs->gather_free, hipEventDisableTiming));
    return RT_OK;
}

// A member's RT_FLAG_ASYNC bookkeeping, set aside while a synchronous
// multi-device frame uses it (so that frame's stats are its own).
struct AsyncStash {
    unsigned long long acc[rtd::kCounterWords];
    double ms;
    bool t0_set;
    std::chrono::steady_clock::time_point t0;
};

void stash_async(rt_ctx *m, AsyncStash &s) {
    std::memcpy(s.acc, m->async_acc, sizeof s.acc);
    s.ms = m->async_ms;
    s.t0_set = m->async_t0_set;
    s.t0 = m->async_t0;
    std::memset(m->async_acc, 0, sizeof m->async_acc);
    m->async_ms = 0.0;
    m->async_t0_set = false;
}

void unstash_async(rt_ctx *m, const AsyncStash &s) {
    std::memcpy(m->async_acc, s.acc, sizeof s.acc);
    m->async_ms = s.ms;
    m->async_t0_set = s.t0_set;
    m->async_t0 = s.t0;
}

// Waits for a member's async frames and takes their counters and device time.
int take_async(rt_ctx *m, unsigned long long counts[rtd::kCounterWords], double &ms) {
    HIP_OR_FAIL(m, hipSetDevice(m->device));
    const int st = settle_async(m);
    if (st) return st;
    std::memcpy(counts, m->async_acc, sizeof m->async_acc);
    ms = m->async_ms;
    std::memset(m->async_acc, 0, sizeof m->async_acc);
    m->async_ms = 0.0;
    m->async_t0_set = false;
    return RT_OK;
}

// A synchronous group frame's stats: every member's counters summed, the
// slowest member's kernel time.
int group_stats(rt_ctx *ctx, const std::vector<AsyncStash> &stash, rt_stats *stats,
                std::chrono::steady_clock::time_point t0) {
    unsigned long long sum[rtd::kCounterWords] = {0};
    double kms = 0.0;
    for (int i = 0; i < nmembers(ctx); ++i) {
        rt_ctx *m = member(ctx, i);
        unsigned long long c[rtd::kCounterWords];
        double ms = 0.0;
        const int st = take_async(m, c, ms);
        unstash_async(m, stash[(size_t)i]);
        if (st) {
            if (i) ctx->err = m->err;
            return st;
        }
        for (int w = 0; w < rtd::kCounterWords; ++w) sum[w] += c[w];
        kms = std::max(kms, ms);
    }
    if (stats)
        fill_stats(stats, sum, kms,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return RT_OK;
}

// Member `band` of `bands` copies its compact band (block-cyclic R-row
// blocks: local slot k holds image block k * bands + band) straight into the
// caller's host frame on its own stream: one 2-D copy for the whole blocks
// (source pitch = destination width = R rows, destination pitch = bands * R
// rows) plus the rows of a last partial block.
int copy_band_rows(rt_ctx *m, const void *band_buf, void *host, int res_x, int res_y, int band, int bands, int R,
                   int px_bytes) {
    const size_t row = (size_t)res_x * px_bytes;
    const int full = res_y / R;                                   // whole blocks of the image
    const int mine = full > band ? (full - band + bands - 1) / bands : 0;  // ... that are this member's
    if (mine > 0 && row > 0)
        HIP_WAIT(m, hipMemcpy2DAsync((char *)host + (size_t)band * R * row, (size_t)bands * R * row, band_buf,
                                        (size_t)R * row, (size_t)R * row, (size_t)mine, hipMemcpyDeviceToHost,
                                        m->stream));
    const int rest = res_y - full * R;  // rows of a last partial block
    if (rest > 0 && full % bands == band && row > 0)
        HIP_WAIT(m, hipMemcpyAsync((char *)host + (size_t)full * R * row,
                                      (const char *)band_buf + (size_t)(full / bands) * R * row, (size_t)rest * row,
                                      hipMemcpyDeviceToHost, m->stream));
    return RT_OK;
}

// One frame on a multi-device context: member i renders row band i of N
// (block-cyclic, 8-row blocks) on a stream of its own, the bands travel to
// the root (RCCL send/recv in one group, or peer copies), the root puts them
// back in row order (assemble kernel) into d_out and, with host_out, copies
// the frame to the host.  SURVEY §8(e); RayTracingSetup.cs:288-301.
int group_frame(rt_ctx *ctx, const rt_camera *cam, const rt_image_plane *plane, const rt_render_params *prm,
                void *d_out, void *host_out, size_t full_bytes, rt_stats *stats,
                std::chrono::steady_clock::time_point t0) {
    Range range("rt_group_frame");
    DeviceGuard guard;
    const int n = nmembers(ctx);
    const bool async = (prm->flags & RT_FLAG_ASYNC) != 0;
    const int R = prm->band_rows > 0 ? prm->band_rows : 8;
    const int px_bytes = rt_pixel_bytes(prm->flags);
    std::vector<rtd::FrameDev> F((size_t)n);
    std::vector<rt_render_params> mp((size_t)n, *prm);
    size_t shard = 0;
    for (int i = 0; i < n; ++i) {
        mp[(size_t)i].band_index = i;
        mp[(size_t)i].band_count = n;
        mp[(size_t)i].band_rows = R;
        mp[(size_t)i].flags |= RT_FLAG_ASYNC;
        size_t b = 0;
        int st = prepare_frame(member(ctx, i), cam, plane, &mp[(size_t)i], F[(size_t)i], b);
        if (st) {
            if (i) ctx->err = member(ctx, i)->err;
            return st;
        }
        shard = std::max(shard, b);  // every band has local_rows rows (the last ones padded)
    }
    GroupSlot *gs = nullptr;
    int st = group_slot(ctx, gs);
    if (st) return st;
    std::vector<AsyncStash> stash((size_t)n);
    const bool rccl_gather = ctx->gather == RT_GATHER_RCCL;
    // the root's band goes straight into the gather buffer unless it travels
    // through RCCL itself (a one-device RCCL context: self send/receive)
    const bool root_self_send = rccl_gather && n == 1;
    // rt_render into the caller's host frame: every member copies its own
    // row blocks straight into their rows over its own link (no gather, no
    // reassembly, no single-link copy of the whole frame from the root)
    const bool direct_host = host_out && full_bytes;
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    if (!direct_host) HIP_OR_FAIL(ctx, ensure(ctx, gs->gather, (size_t)n * shard));
    for (int i = 0; i < n; ++i) {
        rt_ctx *m = member(ctx, i);
        HIP_OR_FAIL(ctx, hipSetDevice(m->device));
        if (!async) {
            st = settle_async(m);  // the caller's pending async frames keep their stats
            if (st) return st;
            stash_async(m, stash[(size_t)i]);
        }
        void *out;
        if (i == 0 && !root_self_send && !direct_host) {
            out = gs->gather.p;
        } else {
            HIP_OR_FAIL(ctx, ensure(m, gs->member_out[(size_t)i], shard));
            out = gs->member_out[(size_t)i].p;
        }
        if (i > 0) {
            m->stream = gs->member_stream[(size_t)i];
            // this band's slot in the gather buffer is free once the previous
            // frame of this root stream has been reassembled
            HIP_OR_FAIL(ctx, hipStreamWaitEvent(m->stream, gs->gather_free, 0));
        }
        m->in_group_frame = true;
        st = run_frame(m, F[(size_t)i], &mp[(size_t)i], out, nullptr, t0, nullptr, 0);
        m->in_group_frame = false;
        if (st) {
            if (i) ctx->err = m->err;
            return st;
        }
        if (direct_host) {
            st = copy_band_rows(m, out, host_out, plane->resolution_x, plane->resolution_y, i, n, R, px_bytes);
            if (st) {
                if (i) ctx->err = m->err;
                return st;
            }
        }
    }
    if (direct_host) {
        for (int i = 0; i < n; ++i) {
            rt_ctx *m = member(ctx, i);
            HIP_OR_FAIL(ctx, hipSetDevice(m->device));
            HIP_WAIT(ctx, hipStreamSynchronize(m->stream));
        }
        HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
        return group_stats(ctx, stash, stats, t0);
    }
    // gather the bands to the root
    if (rccl_gather) {
        Range rr("rt_gather_rccl");
        Rccl &Rc = rccl();
        ncclResult_t r = Rc.group_start();
        for (int i = 1; i < n && r == ncclSuccess; ++i)
            r = Rc.recv((char *)gs->gather.p + (size_t)i * shard, shard, ncclChar, i, ctx->comms[0], ctx->stream);
        for (int i = 1; i < n && r == ncclSuccess; ++i)
            r = Rc.send(gs->member_out[(size_t)i].p, shard, ncclChar, 0, ctx->comms[(size_t)i],
                        gs->member_stream[(size_t)i]);
        if (root_self_send && r == ncclSuccess) {
            r = Rc.send(gs->member_out[0].p, shard, ncclChar, 0, ctx->comms[0], ctx->stream);
            if (r == ncclSuccess) r = Rc.recv(gs->gather.p, shard, ncclChar, 0, ctx->comms[0], ctx->stream);
        }
        ncclResult_t r2;
        {
            const Wait w("ncclGroupEnd (band gather)");
            r2 = Rc.group_end();
        }
        if (r != ncclSuccess || r2 != ncclSuccess)
            return fail(ctx, RT_E_HIP, "RCCL band gather: %s", Rc.error_string(r != ncclSuccess ? r : r2));
    } else {
        Range rr("rt_gather_peer");
        for (int i = 1; i < n; ++i) {
            rt_ctx *m = member(ctx, i);
            HIP_OR_FAIL(ctx, hipSetDevice(m->device));
            HIP_OR_FAIL(ctx, hipMemcpyPeerAsync((char *)gs->gather.p + (size_t)i * shard, ctx->device,
                                                gs->member_out[(size_t)i].p, m->device, shard, m->stream));
            HIP_OR_FAIL(ctx, hipEventRecord(gs->member_done[(size_t)i], m->stream));
        }
        HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
        for (int i = 1; i < n; ++i) HIP_OR_FAIL(ctx, hipStreamWaitEvent(ctx->stream, gs->member_done[(size_t)i], 0));
    }
    // back to row order on the root, then (rt_render) to the host
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    const int local = F[0].local_rows;
    HIP_OR_FAIL(ctx, rtk::launch_assemble(gs->gather.p, plane->resolution_x, plane->resolution_y, n, R, local,
                                          px_bytes, d_out, ctx->stream));
    HIP_OR_FAIL(ctx, hipEventRecord(gs->gather_free, ctx->stream));
    if (host_out && full_bytes)
        HIP_WAIT(ctx, hipMemcpyAsync(host_out, d_out, full_bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (async) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    return group_stats(ctx, stash, stats, t0);
}

}  // namespace rti
