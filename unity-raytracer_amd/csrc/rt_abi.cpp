// rt_abi.cpp — the extern "C" entry points of include/rt_mi355.h.
//
// Host side of the MI355X trace path: validates the reference-shaped scene,
// computes Scene.CalculateAABB exactly (Scene.cs:17-41), builds the BVH,
// lays the scene out in HBM (rt_device.h) and launches the gfx950 kernels
// (trace.hip).  There is no CPU fallback: without a gfx950 device every
// entry point fails with RT_E_NO_DEVICE / RT_E_HIP.  The work is done by the
// modules behind rt_host.h; this file validates arguments and dispatches.
#include "rt_host.h"

using namespace rti;

extern "C" {

int32_t rt_abi_version(void) { return RT_ABI_VERSION; }

float rt_spec_threshold(void) { return spec_threshold(); }

}  // extern "C"

extern "C" {

int rt_create(rt_ctx **out_ctx, int32_t num_gpus) {
    if (!out_ctx) return fail(nullptr, RT_E_INVALID, "out_ctx is null");
    *out_ctx = nullptr;
    if (num_gpus < 1) return fail(nullptr, RT_E_INVALID, "num_gpus must be >= 1, got %d", num_gpus);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(nullptr, RT_E_NO_DEVICE, "no HIP device visible");
    if (num_gpus == 1) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return fail(nullptr, RT_E_NO_DEVICE, "hipGetDevice failed");
        const int st = create_one(dev, out_ctx);
        if (st == RT_OK) register_ctx(*out_ctx);
        return st;
    }
    if (num_gpus > count)
        return fail(nullptr, RT_E_NO_DEVICE, "num_gpus %d > %d visible devices", num_gpus, count);
    std::vector<int32_t> devs((size_t)num_gpus);
    for (int i = 0; i < num_gpus; ++i) devs[(size_t)i] = i;
    const int st = create_group(devs.data(), num_gpus, 0, out_ctx);
    if (st == RT_OK) register_ctx(*out_ctx);
    return st;
}

int rt_create_devices(rt_ctx **out_ctx, const int32_t *devices, int32_t num_devices, int32_t gather) {
    if (!out_ctx) return fail(nullptr, RT_E_INVALID, "out_ctx is null");
    *out_ctx = nullptr;
    if (num_devices < 1 || !devices) return fail(nullptr, RT_E_INVALID, "need at least one device");
    const int st = create_group(devices, num_devices, gather, out_ctx);
    if (st == RT_OK) register_ctx(*out_ctx);
    return st;
}

int rt_get_device_info(const rt_ctx *ctx, rt_device_info *info) {
    if (!ctx || !info) return RT_E_INVALID;
    std::memset(info, 0, sizeof *info);
    info->num_devices = 1 + (int)ctx->peers.size();
    info->gather = ctx->gather;
    for (int i = 0; i < info->num_devices && i < 16; ++i)
        info->devices[i] = i == 0 ? ctx->device : ctx->peers[(size_t)i - 1]->device;
    return RT_OK;
}

void rt_destroy(rt_ctx *ctx) {
    if (!ctx) return;
    DeviceGuard guard;
    unregister_ctx(ctx);  // waits for a report reading it; later reports do not read it
    ctx->destroying.store(true);
    release_group(ctx);
    destroy_one(ctx);
}

const char *rt_last_error(const rt_ctx *ctx) {
    if (!ctx) return g_create_error.c_str();
    return ctx->err.c_str();
}

int rt_set_stream(rt_ctx *ctx, void *hip_stream) {
    if (!ctx) return RT_E_INVALID;
    ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
    return RT_OK;
}

// The default builder is the device LBVH collapsed to 4-wide nodes: a
// millisecond build instead of tens (host SAH) and, measured at round 4's final
// kernels, the faster tree to trace too (C5 -7 %, C4 -3 %, C3 -1..-3 %, C2 +-0;
// profiles/r04/abx_r04w).  A scene whose LBVH is too deep for the traversal
// stack (or that the LBVH path rejects) is built by the host SAH instead.
int rt_set_scene(rt_ctx *ctx, const rt_scene_desc *sc) {
    const int st = rt_set_scene_ex(ctx, sc, RT_BUILD_LBVH_GPU);
    if (st != RT_E_SCENE || !ctx) return st;
    return rt_set_scene_ex(ctx, sc, RT_BUILD_SAH_HOST);
}

int rt_set_scene_ex(rt_ctx *ctx, const rt_scene_desc *sc, int32_t build) {
    if (!ctx) return RT_E_INVALID;
    Range range("rt_set_scene");
    DeviceGuard guard;
    const auto t0 = std::chrono::steady_clock::now();
    return for_members(ctx, [&](rt_ctx *m) {
        m->src.active = false;
        return set_scene_impl(m, sc, build, false, t0);
    });
}

}  // extern "C"

extern "C" {

int rt_set_scene_source_ex(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count,
                           int32_t build) {
    if (!ctx) return RT_E_INVALID;
    Range range("rt_set_scene_source");
    DeviceGuard guard;
    const auto t0 = std::chrono::steady_clock::now();
    return for_members(ctx, [&](rt_ctx *m) { return set_scene_source_one(m, base, meshes, mesh_count, build, t0); });
}

int rt_set_scene_source(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count) {
    return rt_set_scene_source_ex(ctx, base, meshes, mesh_count, RT_BUILD_LBVH_GPU);
}

int rt_update_mesh_transforms(rt_ctx *ctx, const float *local_to_world, int32_t mesh_count) {
    if (!ctx) return RT_E_INVALID;
    Range range("rt_update_mesh_transforms");
    DeviceGuard guard;
    const auto t0 = std::chrono::steady_clock::now();
    return for_members(ctx, [&](rt_ctx *m) { return update_mesh_transforms_one(m, local_to_world, mesh_count, t0); });
}

int rt_get_scene_info(const rt_ctx *ctx, rt_scene_info *info) {
    if (!ctx || !info) return RT_E_INVALID;
    if (!ctx->has_scene) return RT_E_STATE;
    *info = ctx->info;
    return RT_OK;
}

int rt_export_bvh(const rt_ctx *ctx, void *nodes, void *triangle_records, void *sphere_records,
                  rt_bvh_export_info *info) {
    if (!ctx || !info) return RT_E_INVALID;
    if (!ctx->has_scene) return RT_E_STATE;
    std::memset(info, 0, sizeof *info);
    if (ctx->info.primitives > 0 && !ctx->S.bvh4) return RT_E_STATE;
    const int P = ctx->info.primitives;
    info->nodes = P > 0 ? ctx->info.nodes : 0;
    info->triangle_records = ctx->mesh_tri_ranks + ctx->loose_count + 1;  // + the sentinel
    info->sphere_records = ctx->sphere_count;
    DeviceGuard guard;
    if (hipSetDevice(ctx->device) != hipSuccess) return RT_E_HIP;
    const Wait w("rt_export_bvh: hipMemcpy");
    if (nodes && info->nodes &&
        hipMemcpy(nodes, ctx->S.nodes4, sizeof(rtd::BvhNode4) * (size_t)info->nodes, hipMemcpyDeviceToHost) !=
            hipSuccess)
        return RT_E_HIP;
    if (triangle_records && info->triangle_records &&
        hipMemcpy(triangle_records, ctx->S.tris, sizeof(rtd::TriRec) * (size_t)info->triangle_records,
                  hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    if (sphere_records && info->sphere_records &&
        hipMemcpy(sphere_records, ctx->S.sphs, sizeof(rtd::SphRec) * (size_t)info->sphere_records,
                  hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    return RT_OK;
}

int rt_finish(rt_ctx *ctx, rt_stats *stats) {
    if (!ctx) return RT_E_INVALID;
    DeviceGuard guard;
    // a multi-device context: every member's frames; device time = the slowest member's
    unsigned long long sum[rtd::kCounterWords] = {0};
    double kms = 0.0;
    const bool t0_set = ctx->async_t0_set;
    const auto t0 = ctx->async_t0;
    for (int i = 0; i < nmembers(ctx); ++i) {
        rt_ctx *m = member(ctx, i);
        unsigned long long c[rtd::kCounterWords];
        double ms = 0.0;
        const int st = take_async(m, c, ms);
        if (st) {
            if (i) ctx->err = m->err;
            return st;
        }
        for (int w = 0; w < rtd::kCounterWords; ++w) sum[w] += c[w];
        kms = std::max(kms, ms);
    }
    std::memcpy(ctx->last_counts, sum, sizeof sum);
    if (stats) {
        const double wall =
            t0_set ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() : 0.0;
        fill_stats(stats, sum, kms, wall);
    }
    return RT_OK;
}

int32_t rt_band_rows_local(int32_t resolution_y, int32_t band_index, int32_t band_count, int32_t band_rows) {
    (void)band_index;
    return band_local_rows(resolution_y, band_count <= 0 ? 1 : band_count, band_rows <= 0 ? 8 : band_rows);
}

int rt_render(rt_ctx *ctx, const rt_camera *camera, const rt_image_plane *plane, const rt_render_params *params,
              void *out_rgba, rt_stats *stats) {
    if (!ctx) return RT_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    Range range("rt_render");
    DeviceGuard guard;
    if (params && (params->flags & RT_FLAG_ASYNC))
        return fail(ctx, RT_E_INVALID, "RT_FLAG_ASYNC needs a device output (rt_render_device)");
    const bool group = !ctx->peers.empty() || ctx->gather == RT_GATHER_RCCL;
    if (group && params && params->band_count <= 1) {
        if (!camera || !plane) return fail(ctx, RT_E_INVALID, "null camera/plane/params");
        if (plane->resolution_x < 0 || plane->resolution_y < 0)
            return fail(ctx, RT_E_INVALID, "negative resolution (%d, %d)", plane->resolution_x, plane->resolution_y);
        const size_t bytes = (size_t)plane->resolution_x * plane->resolution_y * rt_pixel_bytes(params->flags);
        if (bytes && !out_rgba) return fail(ctx, RT_E_INVALID, "out_rgba is null");
        HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
        // every member copies its own rows to the host: no root-side frame buffer
        return group_frame(ctx, camera, plane, params, nullptr, out_rgba, bytes, stats, t0);
    }
    rtd::FrameDev F;
    size_t bytes = 0;
    int st = prepare_frame(ctx, camera, plane, params, F, bytes);
    if (st) return st;
    if (bytes && !out_rgba) return fail(ctx, RT_E_INVALID, "out_rgba is null");
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_OR_FAIL(ctx, ensure_out(ctx, bytes));
    return run_frame(ctx, F, params, ctx->d_out, stats, t0, out_rgba, bytes);
}

int rt_render_device(rt_ctx *ctx, const rt_camera *camera, const rt_image_plane *plane,
                     const rt_render_params *params, void *d_out_rgba, size_t out_bytes, rt_stats *stats) {
    if (!ctx) return RT_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    DeviceGuard guard;
    const bool group = !ctx->peers.empty() || ctx->gather == RT_GATHER_RCCL;
    if (group && params && params->band_count <= 1) {
        if (!camera || !plane) return fail(ctx, RT_E_INVALID, "null camera/plane/params");
        if (plane->resolution_x < 0 || plane->resolution_y < 0)
            return fail(ctx, RT_E_INVALID, "negative resolution (%d, %d)", plane->resolution_x, plane->resolution_y);
        const size_t bytes = (size_t)plane->resolution_x * plane->resolution_y * rt_pixel_bytes(params->flags);
        if (bytes && !d_out_rgba) return fail(ctx, RT_E_INVALID, "d_out_rgba is null");
        if (out_bytes < bytes)
            return fail(ctx, RT_E_INVALID, "output buffer %zu bytes < %zu required", out_bytes, bytes);
        return group_frame(ctx, camera, plane, params, d_out_rgba, nullptr, 0, stats, t0);
    }
    rtd::FrameDev F;
    size_t bytes = 0;
    int st = prepare_frame(ctx, camera, plane, params, F, bytes);
    if (st) return st;
    if (bytes && !d_out_rgba) return fail(ctx, RT_E_INVALID, "d_out_rgba is null");
    if (out_bytes < bytes)
        return fail(ctx, RT_E_INVALID, "output buffer %zu bytes < %zu required", out_bytes, bytes);
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    return run_frame(ctx, F, params, d_out_rgba, stats, t0, nullptr, 0);
}

int rt_render_device_batch(rt_ctx *ctx, int32_t num_frames, const rt_camera *cameras, const rt_image_plane *plane,
                           const rt_render_params *params, void *d_out, size_t frame_stride_bytes, rt_stats *stats) {
    if (!ctx) return RT_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    DeviceGuard guard;
    if (num_frames < 1 || num_frames > RT_MAX_BATCH)
        return fail(ctx, RT_E_INVALID, "num_frames %d outside [1, %d]", num_frames, RT_MAX_BATCH);
    if (!cameras || !plane || !params) return fail(ctx, RT_E_INVALID, "null cameras/plane/params");
    static_assert(RT_MAX_BATCH == rtd::kMaxBatch, "rt_mi355.h RT_MAX_BATCH");
    const bool group = !ctx->peers.empty() || ctx->gather == RT_GATHER_RCCL;
    rtd::FrameDev F[RT_MAX_BATCH];
    size_t bytes = 0;
    bool one_launch = !group;
    if (one_launch) {
        for (int i = 0; i < num_frames; ++i) {
            const int st = prepare_frame(ctx, &cameras[i], plane, params, F[i], bytes);
            if (st) return st;
        }
        one_launch = batch_launchable(ctx, F[0], params, num_frames);
    }
    if (!one_launch) {
        // frames one by one (the same frames; stats summed, device time added)
        rt_stats sum{}, one{};
        for (int i = 0; i < num_frames; ++i) {
            const int st = rt_render_device(ctx, &cameras[i], plane, params, (char *)d_out + (size_t)i * frame_stride_bytes,
                                            frame_stride_bytes, stats ? &one : nullptr);
            if (st) return st;
            if (!stats) continue;
            sum.primary_rays += one.primary_rays;
            sum.shadow_rays += one.shadow_rays;
            sum.reflection_rays += one.reflection_rays;
            sum.box_tests += one.box_tests;
            sum.triangle_tests += one.triangle_tests;
            sum.sphere_tests += one.sphere_tests;
            sum.shading_fetches += one.shading_fetches;
            sum.primary_scene_misses += one.primary_scene_misses;
            sum.shadow_rays_moot += one.shadow_rays_moot;
            sum.kernel_ms += one.kernel_ms;
        }
        if (stats) {
            sum.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            *stats = sum;
        }
        return RT_OK;
    }
    if (bytes && !d_out) return fail(ctx, RT_E_INVALID, "d_out is null");
    if (frame_stride_bytes < bytes)
        return fail(ctx, RT_E_INVALID, "frame stride %zu bytes < %zu required", frame_stride_bytes, bytes);
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    const BatchIn bi{F, num_frames, frame_stride_bytes};
    rtd::FrameDev H = F[0];
    return run_frame(ctx, H, params, d_out, stats, t0, nullptr, 0, &bi);
}

int rt_assemble_bands(rt_ctx *ctx, const float *d_gathered, int32_t resolution_x, int32_t resolution_y,
                      int32_t band_count, int32_t band_rows, float *d_image) {
    const int st = rt_assemble_bands_ex(ctx, d_gathered, resolution_x, resolution_y, band_count, band_rows, 16,
                                        d_image);
    return st ? st : rt_synchronize(ctx);
}

int32_t rt_pixel_bytes(int32_t flags) {
    return (flags & RT_FLAG_OUT_RGBA8) ? 4 : ((flags & RT_FLAG_OUT_RGBA16F) ? 8 : ((flags & RT_FLAG_OUT_RGB32F) ? 12 : 16));
}

int rt_assemble_bands_ex(rt_ctx *ctx, const void *d_gathered, int32_t resolution_x, int32_t resolution_y,
                         int32_t band_count, int32_t band_rows, int32_t pixel_bytes, void *d_image) {
    if (!ctx) return RT_E_INVALID;
    if (!d_gathered || !d_image || resolution_x < 0 || resolution_y < 0 || band_count < 1 ||
        (pixel_bytes != 4 && pixel_bytes != 8 && pixel_bytes != 12 && pixel_bytes != 16))
        return fail(ctx, RT_E_INVALID, "bad rt_assemble_bands arguments");
    if (band_rows <= 0) band_rows = 8;
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    const int local = band_local_rows(resolution_y, band_count, band_rows);
    HIP_OR_FAIL(ctx, rtk::launch_assemble(d_gathered, resolution_x, resolution_y, band_count, band_rows, local,
                                          pixel_bytes, d_image, ctx->stream));
    return RT_OK;  // stream-ordered: rt_synchronize (or the stream) before reading d_image elsewhere
}

int rt_synchronize(rt_ctx *ctx) {
    if (!ctx) return RT_E_INVALID;
    DeviceGuard guard;
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    for (const GroupSlot &g : ctx->gslots)
        for (size_t i = 1; g.used && i < g.member_stream.size(); ++i) {
            HIP_OR_FAIL(ctx, hipSetDevice(member(ctx, (int)i)->device));
            HIP_WAIT(ctx, hipStreamSynchronize(g.member_stream[i]));
        }
    return RT_OK;
}

int rt_intersect_rays(rt_ctx *ctx, const rt_ray *rays, int32_t n, rt_hit *out_hits) {
    if (!ctx) return RT_E_INVALID;
    if (n < 0 || (n > 0 && (!rays || !out_hits))) return fail(ctx, RT_E_INVALID, "bad rays/out_hits");
    if (!ctx->has_scene) return fail(ctx, RT_E_STATE, "rt_intersect_rays before rt_set_scene");
    if (n == 0) return RT_OK;
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    if ((size_t)n > ctx->rays_cap) {
        if (ctx->d_rays) HIP_OR_FAIL(ctx, hipFree(ctx->d_rays));
        if (ctx->d_hits) HIP_OR_FAIL(ctx, hipFree(ctx->d_hits));
        ctx->d_rays = nullptr;
        ctx->d_hits = nullptr;
        ctx->rays_cap = 0;
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->d_rays, (size_t)n * sizeof(rt_ray)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->d_hits, (size_t)n * sizeof(int4)));
        ctx->rays_cap = (size_t)n;
    }
    HIP_WAIT(ctx, hipMemcpyAsync(ctx->d_rays, rays, (size_t)n * sizeof(rt_ray), hipMemcpyHostToDevice,
                                    ctx->stream));
    HIP_OR_FAIL(ctx, rtk::launch_intersect(ctx->S, ctx->d_rays, n, ctx->d_hits, ctx->stream));
    std::vector<int4> hits((size_t)n);
    HIP_WAIT(ctx, hipMemcpyAsync(hits.data(), ctx->d_hits, (size_t)n * sizeof(int4), hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    for (int32_t i = 0; i < n; ++i) {
        const int rk = hits[i].x;
        rt_hit &h = out_hits[i];
        std::memcpy(&h.distance, &hits[i].y, 4);
        h.type = 0;
        h.index = -1;
        h.mesh_index = -1;
        if (rk < 0) {
            h.distance = FLT_MAX;  // float.MaxValue
        } else if (rk < ctx->mesh_tri_ranks) {
            const auto &f = ctx->mesh_rank_first;
            const int m = (int)(std::upper_bound(f.begin(), f.end() - 1, rk) - f.begin()) - 1;
            h.type = 3;
            h.mesh_index = m;
            h.index = rk - f[m];
        } else {
            if (rk < ctx->mesh_tri_ranks + ctx->sphere_count) {
                h.type = 1;
                h.index = rk - ctx->mesh_tri_ranks;
            } else {
                h.type = 2;
                h.index = rk - ctx->mesh_tri_ranks - ctx->sphere_count;
            }
            // a sphere / loose triangle won after a mesh triangle had been the
            // running closest hit: the reference keeps that mesh's index
            // (Scene.cs:76-79 set it, :94-97 and :109-112 never reset it)
            const int mr = hits[i].z;
            if (mr >= 0 && mr < ctx->mesh_tri_ranks) {
                const auto &f = ctx->mesh_rank_first;
                h.mesh_index = (int)(std::upper_bound(f.begin(), f.end() - 1, mr) - f.begin()) - 1;
            }
        }
    }
    return RT_OK;
}

int rt_debug_set(rt_ctx *ctx, int32_t what, int32_t value) {
    if (!ctx) return RT_E_INVALID;
    if (what == RT_DEBUG_GROUP_SAMPLE_WAVES) {
        for (int i = 0; i < nmembers(ctx); ++i) member(ctx, i)->debug_group_sample_waves = value != 0;
        return RT_OK;
    }
    if (what == RT_DEBUG_SAMPLE_WAVE_STACK) {
        if (value < 0) return fail(ctx, RT_E_INVALID, "RT_DEBUG_SAMPLE_WAVE_STACK: capacity >= 0");
        for (int i = 0; i < nmembers(ctx); ++i) member(ctx, i)->debug_sample_wave_stack = value;
        return RT_OK;
    }
    if (what == RT_DEBUG_FAIL_SLAB) {
        ctx->debug_fail_slab = value;
        return RT_OK;
    }
    if (what == RT_DEBUG_WAVE_CLOCKS) {
        if (!rtk::kWaveClockBuild)
            return fail(ctx, RT_E_STATE, "RT_DEBUG_WAVE_CLOCKS: measuring builds only (-DRT_WAVE_CLOCK)");
        ctx->debug_wave_clock = value != 0;
        return RT_OK;
    }
    return fail(ctx, RT_E_INVALID, "unknown rt_debug_set item %d", what);
}

int rt_debug_read(rt_ctx *ctx, int32_t what, void *out, int64_t capacity_bytes, int64_t *bytes_written) {
    if (bytes_written) *bytes_written = 0;
    if (what == RT_DEBUG_HOST_WAITS) {
        if (!out || capacity_bytes <= 0) return ctx ? fail(ctx, RT_E_INVALID, "rt_debug_read: no output") : RT_E_INVALID;
        const std::string r = host_waits_report(ctx);
        const int64_t n = std::min<int64_t>(capacity_bytes - 1, (int64_t)r.size());
        std::memcpy(out, r.data(), (size_t)n);
        static_cast<char *>(out)[n] = 0;
        if (bytes_written) *bytes_written = n + 1;
        return RT_OK;
    }
    if (!ctx) return RT_E_INVALID;
    if (what == RT_DEBUG_COUNTERS) {
        if (!out || capacity_bytes <= 0) return fail(ctx, RT_E_INVALID, "rt_debug_read: no output");
        const int64_t n = std::min<int64_t>(capacity_bytes, (int64_t)sizeof ctx->last_counts);
        std::memcpy(out, ctx->last_counts, (size_t)n);
        if (bytes_written) *bytes_written = n;
        return RT_OK;
    }
    if (what == RT_DEBUG_LAST_LAUNCH) {
        if (!out || capacity_bytes <= 0) return fail(ctx, RT_E_INVALID, "rt_debug_read: no output");
        const std::string &r = ctx->last_launch;
        const int64_t n = std::min<int64_t>(capacity_bytes - 1, (int64_t)r.size());
        std::memcpy(out, r.data(), (size_t)n);
        static_cast<char *>(out)[n] = 0;
        if (bytes_written) *bytes_written = n + 1;
        return RT_OK;
    }
    if (what != RT_DEBUG_WAVE_CLOCKS) return fail(ctx, RT_E_INVALID, "unknown rt_debug_read item %d", what);
    if (!ctx->debug_wave_clock) return fail(ctx, RT_E_STATE, "RT_DEBUG_WAVE_CLOCKS is off");
    if (!out || capacity_bytes < 0) return fail(ctx, RT_E_INVALID, "rt_debug_read: null output or negative size");
    DeviceGuard guard;
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_WAIT(ctx, hipDeviceSynchronize());
    const int64_t n = std::min<int64_t>(capacity_bytes, ctx->wave_clock_bytes);
    if (n > 0) HIP_WAIT(ctx, hipMemcpy(out, ctx->wave_clock.p, (size_t)n, hipMemcpyDeviceToHost));
    if (bytes_written) *bytes_written = n;
    return RT_OK;
}

}  // extern "C"
