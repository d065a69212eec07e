// rt_frame.cpp — one frame: CastPixelRays' constants (RayTracingSetup.cs:
// 275-302, ImagePlane.cs:26-44), the conservative sky test and tile frustum
// constants, longest-first tile dispatch, the trace launches, the sharded ray
// counters, RT_FLAG_ASYNC bookkeeping and rt_render's host-output pipeline
// (row slabs on two streams, copies from a thread of their own).
#include "rt_host.h"

namespace rti {

int isqrt_exact(int v) {
    if (v <= 0) return -1;
    int n = 1;
    while (n * n < v) ++n;
    return n * n == v ? n : -1;
}

// The conservative sky test's per-frame constants (rt_device.h FrameDev
// sky_*), in double: the Scene.AABB padded by 2^-10 of the camera-relative
// scene scale.  An exact sample ray that passes the exact gate (RMath.cs:12-26)
// comes geometrically within ~1e-7 of that scale of the box; the kernel's
// approximate ray deviates by ~1e-6 of it; the pad is ~1e-3 of it.  Off when
// anything is non-finite or the camera is inside the padded box (every ray
// may then enter it).
void sky_setup(const rtd::SceneDev &S, rtd::FrameDev &F) {
    F.sky_test = 0;
    if (!S.has_prims || F.res_x <= 0 || F.res_y <= 0) return;
    double lo[3], hi[3], c[3], scale = 0.0;
    bool finite = std::isfinite(F.hl) && std::isfinite(F.vl);
    for (int a = 0; a < 3; ++a) {
        c[a] = F.cam_pos[a];
        lo[a] = (double)S.scene_lo[a] - c[a];
        hi[a] = (double)S.scene_hi[a] - c[a];
        finite = finite && std::isfinite(lo[a]) && std::isfinite(hi[a]) && lo[a] <= hi[a] &&
                 std::isfinite(F.top_left[a]) && std::isfinite(F.right[a]) && std::isfinite(F.up[a]);
        scale = std::max(scale, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
    }
    if (!finite) return;
    const double pad = std::ldexp(std::max(scale, 1e-30), -10);
    bool inside = true;
    for (int a = 0; a < 3; ++a) {
        lo[a] -= pad;
        hi[a] += pad;
        inside = inside && lo[a] <= 0.0 && hi[a] >= 0.0;
        F.sky_lo[a] = (float)lo[a];
        F.sky_hi[a] = (float)hi[a];
        F.sky_tlc[a] = (float)((double)F.top_left[a] - c[a]);
    }
    if (inside) return;
    // rounding the padded bounds to float moves them by far less than the pad
    F.sky_hx = (float)((double)F.hl / F.res_x);
    F.sky_vy = (float)((double)F.vl / F.res_y);
    F.sky_test = 1;
}

// The camera packets' tile frustum (FrameDev cut_*, packet.h cut_start):
// D(x, y) = A + x R + y U; the plane through the camera spanned by D(xa, .)
// has the normal cross(A + xa R, U) = cross(A, U) + xa cross(R, U), on the
// side x >= xa when multiplied by sign(det[A, U, R]); likewise y with
// cross(A + ya U, R) and sign(det[A, R, U]).  Computed in double, rounded.
void cut_setup(const rtd::SceneDev &S, rtd::FrameDev &F, bool no_cut) {
    F.cut_test = 0;
    if (!S.cut || !S.bvh4 || !S.has_prims || F.res_x <= 0 || F.res_y <= 0) return;
    if (no_cut) return;  // RT_FLAG_NO_CUT: every camera packet from the root
    // a tile's rows must lie in one band block (contiguous image rows)
    if (F.band_count > 1 && F.band_rows % F.tile_h != 0) return;
    double A[3], R[3], U[3];
    for (int a = 0; a < 3; ++a) {
        A[a] = (double)F.top_left[a] - (double)F.cam_pos[a];
        R[a] = (double)F.right[a] * F.hl / F.res_x;
        U[a] = -(double)F.up[a] * F.vl / F.res_y;
    }
    auto cross = [](const double *p, const double *q, double *o) {
        o[0] = p[1] * q[2] - p[2] * q[1];
        o[1] = p[2] * q[0] - p[0] * q[2];
        o[2] = p[0] * q[1] - p[1] * q[0];
    };
    double aU[3], rU[3], aR[3], uR[3];
    cross(A, U, aU);
    cross(R, U, rU);
    cross(A, R, aR);
    cross(U, R, uR);
    const double det = aU[0] * R[0] + aU[1] * R[1] + aU[2] * R[2];  // det[A, U, R]
    bool finite = std::isfinite(det) && det != 0.0;
    const double sx = det > 0.0 ? 1.0 : -1.0, sy = -sx;  // det[A, R, U] = -det[A, U, R]
    for (int a = 0; a < 3; ++a) {
        F.cut_ax[a] = (float)(sx * aU[a]);
        F.cut_bx[a] = (float)(sx * rU[a]);
        F.cut_ay[a] = (float)(sy * aR[a]);
        F.cut_by[a] = (float)(sy * uR[a]);
        F.cut_a[a] = (float)A[a];
        F.cut_r[a] = (float)R[a];
        F.cut_u[a] = (float)U[a];
        finite = finite && std::isfinite(F.cut_ax[a]) && std::isfinite(F.cut_bx[a]) && std::isfinite(F.cut_ay[a]) &&
                 std::isfinite(F.cut_by[a]) && std::isfinite(F.cam_pos[a]);
    }
    F.cut_test = finite ? 1 : 0;
}

int prepare_frame(rt_ctx *ctx, const rt_camera *cam, const rt_image_plane *plane, const rt_render_params *prm,
                  rtd::FrameDev &F, size_t &out_bytes) {
    if (!cam || !plane || !prm) return fail(ctx, RT_E_INVALID, "null camera/plane/params");
    if (!ctx->has_scene) return fail(ctx, RT_E_STATE, "rt_render before rt_set_scene");
    if (plane->resolution_x < 0 || plane->resolution_y < 0)
        return fail(ctx, RT_E_INVALID, "negative resolution (%d, %d)", plane->resolution_x, plane->resolution_y);
    const int n = isqrt_exact(prm->samples_per_pixel);
    if (n < 0 || n > 8)
        return fail(ctx, RT_E_INVALID, "samples_per_pixel must be n*n with 1 <= n <= 8, got %d",
                    prm->samples_per_pixel);
    const int band_count = prm->band_count <= 0 ? 1 : prm->band_count;
    const int band_rows = prm->band_rows <= 0 ? 8 : prm->band_rows;
    if (prm->band_index < 0 || prm->band_index >= band_count)
        return fail(ctx, RT_E_INVALID, "band_index %d outside [0, %d)", prm->band_index, band_count);
    std::memset(&F, 0, sizeof F);
    // ImagePlane.GetRect(cameraData).TopLeft (ImagePlane.cs:26-44)
    const rtm::f3 center = F3(cam->position) + F3(cam->forward) * plane->distance_to_camera;
    const rtm::f3 half_up = F3(cam->up) * plane->half_vertical_length;
    const rtm::f3 half_right = F3(cam->right) * plane->half_horizontal_length;
    const rtm::f3 tl = (center - half_right) + half_up;
    F.cam_pos[0] = cam->position.x; F.cam_pos[1] = cam->position.y; F.cam_pos[2] = cam->position.z;
    F.right[0] = cam->right.x; F.right[1] = cam->right.y; F.right[2] = cam->right.z;
    F.up[0] = cam->up.x; F.up[1] = cam->up.y; F.up[2] = cam->up.z;
    F.top_left[0] = tl.x; F.top_left[1] = tl.y; F.top_left[2] = tl.z;
    F.hl = plane->half_horizontal_length * 2.0f;  // HorizontalLength, ImagePlane.cs:23
    F.vl = plane->half_vertical_length * 2.0f;
    for (int i = 0; i < 3; ++i) F.bg255[i] = prm->background_color[i] * 255.0f;  // Rgb(Color), Rgb.cs:15-18
    F.res_x = plane->resolution_x;
    F.res_y = plane->resolution_y;
    F.spp = n * n;
    F.spp_n = n;
    F.inv_spp = 1.0f / (float)F.spp;
    F.max_bounces = prm->max_reflection_bounces;
    F.band_index = prm->band_index;
    F.band_count = band_count;
    F.band_rows = band_rows;
    F.band_rows_magic = band_rows <= 1 ? 0xffffffffu : (unsigned)((1ull << 32) / (unsigned long long)band_rows);
    F.local_rows = band_local_rows(F.res_y, band_count, band_rows);
    // tile: 64/spp pixels per wave; a power of two is laid out as a
    // near-square 2^a x 2^b block
    const int ppw = rtd::kWaveSize / F.spp;
    int tw = ppw, th = 1;
    if ((ppw & (ppw - 1)) == 0) {
        int lg = 0;
        while ((1 << lg) < ppw) ++lg;
        th = 1 << (lg / 2);
        tw = ppw / th;
    }
    F.tile_w = tw;
    F.tile_h = th;
    F.tiles_x = (F.res_x + tw - 1) / tw;
    F.tiles_x_magic = F.tiles_x <= 1 ? 0xffffffffu : (unsigned)((1ull << 32) / (unsigned long long)F.tiles_x);
    F.s16_shift = 2;  // finely split tiles: a pixel per wave (lpt_prepare may choose a sample per wave)
    F.sample_wave_stack = ctx->debug_sample_wave_stack;  // 0: the wave's whole LDS stack area
    const int tiles_y = (F.local_rows + th - 1) / th;
    F.num_tiles = F.res_x > 0 ? F.tiles_x * tiles_y : 0;
    const bool f8 = (prm->flags & RT_FLAG_OUT_RGBA8) != 0, f16 = (prm->flags & RT_FLAG_OUT_RGBA16F) != 0,
               f12 = (prm->flags & RT_FLAG_OUT_RGB32F) != 0;
    if ((int)f8 + (int)f16 + (int)f12 > 1)
        return fail(ctx, RT_E_INVALID, "RT_FLAG_OUT_RGBA8, RT_FLAG_OUT_RGBA16F and RT_FLAG_OUT_RGB32F are exclusive");
    F.out_format = f8 ? rtd::kOutRGBA8 : (f16 ? rtd::kOutRGBA16F : (f12 ? rtd::kOutRGB32F : rtd::kOutFloat4));
    out_bytes = (size_t)F.local_rows * F.res_x * rt_pixel_bytes(prm->flags);
    sky_setup(ctx->S, F);
    cut_setup(ctx->S, F, (prm->flags & RT_FLAG_NO_CUT) != 0);
    return RT_OK;
}

// Upper bound on wavefront pool entries (64 B each) per chunk: 160M = 10 GB.
constexpr size_t kPoolBudget = (size_t)160 << 20;
constexpr size_t kShadowBudget = (size_t)96 << 20;

void free_wavefront(rt_ctx *c) {
    void *ps[] = {c->wf_ray_o, c->wf_ray_d, c->wf_col, c->wf_sh_o, c->wf_sh_d, c->wf_hit, c->wf_occ};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    c->wf_ray_o = c->wf_ray_d = c->wf_col = c->wf_sh_o = c->wf_sh_d = nullptr;
    c->wf_hit = nullptr;
    c->wf_occ = nullptr;
    c->pool_cap = c->shadow_cap = 0;
}

// Chunk size (tiles) so that the worst case (every hit a mirror down to the
// bounce limit) fits the pool budget, and (re)allocation of the queues.
int prepare_wavefront(rt_ctx *ctx, const rtd::FrameDev &F, int &chunk_tiles, rtw::Args &A) {
    const size_t levels = (size_t)(F.max_bounces > 0 ? F.max_bounces : 0) + 1;
    const size_t lights = (size_t)std::max(1, ctx->S.num_lights);
    size_t tiles = (size_t)std::max(1, F.num_tiles);
    tiles = std::min(tiles, std::max<size_t>(1, kPoolBudget / (levels * 64)));
    tiles = std::min(tiles, std::max<size_t>(1, kShadowBudget / (lights * 64)));
    chunk_tiles = (int)tiles;
    const size_t pool = tiles * 64 * levels, shadow = tiles * 64 * lights;
    if (!ctx->wf_ctr) HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_ctr, sizeof(rtw::Counters)));
    if (pool > ctx->pool_cap || shadow > ctx->shadow_cap) {
        HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
        free_wavefront(ctx);
        const size_t p = std::max(pool, ctx->pool_cap), q = std::max(shadow, ctx->shadow_cap);
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_ray_o, p * sizeof(float4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_ray_d, p * sizeof(float4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_col, p * sizeof(float4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_hit, p * sizeof(int4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_sh_o, q * sizeof(float4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_sh_d, q * sizeof(float4)));
        HIP_OR_FAIL(ctx, hipMalloc(&ctx->wf_occ, q));
        ctx->pool_cap = p;
        ctx->shadow_cap = q;
    }
    A.ctr = ctx->wf_ctr;
    A.ray_o = ctx->wf_ray_o;
    A.ray_d = ctx->wf_ray_d;
    A.hit = ctx->wf_hit;
    A.col = ctx->wf_col;
    A.sh_o = ctx->wf_sh_o;
    A.sh_d = ctx->wf_sh_d;
    A.occ = ctx->wf_occ;
    A.tile0 = 0;
    A.n0 = 0;
    A.max_level = (int)levels - 1;
    return RT_OK;
}


// Quarter-wave splitting of a frame's slowest tiles trades extra work (each
// quarter re-walks the BVH top) for a shorter critical path; it pays only
// when the frame (shard) is small enough for its slowest wave to set its
// time: measured with 3 frames in flight, a 1/8 C3 shard (16,200 tiles)
// +18 %, a 1/4 shard (32,400) -7 %, a whole frame (129,600) -7 %.  The very
// slowest of them (1/2048 of the tiles) go further, to sixteen waves of one
// pixel each: a 1/8 shard's single frame -14 % more, throughput with frames
// in flight +-1 % (1/512 or more: -5..-15 %).
#ifdef RT_EXP_SPLIT16DIV
constexpr int kSplit16Div = RT_EXP_SPLIT16DIV;  // measuring builds only
#else
constexpr int kSplit16Div = 2048;  // of those, 1/kSplit16Div of the tiles as sixteenth-waves; 0: off
#endif
#ifdef RT_EXP_SPLITDIV
constexpr int kSplitDiv = RT_EXP_SPLITDIV;  // measuring builds only
#else
constexpr int kSplitDiv = 256;  // 1/kSplitDiv of the tiles (the slowest) run as quarter-waves; 0: off
#endif
// A lone shard's finely split tiles run as one-sample waves traced by the
// whole wave (trace.hip render_sample_wave, csrc/coop.h): cheap enough to
// split its slowest 1/256 so (1/1024 before the whole-wave traversal: the
// rest of a 1/8 C3 share's slowest waves were whole tiles of ~105 us):
// single frame -13 % on two 1/8 shares against 1/1024 (r05q).
#ifdef RT_EXP_SPLIT16SAMPLE
constexpr int kSplit16DivSample = RT_EXP_SPLIT16SAMPLE;  // measuring builds only
#else
constexpr int kSplit16DivSample = 256;
#endif
// Larger shards (up to 70,000 tiles: a 1/2 or 1/4 shard of 1080p) split only
// their slowest 1/4096 into sixteenth-waves: single frame -15..-30 %,
// throughput with frames in flight +2..4 % on a 1/4 shard; a whole frame
// (129,600 tiles) loses 2-6 % and does not split.
#ifdef RT_EXP_SPLITMAX
constexpr int kSplitMaxTiles = RT_EXP_SPLITMAX;  // measuring builds only
#else
constexpr int kSplitMaxTiles = 24000;    // ... in frames/shards of at most this many tiles
#endif
#ifdef RT_EXP_SPLIT16MAX
constexpr int kSplit16MaxTiles = RT_EXP_SPLIT16MAX;  // measuring builds only
#else
constexpr int kSplit16MaxTiles = 70000;
#endif
constexpr int kSplit16DivLarge = 4096;
// A lone whole frame (more than kSplit16MaxTiles tiles, no other frame beside
// it) splits only its slowest 1/16384: C3 single frame -1.7 %, C2 -2.1 %
// against 1/4096 (1/8192: -1.1 / -1.1 %; r04aq, r04ar); 1/32768 +6 %, one
// tile +15 % on C3 (r04au).
#ifdef RT_EXP_SPLIT16WHOLE
constexpr int kSplit16DivWhole = RT_EXP_SPLIT16WHOLE;  // measuring builds only
#else
constexpr int kSplit16DivWhole = 16384;
#endif
#ifdef RT_EXP_S64LONE
constexpr int kSample16LoneTiles = RT_EXP_S64LONE;  // measuring builds only
#else
constexpr int kSample16LoneTiles = 40000;  // lone shards up to this many tiles: a sample per wave
#endif
// ... and a shard of that size with no other frame beside it (lpt_prepare
// overlapped_frame: a synchronous Update() frame of one rank) its slowest
// 1/1024: a 1/2 C3 shard's single frame -10.6 %, frames in flight +-0 (r04n;
// its slowest waves were whole tiles of ~190 us against a 148-us dispatch).
// One whose split tiles run as one-sample waves (<= kSample16LoneTiles: a 1/4
// shard) 1/512 since those trace with the whole wave (its slowest waves were
// then whole tiles of 120-130 us, wclk_r05p): -12.5 % and +1.4 % on two 1/4
// shares (r05q).
#ifdef RT_EXP_SPLIT16LONE
constexpr int kSplit16DivLone = RT_EXP_SPLIT16LONE;  // measuring builds only
constexpr int kSplit16DivLoneSample = RT_EXP_SPLIT16LONE;
#else
constexpr int kSplit16DivLone = 1024;
constexpr int kSplit16DivLoneSample = 512;
#endif
#ifdef RT_EXP_NOSYNCSPLIT
constexpr bool kSplitSync = false;  // measuring builds only
#else
constexpr bool kSplitSync = true;
#endif
// A frame with no other frame beside it (synchronous: Update() waits for it,
// RayTracingSetup.cs:171-199; or async frames on a single stream) has nothing to
// hide its tail behind, so whole frames of any size split their slowest 1/4096
// into sixteenth-waves too: C3 single frame -9 % (0.290 -> 0.264 ms,
// profiles/r04/abx_split) — a C3 frame's slowest wave, one tile's mirror chains,
// ran 0.32 ms against 0.24 ms for all the others (tools/wave_clock.py, r04i);
// frames in flight on several streams keep the 70,000-tile limit.
// Sky batches only for frames in flight of more than this many tiles: the
// batch waves run after the frame's render launch, and a small frame in
// flight is bound by its own latency (a 1/8 C3 share: +32 %; 1/4 −3.1 %, 1/2
// −1.5 %, whole frames −4.9 % per frame, r06d).
#ifdef RT_EXP_SKYMIN
constexpr int kSkyMinTiles = RT_EXP_SKYMIN;  // measuring builds only
#else
constexpr int kSkyMinTiles = 24000;
#endif
// Lone whole frames take sky batches too (measuring builds: -DRT_EXP_SKYLONE=1)
#ifdef RT_EXP_SKYLONE
constexpr bool kSkyLone = RT_EXP_SKYLONE != 0;
#else
constexpr bool kSkyLone = false;
#endif
#ifdef RT_EXP_LPTPERIOD
constexpr int kLptPeriod = RT_EXP_LPTPERIOD;  // measuring builds only
#else
// frames between longest-first re-sorts (one hipCUB sort ~46 us, plus the
// measuring launch's clock reads): 32 since round 5 (C3 in flight +1.9 %
// against 16, 64 +0.4 %: r06p)
constexpr int kLptPeriod = 32;
#endif
// rt_render's host-output pipeline: row slabs alternating over two streams, relative row counts
// kSlabsCopyBound when the PCIe copy is the longer part (float RGBA: 33 MB at 1080p, 0.59 ms against
// a 0.29 ms frame — small slabs first so the copy starts early, then slabs the render keeps ahead
// of); measured best of 9 weight vectors on C3 (tools/exp/e2e_weights.py, profiles/r03_e2e/).
// Render-bound formats (RGBA8 / RGBA16F: an 8-MB copy against a 0.24-ms frame) go in one piece
// since round 5: every slab ends in its own slowest tiles, and with the one-sample and whole-frame
// splits a lone frame's tail is short — RGBA8 0.497 -> 0.472 ms against {1, 2, 2, 1} (and 2 / 3
// slabs 0.50-0.52; tools/exp/e2e_ab.sh, profiles/r05/r06g/).  Frames under kSlabMinFrame go in
// one piece too.
constexpr double kSlabsCopyBound[] = {1, 2, 2, 3, 3, 4};
constexpr size_t kSlabMinFrame = (size_t)2 << 20;
constexpr int kMaxSlabs = 16;  // slab count range (RT_EXP_SLAB_WEIGHTS measuring builds)

// Enqueues the sum of the sharded ray/test counters into ctx->h_counts (read
// after the stream's synchronisation by read_folded).
int fold_counters(rt_ctx *ctx, hipStream_t stream) {
    HIP_OR_FAIL(ctx, rtk::launch_fold_counters(ctx->d_counters, ctx->h_counts, stream));
    return RT_OK;
}

void read_folded(const rt_ctx *ctx, unsigned long long counts[rtd::kCounterWords]) {
    const volatile unsigned long long *h = ctx->h_counts;
    for (int w = 0; w < rtd::kCounterWords; ++w) counts[w] = h[w];
}

// Sums the sharded ray/test counters (the counters' frames must have ended).
int read_counters(rt_ctx *ctx, unsigned long long counts[rtd::kCounterWords]) {
    int st = fold_counters(ctx, ctx->stream);
    if (st) return st;
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    read_folded(ctx, counts);
    return RT_OK;
}

void fill_stats(rt_stats *stats, const unsigned long long counts[rtd::kCounterWords], double kernel_ms,
                double total_ms) {
    stats->primary_rays = counts[0];
    stats->shadow_rays = counts[1];
    stats->reflection_rays = counts[2];
    stats->box_tests = counts[3];
    stats->triangle_tests = counts[4];
    stats->sphere_tests = counts[5];
    stats->shading_fetches = counts[6];
    stats->primary_scene_misses = counts[7];
    stats->shadow_rays_moot = counts[8];
    stats->kernel_ms = kernel_ms;
    stats->total_ms = total_ms;
}

// Folds the counters and device time of pending RT_FLAG_ASYNC frames into the
// context's accumulator (for rt_finish); waits for the stream.
int settle_async(rt_ctx *ctx) {
    if (ctx->async_frames == 0) return RT_OK;
    // the pending frames may sit on several streams (rt_set_stream between them)
    HIP_WAIT(ctx, hipDeviceSynchronize());
    unsigned long long counts[rtd::kCounterWords];
    int st = read_counters(ctx, counts);
    if (st) return st;
    for (int w = 0; w < rtd::kCounterWords; ++w) ctx->async_acc[w] += counts[w];
    // the frames since ev_a0 may have run on several streams: their device
    // time ends with the last of the streams' final frames
    float ms = 0.0f;
    for (auto &se : ctx->async_end) {
        if (!se.first) continue;
        float m = 0.0f;
        HIP_OR_FAIL(ctx, hipEventElapsedTime(&m, ctx->ev_a0, se.second));
        ms = std::max(ms, m);
        se.first = nullptr;  // the event object is kept for reuse
    }
    ctx->async_ms += ms;
    ctx->async_frames = 0;
    return RT_OK;
}

// Records the end of an RT_FLAG_ASYNC frame on the context's current stream.
int record_async_end(rt_ctx *ctx) {
    hipEvent_t ev = nullptr;
    for (auto &se : ctx->async_end)
        if (se.first == ctx->stream) ev = se.second;
    if (!ev) {
        for (auto &se : ctx->async_end)
            if (!se.first && !ev) {
                se.first = ctx->stream;
                ev = se.second;
            }
    }
    if (!ev) {
        HIP_OR_FAIL(ctx, hipEventCreate(&ev));
        ctx->async_end.emplace_back(ctx->stream, ev);
    }
    HIP_OR_FAIL(ctx, hipEventRecord(ev, ctx->stream));
    return RT_OK;
}

// True when this frame may run beside another of the context's frames: an
// RT_FLAG_ASYNC frame while a frame enqueued on another stream is pending
// (since the last rt_finish), whose tiles then fill the GPU during this
// frame's tail — or the first async frame after an rt_finish when the async
// frame before it ran on another stream: a caller that cycles its frames over
// several streams enqueues the others right behind it (bench.py's timed
// frames after its warm-up: as a lone frame that first frame ran the split
// instance without sky batches, 2.0 ms instead of 0.68 beside the others, and
// held its stream a frame behind for the rest of a 20-frame window, r07f).
// A frame with nothing beside it (synchronous, or async frames on one
// stream) is its own critical path and splits its slowest tiles.
static bool overlapped_frame(const rt_ctx *ctx, const rt_render_params *prm) {
    if ((prm->flags & RT_FLAG_ASYNC) == 0) return false;
    for (const auto &se : ctx->async_end)
        if (se.first && se.first != ctx->stream) return true;
    return ctx->async_frames == 0 && ctx->last_async_stream && ctx->last_async_stream != ctx->stream;
}

// One-sample waves in this frame's band.  The bands of a multi-device frame
// (rt_group.cpp group_frame) take them too since round 5: round 4 had kept
// them out after two stalled GPU-suite runs in the 8-member group tests
// (r04s, r04an; cause not found then).  Round 5 re-ran that configuration —
// four whole GPU suites and 230 stall-probe rounds (tools/stall_probe.py,
// about 5,000 group contexts) — with no stall and bit-identical frames, after
// fixing the lane stack of the 5-wave instances (traverse() had dropped its
// LDS depth); tests/conftest.py's watchdog and rt_debug_read
// RT_DEBUG_HOST_WAITS now name the blocking call should a stall recur.
// rt_debug_set(RT_DEBUG_GROUP_SAMPLE_WAVES, 0) keeps a context's group bands
// on one-pixel waves.
static bool group_sample_waves(const rt_ctx *ctx) { return !ctx->in_group_frame || ctx->debug_group_sample_waves; }

// Longest-first dispatch of a megakernel launch: picks the state of
// (stream, slab), points F at the last measured order and decides whether
// this launch measures costs (the caller sorts them after the launch).
int lpt_prepare(rt_ctx *ctx, rtd::FrameDev &F, const rt_render_params *prm, bool mega, bool count, int slab,
                LptSlot *&ls, bool &lpt_sort) {
    ls = nullptr;
    lpt_sort = false;
    ctx->last_lpt.clear();
    F.tile_order = nullptr;
    F.tile_cost = nullptr;
    F.wave_counts = nullptr;
    // (a counting launch measures tests, not costs: its per-lane walk is not the
    // frame a longest-first order is for, and it never answers a tile as sky)
    if (!mega || count || (prm->flags & RT_FLAG_ROW_ORDER) != 0 || F.num_tiles <= 0) return RT_OK;
    // a batch launch (rt_render_device_batch): its 6-wave instances split tiles
    // into quarter- and one-pixel waves, never one-sample waves
    const bool batch = slab >= kBatchSlab;
    for (LptSlot &l : ctx->lpt)
        if (l.used && l.stream == ctx->stream && l.slab == slab) ls = &l;
    if (!ls)
        for (LptSlot &l : ctx->lpt)
            if (!l.used && !ls) {
                ls = &l;
                ls->used = true;
                ls->stream = ctx->stream;
                ls->slab = slab;
            }
    F.in_flight = overlapped_frame(ctx, prm) ? 1 : 0;
    if (!ls) return RT_OK;  // more (stream, slab) pairs than slots: row-major order
    const long long key = ((long long)F.num_tiles << 32) ^ ((long long)F.tiles_x << 20) ^ ((long long)F.spp << 12) ^
                          ((long long)F.band_count << 6) ^ F.band_index ^ ((long long)F.row0 << 44);
    if (key != ls->key) {
        const size_t n = (size_t)F.num_tiles;
        HIP_OR_FAIL(ctx, ensure(ctx, ls->cost, n * 4));
        HIP_OR_FAIL(ctx, ensure(ctx, ls->cost_sorted, n * 4));
        HIP_OR_FAIL(ctx, ensure(ctx, ls->order, n * 4));
        HIP_OR_FAIL(ctx, ensure(ctx, ls->scratch, rtk::tile_sort_scratch_bytes(F.num_tiles)));
        HIP_OR_FAIL(ctx, ensure(ctx, ls->iota, n * 4));
        HIP_OR_FAIL(ctx, rtk::launch_iota((int *)ls->iota.p, F.num_tiles, ctx->stream));
        ls->key = key;
        ls->valid = false;
        ls->sky_tail = 0;
        ls->sky_pending = ls->sky_known = false;  // (a count still in flight is for the old layout)
    }
    // the sky tail of the last sort, once its count has reached the host (a
    // plain read of host memory: the count arrives tagged with its sort)
    if (ls->sky_pending) {
        const unsigned long long v = *(volatile unsigned long long *)ls->sky_host;
        if ((unsigned)(v >> 32) == ls->sky_seq) {
            ls->sky_tail = std::max(0, std::min(F.num_tiles, F.num_tiles - (int)(unsigned)v));
            ls->sky_pending = false;
        }
    }
    if (ls->scene != ctx->scene_version) {
        // a new or updated scene (rt_update_mesh_transforms every Update): the
        // last order stays a valid permutation of the tiles and, animation being
        // temporally coherent, a good one — keep dispatching by it and keep the
        // re-sort period (re-sorting after every update cost ~55 us a frame)
        ls->scene = ctx->scene_version;
    }
    if (!ls->valid) ls->frames = 0;
    F.tile_order = ls->valid ? (const int *)ls->order.p : nullptr;
    // costs are measured and re-sorted every kLptPeriod frames (the sort
    // costs more than a small frame's tail)
    lpt_sort = !ls->valid || ls->frames % kLptPeriod == 0;
    F.tile_cost = lpt_sort ? (unsigned *)ls->cost.p : nullptr;
    ++ls->frames;
    // the most expensive tiles of the last measurement are split into
    // quarter-waves (a frame's time is bounded below by its slowest wave);
    // render_kernel only: 16 lanes must hold whole pixels
    const bool levels = (ctx->S.bvh4 && F.spp >= 16) || F.max_bounces > rtd::kMaxBounces;  // (or deep: no splits)
    if (F.tile_order && !count && !levels && kSplitDiv > 0 && 16 % F.spp == 0 && F.num_tiles <= kSplitMaxTiles) {
        F.split_tiles = std::max(1, F.num_tiles / kSplitDiv);
        // sixteenth-waves (4 lanes) must hold whole pixels too
        if (kSplit16Div > 0 && 4 % F.spp == 0) {
            // a lone shard's (one-sample waves, below) more (kSplit16DivSample)
            const bool sample_waves = F.spp == 4 && !overlapped_frame(ctx, prm) && group_sample_waves(ctx) && !batch;
            const int div = sample_waves ? kSplit16DivSample : kSplit16Div;
            F.split16_tiles = std::min(F.split_tiles, std::max(1, F.num_tiles / div));
            F.split_tiles -= F.split16_tiles;
        }
    } else if (F.tile_order && !count && !levels && kSplit16DivLarge > 0 && 4 % F.spp == 0 &&
               (F.num_tiles <= kSplit16MaxTiles || (kSplitSync && !overlapped_frame(ctx, prm)))) {
        const bool lone_shard = F.num_tiles <= kSplit16MaxTiles && !overlapped_frame(ctx, prm);
        // (one-sample waves below: kSplit16DivLoneSample)
        const bool sample_waves =
            lone_shard && F.spp == 4 && F.num_tiles <= kSample16LoneTiles && group_sample_waves(ctx) && !batch;
        const int div = sample_waves ? kSplit16DivLoneSample
                        : lone_shard ? kSplit16DivLone
                        : F.num_tiles > kSplit16MaxTiles ? kSplit16DivWhole : kSplit16DivLarge;
        F.split16_tiles = std::max(1, F.num_tiles / div);
    }
    // the split-tile instance's shadow occluder hints (packet.h packet_trace
    // HINT): leaf refs of the tree they were recorded on, so cleared whenever
    // the scene changed (another tree's refs may lie outside this one's arrays)
    if (!count && !levels && (F.split_tiles > 0 || F.split16_tiles > 0)) {
        const size_t hb = (size_t)F.num_tiles * rtd::kHintLights * sizeof(int);
        bool clear = ls->hints_scene != ctx->scene_version || ls->hints_key != key;
        if (hb > ls->hints.cap) {
            HIP_OR_FAIL(ctx, ensure(ctx, ls->hints, hb));
            clear = true;
        }
        if (clear) HIP_OR_FAIL(ctx, hipMemsetAsync(ls->hints.p, 0, hb, ctx->stream));
        ls->hints_scene = ctx->scene_version;
        ls->hints_key = key;
        F.shadow_hint = (int *)ls->hints.p;
    }
    // In small shards the finely split tiles go one step further, to a sample
    // per wave (F.s16_shift 0; the shard instance sums each pixel's four
    // samples when the last arrives): a pixel's four samples no longer wait for
    // each other's divergent mirror chains.  Lone frames only (nothing beside
    // them hides their slowest chain): a 1/8 C3 shard's single frame -20 %, a
    // 1/4 shard's -15 %; a lone 1/2 shard +5 %, whole frames +6 %; with four
    // frames in flight a 1/8 shard's throughput is -3 % to +-0 (r04r, r04ag,
    // r04ai, 200-frame runs alternated on one box).  The bands of a multi-device
    // frame too, unless rt_debug_set(RT_DEBUG_GROUP_SAMPLE_WAVES, 0)
    // (group_sample_waves above).
    if (F.split16_tiles > 0 && !count && !levels && F.spp == 4 && F.num_tiles <= rtk::kShardTilesMax &&
        F.num_tiles <= kSample16LoneTiles && !overlapped_frame(ctx, prm) && group_sample_waves(ctx) && !batch) {
        F.s16_shift = 0;
        const size_t sb = (size_t)F.split16_tiles * rtd::kWaveSize * 4 * sizeof(float);
        const size_t cb = (size_t)F.split16_tiles * (rtd::kWaveSize / 4) * sizeof(int);
        HIP_OR_FAIL(ctx, ensure(ctx, ls->split_samples, sb));
        if (cb > ls->split_count.cap) {  // counts start at 0; the fourth arrival resets its pixel's
            HIP_OR_FAIL(ctx, ensure(ctx, ls->split_count, cb));
            HIP_OR_FAIL(ctx, hipMemsetAsync(ls->split_count.p, 0, ls->split_count.cap, ctx->stream));
        }
        F.split_samples = (float *)ls->split_samples.p;
        F.split_count = (int *)ls->split_count.p;
    }
    // The sorted order ends with the tiles the last measurement found to be
    // sky (cost key 0, row order): with other frames in flight beside this
    // one, sky_batch_kernel takes them rtk::kSkyBatch a wave after
    // render_kernel, together with the launch's tallies (C3 frames in flight
    // -4.9 % per frame, r06d; a lone frame, whose critical path the batches
    // lengthen, +0.5 % C3, +5 % a 1/8 shard: abx_r05t).  Only the grids depend on this count (a stale one costs time,
    // not pixels: a batch renders any tile that is not sky in full).
    if (F.tile_order && !count && !levels && rtk::kSkyBatch > 1 && F.num_tiles > kSkyMinTiles &&
        (overlapped_frame(ctx, prm) || (kSkyLone && F.num_tiles > rtk::kShardTilesMax)))
        // (render_kernel keeps one wave at least: its launch and tallies stay, an all-sky view included)
        F.sky_batch_tiles = std::max(0, std::min(ls->sky_tail, F.num_tiles - F.split_tiles - F.split16_tiles - 1));
    {
        char b[160];
        snprintf(b, sizeof b, " lpt: frame=%lld sky_tail=%d known=%d pending=%d overlapped=%d sky_waits=%lld",
                 ls->frames, ls->sky_tail, (int)ls->sky_known, (int)ls->sky_pending, (int)overlapped_frame(ctx, prm),
                 ctx->sky_waits);
        ctx->last_lpt = b;
    }
    if (levels && !(F.max_bounces > rtd::kMaxBounces)) {
        // the levels kernel dispatches XCD-aware stripes (trace_levels.hip)
        // in row order, without splits.  Its 16-spp instance (the one with
        // the sky test) measures which tiles are sky, and whole frames in
        // flight leave those to sky_batch_kernel: its positions are then the
        // measured non-sky tiles, longest first (trace_levels.hip kLvRowKeys:
        // or in row order) (C4 all-sky frames cost 0.955 ms in flight as a
        // wave per tile; skycost, r05z).
        if (F.spp == 16 && rtk::kSkyBatch > 1) {
            if (F.tile_order && !count && overlapped_frame(ctx, prm))
                F.sky_batch_tiles = std::max(0, std::min(ls->sky_tail, F.num_tiles - 1));
            if (F.sky_batch_tiles == 0) F.tile_order = nullptr;  // plain stripes
        } else {
            F.tile_order = nullptr;
            F.tile_cost = nullptr;
            lpt_sort = false;
        }
    }
    // render_kernel's ray tallies: one plain store per wave into this slot's
    // buffer, reduced after the launch on the same stream (an atomic per wave
    // holds the wave's slot for its round trip: C2 -13 %, C3 -4 %)
    if (!count) {  // render_kernel and render_levels_kernel
        const size_t bytes = (size_t)rtk::render_mega_waves(F) * sizeof(uint4);
        if (bytes > ls->wave_counts.cap) {  // a new buffer carries no launch's tag
            HIP_OR_FAIL(ctx, ensure(ctx, ls->wave_counts, bytes));
            HIP_OR_FAIL(ctx, hipMemsetAsync(ls->wave_counts.p, 0, ls->wave_counts.cap, ctx->stream));
        }
        F.wave_counts = (uint4 *)ls->wave_counts.p;
        if (++ctx->count_tag == 0) ++ctx->count_tag;
        F.count_tag = ctx->count_tag;
    }
#ifdef RT_EXP_PERSIST
    // measuring builds: whole frames' non-split launches as resident waves
    if (!count && !levels && F.split_tiles == 0 && F.split16_tiles == 0 && F.num_tiles > kSplit16MaxTiles) {
        HIP_OR_FAIL(ctx, ensure(ctx, ls->persist_ctr, 8 * 16 * sizeof(int)));
        HIP_OR_FAIL(ctx, hipMemsetAsync(ls->persist_ctr.p, 0, 8 * 16 * sizeof(int), ctx->stream));
        F.persist_ctr = (int *)ls->persist_ctr.p;
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
        F.persist_waves = (cus > 0 ? cus : 256) * 4 * RT_EXP_PERSIST;  // RT_EXP_PERSIST waves per SIMD
    }
#endif
    // measuring builds (rt_debug_set RT_DEBUG_WAVE_CLOCKS): the launch's per-wave clocks
    if (rtk::kWaveClockBuild && ctx->debug_wave_clock && !count && !levels) {
        const size_t bytes = (size_t)rtk::render_mega_waves(F) * sizeof(uint4);
        HIP_OR_FAIL(ctx, ensure(ctx, ctx->wave_clock, bytes));
        HIP_OR_FAIL(ctx, hipMemsetAsync(ctx->wave_clock.p, 0, bytes, ctx->stream));
        F.wave_clock = (uint4 *)ctx->wave_clock.p;
        ctx->wave_clock_bytes = (int64_t)bytes;
    }
    return RT_OK;
}

// Whether a frame like F (same layout, same overlap) takes sky batches, i.e.
// whether the sky tail of F's order is worth a host wait (lpt_prepare's rules:
// megakernel frames in flight of more than kSkyMinTiles tiles, 16-spp levels
// frames in flight).  Lone frames, small shares and rt_render's row slabs
// never use the tail, so their first sort does not wait for its count.
static bool sky_tail_usable(const rt_ctx *ctx, const rtd::FrameDev &F) {
    if (rtk::kSkyBatch <= 1 || F.max_bounces > rtd::kMaxBounces) return false;
    if (ctx->S.bvh4 && F.spp >= 16) return F.spp == 16 && F.in_flight;
    return F.num_tiles > kSkyMinTiles && (F.in_flight || (kSkyLone && F.num_tiles > rtk::kShardTilesMax));
}

int lpt_sort_now(rt_ctx *ctx, const rtd::FrameDev &F, LptSlot *ls) {
    HIP_OR_FAIL(ctx, rtk::sort_tiles_by_cost((const unsigned *)ls->cost.p, (unsigned *)ls->cost_sorted.p,
                                             (const int *)ls->iota.p, (int *)ls->order.p, F.num_tiles,
                                             ls->scratch.p, ls->scratch.cap, ctx->stream));
    ls->valid = true;
    if (rtk::kSkyBatch > 1) {
        if (!ls->sky_host)
            HIP_OR_FAIL(ctx, hipHostMalloc((void **)&ls->sky_host, sizeof(unsigned long long), hipHostMallocDefault));
        unsigned long long *dev = nullptr;
        HIP_OR_FAIL(ctx, hipHostGetDevicePointer((void **)&dev, ls->sky_host, 0));
        HIP_OR_FAIL(ctx, rtk::launch_sky_count((const unsigned *)ls->cost_sorted.p, F.num_tiles, ++ls->sky_seq, dev,
                                               ctx->stream));
        ls->sky_pending = true;
        if (!ls->sky_known && sky_tail_usable(ctx, F)) {
            // the slot's first order that a frame in flight can use: wait for
            // its count once (frames in flight run far ahead of the device, so
            // a lagged count of the first sort would arrive only after the
            // frames that need it); other frames read it later, untagged
            // counts are never used (lpt_prepare)
            ++ctx->sky_waits;
            if (!ls->sky_ev) HIP_OR_FAIL(ctx, hipEventCreateWithFlags(&ls->sky_ev, hipEventDisableTiming));
            HIP_OR_FAIL(ctx, hipEventRecord(ls->sky_ev, ctx->stream));
            HIP_WAIT(ctx, hipEventSynchronize(ls->sky_ev));
            const unsigned long long v = *(volatile unsigned long long *)ls->sky_host;
            if ((unsigned)(v >> 32) == ls->sky_seq) {
                ls->sky_tail = std::max(0, std::min(F.num_tiles, F.num_tiles - (int)(unsigned)v));
                ls->sky_pending = false;
            }
            ls->sky_known = true;
        }
    }
    return RT_OK;
}

// The render path a frame takes.
struct Path {
    bool count, packet, wavefront, mega;
};

Path frame_path(const rt_ctx *ctx, const rt_render_params *prm) {
    Path p;
    p.count = (prm->flags & RT_FLAG_COUNT_TESTS) != 0;
    // MaxReflectionBounces beyond the fold stack: only the megakernel's
    // deep-chain instance folds unbounded chains
    const bool deep = prm->max_reflection_bounces > rtd::kMaxBounces;
    p.packet = !deep && (prm->flags & RT_FLAG_PACKET) != 0 && ctx->S.bvh4;  // packets walk 4-wide nodes
    p.wavefront = !deep && !p.packet && (prm->flags & RT_FLAG_WAVEFRONT) != 0;
    p.mega = !p.packet && !p.wavefront;  // default
    return p;
}

// The frames of a batch launch (batch_frame: whole frames of one layout, one
// launch; F is its head).  The dispatch fields lpt_prepare set on the head
// are the batch's: every frame block carries them, with its own camera
// constants and output.
static void fill_batch(const rtd::FrameDev &H, const BatchIn &bi, rtd::FrameBatch &B) {
    std::memset(&B, 0, sizeof B);
    B.frames = bi.n;
    B.frame_tiles = bi.frames[0].num_tiles;
    B.frame_tiles_magic = B.frame_tiles <= 1 ? 0xffffffffu : (unsigned)((1ull << 32) / (unsigned long long)B.frame_tiles);
    for (int i = 0; i < bi.n; ++i) {
        rtd::FrameDev &f = B.f[i];
        f = bi.frames[i];
        f.out = (char *)H.out + (size_t)i * bi.stride;
        f.counters = H.counters;
        f.num_tiles = H.num_tiles;
        f.tile_order = H.tile_order;
        f.tile_cost = H.tile_cost;
        f.split16_tiles = H.split16_tiles;
        f.split_tiles = H.split_tiles;
        f.sky_batch_tiles = H.sky_batch_tiles;
        f.s16_shift = H.s16_shift;
        f.split_samples = H.split_samples;
        f.split_count = H.split_count;
        f.shadow_hint = nullptr;  // (the batch instances take no occluder hints)
        f.wave_counts = H.wave_counts;
        f.count_tag = H.count_tag;
        f.in_flight = H.in_flight;
        f.wave_clock = H.wave_clock;
    }
}

// Enqueues the trace launch(es) of F on the context's stream (bi: F is the
// head of a batch launch).
int launch_frame(rt_ctx *ctx, rtd::FrameDev &F, const Path &P, const rtw::Args &A, int chunk_tiles,
                 const BatchIn *bi) {
    if (bi) {
        static thread_local rtd::FrameBatch B;  // (3.3 KB: off the stack)
        fill_batch(F, *bi, B);
        const char *inst = nullptr;
        HIP_OR_FAIL(ctx, rtk::launch_render_batch(ctx->S, B, ctx->stream, &inst));
        if (inst) {
            char b[256];
            snprintf(b, sizeof b, "%s frames=%d tiles=%d split16=%d split=%d s16_shift=%d rows=%d band=%d/%d sky=%d",
                     inst, bi->n, F.num_tiles, F.split16_tiles, F.split_tiles, F.s16_shift, F.local_rows, F.band_index,
                     F.band_count, F.sky_batch_tiles);
            ctx->last_launch = b;
            ctx->last_launch += ctx->last_lpt;
        }
        return RT_OK;
    }
    if (P.packet)
        HIP_OR_FAIL(ctx, rtk::launch_render_packet(ctx->S, F, P.count, ctx->stream));
    else if (P.mega) {
        const char *inst = nullptr;
        HIP_OR_FAIL(ctx, rtk::launch_render_mega(ctx->S, F, P.count, ctx->stream, &inst));
        if (inst) {  // rt_debug_read RT_DEBUG_LAST_LAUNCH
            char b[256];
            snprintf(b, sizeof b, "%s tiles=%d split16=%d split=%d s16_shift=%d rows=%d band=%d/%d sky=%d", inst,
                     F.num_tiles, F.split16_tiles, F.split_tiles, F.s16_shift, F.local_rows, F.band_index,
                     F.band_count, F.sky_batch_tiles);
            ctx->last_launch = b;
            ctx->last_launch += ctx->last_lpt;
        }
    }
    else if (P.wavefront && F.num_tiles > 0)
        HIP_OR_FAIL(ctx, rtk::launch_render_wavefront(ctx->S, F, A, chunk_tiles, P.count, ctx->stream));
    return RT_OK;
}

bool batch_launchable(const rt_ctx *ctx, const rtd::FrameDev &F, const rt_render_params *prm, int n) {
    const Path P = frame_path(ctx, prm);
    return n > 1 && n <= rtd::kMaxBatch && P.mega && !P.count && F.spp == 4 && F.tile_w == 4 && F.tile_h == 4 &&
           F.max_bounces <= rtd::kMaxBounces && F.num_tiles > 0 && (long long)F.num_tiles * n < (1ll << 30);
}

int run_frame(rt_ctx *ctx, rtd::FrameDev &F, const rt_render_params *prm, void *d_out, rt_stats *stats,
              std::chrono::steady_clock::time_point t_start, void *host_out, size_t out_bytes, const BatchIn *bi) {
    Range range(bi ? "rt_frame_batch" : "rt_frame");
    F.out = d_out;
    F.counters = ctx->d_counters;
    if (bi) {
        // the batch's head: its tiles are every frame's (one index space)
        if (host_out) return fail(ctx, RT_E_INVALID, "a batch renders into device memory");
        F.num_tiles = bi->frames[0].num_tiles * bi->n;
    }
    const Path P = frame_path(ctx, prm);
    const bool async = (prm->flags & RT_FLAG_ASYNC) != 0;
    if (async && host_out) return fail(ctx, RT_E_INVALID, "RT_FLAG_ASYNC needs a device output (rt_render_device)");
    if (!async) {
        int st = settle_async(ctx);
        if (st) return st;
    }
    int chunk_tiles = 0;
    rtw::Args A{};
    if (P.wavefront && F.num_tiles > 0) {
        int st = prepare_wavefront(ctx, F, chunk_tiles, A);
        if (st) return st;
    }
    // rt_render into a host Color[]: the frame in row slabs, each copied to the
    // host while the next ones render (the PCIe copy is the longer part) —
    // copy-bound formats (float RGBA / RGB) of 2 MB or more; the others go
    // in one piece, copied by this thread right behind the launch on the
    // same stream (no copier hand-off)
    const bool copy_bound = F.out_format == rtd::kOutFloat4 || F.out_format == rtd::kOutRGB32F;
    bool slabs = host_out && out_bytes && F.band_count == 1 && !P.wavefront && copy_bound && out_bytes >= kSlabMinFrame;
#ifdef RT_EXP_SLAB_WEIGHTS
    slabs = host_out && out_bytes && F.band_count == 1 && !P.wavefront;  // measuring builds: the weights below
#endif
    struct Launch {
        rtd::FrameDev F;
        LptSlot *ls;
        bool sort;
        hipStream_t stream;
        int r0, r1;
    };
    std::vector<Launch> launches;
    const hipStream_t base = ctx->stream;
    struct Restore {
        rt_ctx *c;
        hipStream_t s;
        ~Restore() { c->stream = s; }
    } restore{ctx, base};
    int row_bytes = 0;
    // every launch's longest-first state first (its first use allocates):
    // outside the timed region, which covers device work only
    if (slabs) {
        row_bytes = (int)(out_bytes / (size_t)std::max(1, F.local_rows));
        double wts[kMaxSlabs];
        for (int k = 0; k < kMaxSlabs; ++k) wts[k] = 1.0;
        int nslab = out_bytes < kSlabMinFrame || !copy_bound ? 1 : 6;
        if (nslab > 1)
            for (int k = 0; k < nslab; ++k) wts[k] = kSlabsCopyBound[k];
#ifdef RT_EXP_SLAB_WEIGHTS
        {  // measuring builds: -DRT_EXP_SLAB_WEIGHTS=1,1,2,4,8 (relative slab rows)
            constexpr double w[] = {RT_EXP_SLAB_WEIGHTS};
            nslab = std::min(kMaxSlabs, (int)(sizeof w / sizeof w[0]));
            for (int k = 0; k < nslab; ++k) wts[k] = w[k];
        }
#endif
        double cum[kMaxSlabs + 1];
        cum[0] = 0.0;
        for (int k = 0; k < nslab; ++k) cum[k + 1] = cum[k] + wts[k];
        // slab boundaries on whole tile rows
        const int tile_rows = (F.local_rows + F.tile_h - 1) / F.tile_h;
        auto bound = [&](int k) {
            return std::min(F.local_rows, (int)std::lround((double)tile_rows * cum[k] / cum[nslab]) * F.tile_h);
        };
        if (!ctx->copy_stream) HIP_OR_FAIL(ctx, hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
        while ((int)ctx->slab_done.size() < nslab) {
            hipEvent_t e;
            HIP_OR_FAIL(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ctx->slab_done.push_back(e);
        }
        // slabs alternate between two streams, so a slab's tail overlaps the
        // next slab instead of idling the GPU
        if (!ctx->slab_stream2) HIP_OR_FAIL(ctx, hipStreamCreateWithFlags(&ctx->slab_stream2, hipStreamNonBlocking));
        for (int k = 0; k < nslab; ++k) {
            Launch L{};
            L.stream = ctx->stream = (k & 1) ? ctx->slab_stream2 : base;
            L.r0 = bound(k);
            L.r1 = k + 1 == nslab ? F.local_rows : bound(k + 1);
            L.F = F;
            L.F.row0 = L.r0;
            L.F.local_rows = L.r1 - L.r0;
            L.F.num_tiles = L.F.res_x > 0 ? L.F.tiles_x * ((L.F.local_rows + L.F.tile_h - 1) / L.F.tile_h) : 0;
            L.F.out = (char *)d_out + (size_t)L.r0 * row_bytes;
            int st = lpt_prepare(ctx, L.F, prm, P.mega, P.count, k, L.ls, L.sort);
            if (st) return st;
            launches.push_back(L);
        }
        ctx->stream = base;
    } else {
        // megakernel frames dispatch a previous frame's most expensive tiles
        // first (a frame's tail is its slowest tiles); the order is kept per stream
        Launch L{};
        L.F = F;
        L.stream = base;
        // (a batch keeps its order apart from single frames on the same stream: slot kBatchSlab + frames)
        int st = lpt_prepare(ctx, L.F, prm, P.mega, P.count, bi ? kBatchSlab + bi->n : 0, L.ls, L.sort);
        if (st) return st;
        launches.push_back(L);
    }
    bool sync_done = false;  // the frame's work (and its counters' fold) has completed
    const size_t ctr_bytes = rtd::kCounterSlots * rtd::kCounterWords * sizeof(unsigned long long);
    if (!async || ctx->async_frames == 0) {
        // async frames share one set of counters until rt_finish / the next synchronous frame
        HIP_OR_FAIL(ctx, hipMemsetAsync(ctx->d_counters, 0, ctr_bytes, ctx->stream));
        HIP_OR_FAIL(ctx, hipEventRecord(async ? ctx->ev_a0 : ctx->ev0, ctx->stream));
    } else {
        // a later async frame may be on another stream (rt_set_stream between
        // frames): it must not count before the counters were zeroed
        HIP_OR_FAIL(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_a0, 0));
    }
    if (slabs) {
        const int nslab = (int)launches.size();
        HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev_slab0, base));
        HIP_OR_FAIL(ctx, hipStreamWaitEvent(ctx->slab_stream2, ctx->ev_slab0, 0));
        if (!ctx->copier.th.joinable()) ctx->copier.start(ctx->device, ctx->copy_stream);
        // once a copy is posted, every return waits for the posted copies:
        // the copier must never write into the caller's buffer after
        // rt_render has returned (an error return included), nor leave an
        // error behind for the next frame's wait
        struct Drain {
            Copier *c = nullptr;
            ~Drain() {
                if (c) (void)c->wait();
            }
        } drain;
        for (int k = 0; k < nslab; ++k) {
            ctx->stream = launches[k].stream;
            if (k == ctx->debug_fail_slab)  // rt_debug_set(RT_DEBUG_FAIL_SLAB): tests only
                return fail(ctx, RT_E_INTERNAL, "injected failure before slab %d (RT_DEBUG_FAIL_SLAB)", k);
            int st = launch_frame(ctx, launches[k].F, P, A, chunk_tiles, nullptr);
            if (st) return st;
            HIP_OR_FAIL(ctx, hipEventRecord(ctx->slab_done[k], ctx->stream));
            // the copier thread copies slab k once its launch has ended, while
            // this thread enqueues the next launches
            const int r0 = launches[k].r0, r1 = launches[k].r1;
            if (r1 > r0) {
                ctx->copier.post({ctx->slab_done[k], (char *)host_out + (size_t)r0 * row_bytes,
                                  (const char *)d_out + (size_t)r0 * row_bytes, (size_t)(r1 - r0) * row_bytes});
                drain.c = &ctx->copier;
            }
        }
        ctx->stream = base;
        if (nslab > 1) HIP_OR_FAIL(ctx, hipStreamWaitEvent(base, ctx->slab_done[nslab - (nslab & 1 ? 2 : 1)], 0));
        HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, base));
        for (Launch &L : launches) {  // after the timed region: the order of the next frames
            if (!L.sort) continue;
            ctx->stream = L.stream;
            int st = lpt_sort_now(ctx, L.F, L.ls);
            if (st) return st;
        }
        ctx->stream = base;
        int st = fold_counters(ctx, base);  // base has waited for every launch
        if (st) return st;
        drain.c = nullptr;
        HIP_OR_FAIL(ctx, ctx->copier.wait());  // every slab is in the caller's buffer
    } else {
        Launch &L = launches[0];
        int st = launch_frame(ctx, L.F, P, A, chunk_tiles, bi);
        if (st) return st;
        if (async) {
            if (L.sort) {
                st = lpt_sort_now(ctx, L.F, L.ls);
                if (st) return st;
            }
            st = record_async_end(ctx);
            if (st) return st;
            ctx->last_async_stream = ctx->stream;
            if (ctx->async_frames++ == 0 && ctx->async_t0_set == false) {
                ctx->async_t0 = t_start;
                ctx->async_t0_set = true;
            }
            if (stats) std::memset(stats, 0, sizeof *stats);
            return RT_OK;
        }
        HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
        st = fold_counters(ctx, ctx->stream);  // (a 256-thread launch into host-mapped words)
        if (st) return st;
        if (host_out && out_bytes) {
            // the host copy right behind the launch and the counters' fold;
            // once the stream has drained up to here the frame is complete and
            // its folded counters readable — a re-sort is enqueued after that,
            // off the frame's critical path, and not awaited (the next frame on
            // the stream follows it)
            HIP_WAIT(ctx, hipMemcpyAsync(host_out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
            HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));  // (a page-locked host_out: the copy was async)
            if (L.sort) {
                st = lpt_sort_now(ctx, L.F, L.ls);
                if (st) return st;
            }
            sync_done = true;
        } else if (L.sort) {  // after the timed region: the order of the next frames
            st = lpt_sort_now(ctx, L.F, L.ls);
            if (st) return st;
        }
    }
    if (!sync_done) HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    unsigned long long counts[rtd::kCounterWords];
    read_folded(ctx, counts);
    std::memcpy(ctx->last_counts, counts, sizeof counts);
    if (stats) {
        float ms = 0.0f;
        HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        fill_stats(stats, counts, ms,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    }
    return RT_OK;
}

}  // namespace rti
