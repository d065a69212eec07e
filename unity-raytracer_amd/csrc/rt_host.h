// rt_host.h — internal host state of the C-ABI library (include/rt_mi355.h):
// the context (rt_ctx), its grow-only device buffers and the functions the
// host modules share.  Not installed; nothing here crosses the ABI.
//
// Modules: rt_abi.cpp (the extern "C" entry points), rt_scene.cpp (scene
// validation and upload, BVH builds, the top-level cut, device extraction and
// refit), rt_frame.cpp (frame constants, longest-first dispatch, launches,
// counters, rt_render's host-output slab pipeline), rt_group.cpp (contexts,
// multi-device frames, the RCCL band gather), rt_util.cpp (errors, buffers).
#pragma once

#include "../../include/rt_mi355.h"

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <string>
#include <vector>

#include <dlfcn.h>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include "bvh.h"
#include "kernels.h"
#include "lbvh.h"
#include "scene_xform.h"
#include "rt_device.h"
#include "rt_math.h"

namespace rti {

struct GrowBuf {
    void *p = nullptr;
    size_t cap = 0;
};

// Device buffers of the GPU (LBVH) build path, kept across rebuilds.
struct LbvhBufs {
    GrowBuf meshes, mesh_tris, mesh_normals, spheres, sphere_mat, loose_tris, loose_normals, loose_mat;
    GrowBuf nodes, nodes4, tris, sphs, shade, scratch;
    // device mesh extraction (scene_xform.hip): resident sources + matrices
    GrowBuf src_meshes, src_local, src_indices, src_matrices, src_world, src_aabbs, src_parts;
    GrowBuf scene_box;  // {lo[3], hi[3], pad_abs} of an animated scene (scene_xform.hip k_scene_box)
    void release() {
        GrowBuf *all[] = {&meshes, &mesh_tris, &mesh_normals, &spheres, &sphere_mat, &loose_tris, &loose_normals,
                          &loose_mat, &nodes, &nodes4, &tris, &sphs, &shade, &scratch, &src_meshes, &src_local,
                          &src_indices, &src_matrices, &src_world, &src_aabbs, &src_parts, &scene_box};
        for (GrowBuf *b : all) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
    }
};

// Longest-first dispatch state of one stream: the last measured per-tile cost
// keys, the order sorted from them, for one frame layout and scene version.
struct LptSlot {
    hipStream_t stream = nullptr;
    int slab = 0;  // rt_render row slab (0 for whole frames)
    bool used = false;
    GrowBuf cost, cost_sorted, iota, order, scratch;
    GrowBuf wave_counts;  // render_kernel's per-wave ray tallies (rtd::FrameDev::wave_counts)
    GrowBuf hints;        // render_kernel's shadow-packet occluder hints (rtd::FrameDev::shadow_hint)
    GrowBuf split_samples, split_count;  // one-sample split waves' hand-off (rtd::FrameDev::split_*)
    GrowBuf persist_ctr;                 // measuring builds (RT_EXP_PERSIST): per-XCD tile counters
    // the sorted order's sky tail (render_kernel sky batches): counted on the
    // device after each sort into host-mapped memory — awaited after the
    // slot's first sort, later ones taken once their event has fired
    unsigned long long *sky_host = nullptr;  // (sort sequence << 32) | tiles before the sky tail
    hipEvent_t sky_ev = nullptr;
    unsigned sky_seq = 0;
    bool sky_pending = false, sky_known = false;
    int sky_tail = 0;
    unsigned long long hints_scene = ~0ull;  // the scene version and layout the hints were recorded for
    long long hints_key = -1;
    long long key = -1;
    unsigned long long scene = ~0ull;
    bool valid = false;
    long long frames = 0;
    void release() {
        for (GrowBuf *b : {&cost, &cost_sorted, &iota, &order, &scratch, &wave_counts, &hints, &split_samples,
                           &split_count, &persist_ctr}) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
        if (sky_ev) (void)hipEventDestroy(sky_ev);
        if (sky_host) (void)hipHostFree(sky_host);
        sky_ev = nullptr;
        sky_host = nullptr;
        sky_pending = sky_known = false;
        sky_tail = 0;
    }
};
constexpr int kLptSlots = 16;  // streams x row slabs

// Host copy of rt_set_scene_source's base scene (the caller's arrays are not
// kept): a refitted scene's full rebuild needs it.
struct BaseCopy {
    std::vector<rt_triangle> tris;
    std::vector<rt_float3> normals;
    std::vector<rt_material> tri_mats, sph_mats;
    std::vector<rt_sphere> sphs;
    std::vector<rt_point_light> lights;
    rt_scene_desc desc{};
    void set(const rt_scene_desc &b) {
        auto cp = [](auto &v, const auto *p, int n) { v.assign(p, p + (p ? std::max(0, n) : 0)); };
        cp(tris, b.triangles, b.triangle_count);
        cp(normals, b.triangle_normals, b.triangle_count);
        cp(tri_mats, b.triangle_materials, b.triangle_count);
        cp(sphs, b.spheres, b.sphere_count);
        cp(sph_mats, b.sphere_materials, b.sphere_count);
        cp(lights, b.point_lights, b.point_light_count);
        desc = b;
        desc.triangles = tris.data();
        desc.triangle_normals = normals.data();
        desc.triangle_materials = tri_mats.data();
        desc.spheres = sphs.data();
        desc.sphere_materials = sph_mats.data();
        desc.point_lights = lights.data();
    }
};

// RT_BUILD_SAH_REFIT: the host SAH tree's topology kept across updates and
// refitted on the device (scene_xform.hip refit_tree).
// full rebuild once the tree's relative surface area grows past this: 1.05 / 1.1 / 1.25 / never gave C3
// 0.470 / 0.465 / 0.475 / 0.472 ms and C5i 1.048 / 1.028 / 1.037 / 1.320 ms per update + frame
// (tools/exp/refit_sweep.sh, profiles/r03_rebuild/refit_sweep.txt)
constexpr float kRefitRebuild = 1.1f;
struct RefitState {
    GrowBuf parent_slot, internal_children, arrivals, prim_lo, prim_hi, quality, rank_first, geom_first, loose;
    int nnodes = 0, ntri = 0, nsph = 0;
    float area_built = 0.0f;    // internal slots' half areas / the root's, after the last full build
    int rebuilds = 0;           // full rebuilds after the first (degraded refits)
    std::vector<rt_mesh> meshes;  // first triangle, count, material; AABBs of the last full build
    BaseCopy base;
    void release() {
        for (GrowBuf *b : {&parent_slot, &internal_children, &arrivals, &prim_lo, &prim_hi, &quality, &rank_first,
                           &geom_first, &loose}) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
    }
};

// State kept by rt_set_scene_source for rt_update_mesh_transforms.
struct SourceState {
    bool active = false;
    int build = RT_BUILD_LBVH_GPU;  // or RT_BUILD_SAH_REFIT
    int mesh_count = 0, vertex_total = 0, tri_total = 0, part_total = 0;
    float rest_lo[3], rest_hi[3];  // Scene.CalculateAABB over loose triangles and spheres
    rtl::LbvhInput in{};           // device inputs of the last build
    bool wide = true;
    RefitState refit;
};

struct DeviceArrays {
    void *nodes = nullptr, *nodes4 = nullptr, *leaves = nullptr, *tris = nullptr, *sphs = nullptr, *shade = nullptr,
         *mats = nullptr, *lights = nullptr, *gates = nullptr;
};

// Frame buffers of a multi-device context for one stream of device 0 (frames
// in flight on different streams never share them).
constexpr int kGroupSlots = 8;
struct GroupSlot {
    hipStream_t root_stream = nullptr;
    bool used = false;
    std::vector<hipStream_t> member_stream;  // per member (member 0: a stream of its own for the RCCL self send)
    std::vector<hipEvent_t> member_done;     // recorded on a member's stream after its band left
    std::vector<GrowBuf> member_out;         // per member: its band, on its device
    GrowBuf gather;                          // device 0: every band back to back
    hipEvent_t gather_free = nullptr;        // device 0: the last frame's bands are reassembled
};

// Host waits (rt_debug_read RT_DEBUG_HOST_WAITS): every runtime call of the
// library that can block its thread (synchronisations, copies into pageable
// host memory, frees, the copier hand-off, RCCL group ends, thread joins)
// runs inside a Wait scope, which records in its thread's slot of a fixed
// table what the thread waits for and since when.  A report of that table
// (and of the context's streams) names the call a stalled thread sits in.
class Wait {
  public:
    explicit Wait(const char *what);
    ~Wait();
    Wait(const Wait &) = delete;
    Wait &operator=(const Wait &) = delete;

  private:
    int slot_;
    const char *prev_what_;
    long long prev_since_;
};
std::string host_waits_report(rt_ctx *ctx);
// The registry of live contexts host_waits_report may read (rt_create* register
// a context, rt_destroy unregisters it before tearing it down).
void register_ctx(const rt_ctx *ctx);
void unregister_ctx(const rt_ctx *ctx);

// rt_render's host-output copies, issued from a thread of their own: a copy
// into pageable memory holds the calling thread until it is done, so the
// thread that enqueues the slab launches must not be the one that copies — the
// first slab's copy then starts as soon as that slab is rendered.
struct Copier {
    struct Job {
        hipEvent_t ready;  // the slab's launch has ended
        void *dst;
        const void *src;
        size_t bytes;
    };
    std::thread th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::deque<Job> jobs;
    int device = 0;
    hipStream_t stream = nullptr;
    bool quit = false, busy = false;
    hipError_t err = hipSuccess;

    void start(int dev, hipStream_t s) {
        device = dev;
        stream = s;
        th = std::thread([this] { run(); });
    }
    void run() {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [this] { return quit || !jobs.empty(); });
            if (jobs.empty()) return;  // quit
            const Job j = jobs.front();
            jobs.pop_front();
            busy = true;
            lk.unlock();
            // the copy stream waits for the slab on the device; a pageable
            // copy returns once it is done
            hipError_t e = hipStreamWaitEvent(stream, j.ready, 0);
            {
                const Wait w("copier: slab copy into the host frame");
                if (e == hipSuccess) e = hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess) e = hipStreamSynchronize(stream);
            }
            lk.lock();
            if (e != hipSuccess && err == hipSuccess) err = e;
            busy = false;
            if (jobs.empty()) done_cv.notify_all();
        }
    }
    void post(const Job &j) {
        {
            std::lock_guard<std::mutex> lk(mu);
            jobs.push_back(j);
        }
        cv.notify_one();
    }
    hipError_t wait() {  // every posted copy is done; returns (and clears) the first error
        const Wait w("copier.wait (posted slab copies)");
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [this] { return jobs.empty() && !busy; });
        const hipError_t e = err;
        err = hipSuccess;
        return e;
    }
    void stop() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv.notify_all();
        const Wait w("copier.stop join");
        th.join();
    }
};


// roctx ranges around the host-side phases (visible in rocprofv3
// --marker-trace).  The roctx library is resolved lazily like RCCL, so a host
// whose loader path lacks it still loads this library (ranges become no-ops).
struct Roctx {
    decltype(&roctxRangePushA) push = nullptr;
    decltype(&roctxRangePop) pop = nullptr;
};

const Roctx &roctx();


struct Range {
    explicit Range(const char *name) {
        if (roctx().push) roctx().push(name);
    }
    ~Range() {
        if (roctx().pop) roctx().pop();
    }
};

}  // namespace rti

struct rt_ctx {
    int device = -1;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    bool has_scene = false;
    rti::DeviceArrays arr;
    rtd::SceneDev S{};
    std::vector<int> mesh_rank_first;  // prefix of mesh triangle counts (rank decode)
    int mesh_tri_ranks = 0, sphere_count = 0, loose_count = 0;
    float4 *d_out = nullptr;
    size_t d_out_cap = 0;
    unsigned long long *d_counters = nullptr;
    unsigned long long *h_counts = nullptr;  // page-locked: the folded counters (fold_counters_kernel)
    // page-locked results of rt_update_mesh_transforms' one synchronisation
    struct UpdateHost {
        float box[8];  // lo[3], hi[3], pad_abs
        int binfo[4];  // lbvh_info_ptr: 2-wide depth, 4-wide nodes, 4-wide depth
        float quality[2];  // refit: internal slots' half areas, the root's
    } *h_update = nullptr;
    hipEvent_t ev_x = nullptr;  // end of the device extraction in an update
    float *d_rays = nullptr;
    int4 *d_hits = nullptr;
    size_t rays_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_slab0 = nullptr;  // rt_render's slab pipeline: the second stream starts after this point
    // RT_FLAG_ASYNC frames: pending count, accumulated counters and device time
    hipEvent_t ev_a0 = nullptr;
    int async_frames = 0;
    long long async_total_frames = 0;
    unsigned long long async_acc[rtd::kCounterWords] = {0};
    double async_ms = 0.0;
    std::chrono::steady_clock::time_point async_t0;
    bool async_t0_set = false;
    // wavefront queues (trace_wf.hip); pool_cap entries, shadow_cap shadow rays
    rtw::Counters *wf_ctr = nullptr;
    float4 *wf_ray_o = nullptr, *wf_ray_d = nullptr, *wf_col = nullptr, *wf_sh_o = nullptr, *wf_sh_d = nullptr;
    int4 *wf_hit = nullptr;
    unsigned char *wf_occ = nullptr;
    size_t pool_cap = 0, shadow_cap = 0;
    int last_bvh_depth = 0;
    rt_scene_info info{};
    rti::LbvhBufs lb;
    // longest-first tile order of megakernel frames (a previous frame's
    // per-tile cost), one state per stream the frames run on, so frames in
    // flight on different streams never read an order being rewritten
    rti::LptSlot lpt[rti::kLptSlots];
    unsigned long long scene_version = 0;
    rti::SourceState src;
    // end event of the last RT_FLAG_ASYNC frame per stream: rt_finish's device
    // time spans from the first async frame to the last of them to finish
    std::vector<std::pair<hipStream_t, hipEvent_t>> async_end;
    hipStream_t last_async_stream = nullptr;  // the stream of the last RT_FLAG_ASYNC frame (kept across rt_finish)
    // rt_render's slab pipeline: copy stream + one event per slab
    hipStream_t copy_stream = nullptr;
    rti::Copier copier;  // its thread runs only after a context's first host-output frame
    std::vector<hipEvent_t> slab_done;
    hipStream_t slab_stream2 = nullptr;  // ... odd slabs render here, even ones on the context's stream
    // multi-device context: this context is member 0 (the root, device 0 of
    // the frame); peers[i] is member i + 1, a single-device context of its own
    std::vector<rt_ctx *> peers;
    int gather = RT_GATHER_NONE;
    std::vector<ncclComm_t> comms;  // one per member (RT_GATHER_RCCL)
    rti::GroupSlot gslots[rti::kGroupSlots];
    rtd::CutTable *d_cut = nullptr;  // the 4-wide tree's top-level cut (enqueue_cut), once allocated
    bool warmed = false;  // the render kernels have run once on this device (warm_up)
    unsigned count_tag = 0;  // the last render_kernel launch's wave_counts tag
    int debug_fail_slab = -1;  // rt_debug_set(RT_DEBUG_FAIL_SLAB): rt_render fails before this row slab
    // rt_debug_set(RT_DEBUG_WAVE_CLOCKS), measuring builds: the last render_kernel launch's per-wave clocks
    bool debug_wave_clock = false;
    bool in_group_frame = false;  // rendering one band of a multi-device frame (rt_group.cpp group_frame)
    int debug_sample_wave_stack = 0;  // rt_debug_set(RT_DEBUG_SAMPLE_WAVE_STACK, n): one-sample waves' wide-step limit (testing)
    bool debug_group_sample_waves = true;  // rt_debug_set(RT_DEBUG_GROUP_SAMPLE_WAVES, 0): group bands without them
    std::atomic<bool> destroying{false};  // rt_destroy has begun (host_waits_report skips the context)
    std::string last_launch;
    std::string last_lpt;  // the longest-first slot's state of the last launch (RT_DEBUG_LAST_LAUNCH)
    long long sky_waits = 0;
    unsigned long long last_counts[rtd::kCounterWords] = {0};  // rt_debug_read RT_DEBUG_COUNTERS  // host waits for a first sort's sky-tail count (lpt_sort_now; RT_DEBUG_LAST_LAUNCH)
    rti::GrowBuf wave_clock;
    int64_t wave_clock_bytes = 0;
};

namespace rti {

extern thread_local std::string g_create_error;

// Records the message (on ctx, or for rt_last_error(NULL)) and returns status.
int fail(rt_ctx *ctx, int status, const char *fmt, ...);

#define HIP_OR_FAIL(ctx, call)                                                                   \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail((ctx), RT_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_));         \
    } while (0)


#define HIP_WAIT(ctx, call)                                                                      \
    do {                                                                                         \
        hipError_t e_;                                                                           \
        {                                                                                        \
            const rti::Wait w_(#call);                                                           \
            e_ = (call);                                                                         \
        }                                                                                        \
        if (e_ != hipSuccess)                                                                    \
            return fail((ctx), RT_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_));         \
    } while (0)

inline rtm::f3 F3(const rt_float3 &v) { return rtm::mk(v.x, v.y, v.z); }

// Grow-only device buffer (per-frame rebuilds reuse their memory).
hipError_t ensure(rt_ctx *ctx, GrowBuf &b, size_t bytes);
// The context's own device output buffer (rt_render), grow-only.
hipError_t ensure_out(rt_ctx *ctx, size_t bytes);
// Rows of one block-cyclic band's compact buffer.
int32_t band_local_rows(int32_t res_y, int32_t band_count, int32_t band_rows);

// ---- scenes (rt_scene.cpp)
float spec_threshold();
void free_scene(rt_ctx *c);
int set_scene_impl(rt_ctx *ctx, const rt_scene_desc *sc, int32_t build, bool geom_on_device,
                   std::chrono::steady_clock::time_point t_start);
int set_scene_source_one(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count,
                         int32_t build, std::chrono::steady_clock::time_point t0);
int update_mesh_transforms_one(rt_ctx *ctx, const float *local_to_world, int32_t mesh_count,
                               std::chrono::steady_clock::time_point t0);

// ---- frames (rt_frame.cpp)
int prepare_frame(rt_ctx *ctx, const rt_camera *cam, const rt_image_plane *plane, const rt_render_params *prm,
                  rtd::FrameDev &F, size_t &out_bytes);
// The frames of a batch launch (rt_render_device_batch): n frames of one
// layout, prepared from their cameras, outputs `stride` bytes apart.
struct BatchIn {
    const rtd::FrameDev *frames;
    int n;
    size_t stride;
};
// longest-first slots of batches: slab kBatchSlab + frames (apart from single frames)
constexpr int kBatchSlab = 1000;
// Whether n frames like F can go as one batch launch (4 spp megakernel frames).
bool batch_launchable(const rt_ctx *ctx, const rtd::FrameDev &F, const rt_render_params *prm, int n);
// bi: F is the head of a batch (prepared like its first frame), rendered as one launch
int run_frame(rt_ctx *ctx, rtd::FrameDev &F, const rt_render_params *prm, void *d_out, rt_stats *stats,
              std::chrono::steady_clock::time_point t_start, void *host_out, size_t out_bytes,
              const BatchIn *bi = nullptr);
void free_wavefront(rt_ctx *c);
int settle_async(rt_ctx *ctx);
void fill_stats(rt_stats *stats, const unsigned long long counts[rtd::kCounterWords], double kernel_ms,
                double total_ms);

// ---- contexts and multi-device frames (rt_group.cpp)
int create_one(int dev, rt_ctx **out);
void destroy_one(rt_ctx *ctx);
void release_group(rt_ctx *ctx);
int create_group(const int32_t *devices, int32_t n, int32_t gather, rt_ctx **out_ctx);
int take_async(rt_ctx *m, unsigned long long counts[rtd::kCounterWords], double &ms);
int group_frame(rt_ctx *ctx, const rt_camera *cam, const rt_image_plane *plane, const rt_render_params *prm,
                void *d_out, void *host_out, size_t full_bytes, rt_stats *stats,
                std::chrono::steady_clock::time_point t0);

inline int nmembers(const rt_ctx *c) { return 1 + (int)c->peers.size(); }
inline rt_ctx *member(rt_ctx *c, int i) { return i == 0 ? c : c->peers[(size_t)i - 1]; }

// The library switches devices; the caller's current device is restored on return.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// fn(member) for every member of a context, each on a host thread of its own
// when there are several (the host BVH build of a scene runs on every device
// at once); the first failure is reported on ctx.
template <typename Fn>
int for_members(rt_ctx *ctx, Fn fn) {
    const int n = nmembers(ctx);
    if (n == 1) return fn(ctx);
    std::vector<int> st((size_t)n, RT_OK);
    std::vector<std::thread> th;
    th.reserve((size_t)n);
    for (int i = 0; i < n; ++i) th.emplace_back([&, i] { st[(size_t)i] = fn(member(ctx, i)); });
    {
        const Wait w("for_members join");
        for (auto &t : th) t.join();
    }
    for (int i = 0; i < n; ++i)
        if (st[(size_t)i] != RT_OK) {
            if (i) ctx->err = "device " + std::to_string(member(ctx, i)->device) + ": " + member(ctx, i)->err;
            return st[(size_t)i];
        }
    return RT_OK;
}

}  // namespace rti
