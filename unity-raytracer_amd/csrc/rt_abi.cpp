// rt_abi.cpp — implementation of the C-ABI in include/rt_mi355.h.
//
// Host side of the MI355X trace path: validates the reference-shaped scene,
// computes Scene.CalculateAABB exactly (Scene.cs:17-41), builds the BVH,
// lays the scene out in HBM (rt_device.h) and launches the gfx950 kernels
// (trace.hip).  There is no CPU fallback: without a gfx950 device every
// entry point fails with RT_E_NO_DEVICE / RT_E_HIP.
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

namespace {

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
    long long key = -1;
    unsigned long long scene = ~0ull;
    bool valid = false;
    long long frames = 0;
    void release() {
        for (GrowBuf *b : {&cost, &cost_sorted, &iota, &order, &scratch, &wave_counts}) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
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
            if (e == hipSuccess) e = hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipStreamSynchronize(stream);
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
        th.join();
    }
};

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

// roctx ranges around the host-side phases (visible in rocprofv3
// --marker-trace).  The roctx library is resolved lazily like RCCL, so a host
// whose loader path lacks it still loads this library (ranges become no-ops).
struct Roctx {
    decltype(&roctxRangePushA) push = nullptr;
    decltype(&roctxRangePop) pop = nullptr;
};

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

struct Range {
    explicit Range(const char *name) {
        if (roctx().push) roctx().push(name);
    }
    ~Range() {
        if (roctx().pop) roctx().pop();
    }
};

}  // namespace

struct rt_ctx {
    int device = -1;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    bool has_scene = false;
    DeviceArrays arr;
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
    LbvhBufs lb;
    // longest-first tile order of megakernel frames (a previous frame's
    // per-tile cost), one state per stream the frames run on, so frames in
    // flight on different streams never read an order being rewritten
    LptSlot lpt[kLptSlots];
    unsigned long long scene_version = 0;
    SourceState src;
    // end event of the last RT_FLAG_ASYNC frame per stream: rt_finish's device
    // time spans from the first async frame to the last of them to finish
    std::vector<std::pair<hipStream_t, hipEvent_t>> async_end;
    // rt_render's slab pipeline: copy stream + one event per slab
    hipStream_t copy_stream = nullptr;
    Copier copier;  // its thread runs only after a context's first host-output frame
    std::vector<hipEvent_t> slab_done;
    hipStream_t slab_stream2 = nullptr;  // ... odd slabs render here, even ones on the context's stream
    // multi-device context: this context is member 0 (the root, device 0 of
    // the frame); peers[i] is member i + 1, a single-device context of its own
    std::vector<rt_ctx *> peers;
    int gather = RT_GATHER_NONE;
    std::vector<ncclComm_t> comms;  // one per member (RT_GATHER_RCCL)
    GroupSlot gslots[kGroupSlots];
    rtd::CutTable *d_cut = nullptr;  // the 4-wide tree's top-level cut (enqueue_cut), once allocated
    bool warmed = false;  // the render kernels have run once on this device (warm_up)
    unsigned count_tag = 0;  // the last render_kernel launch's wave_counts tag
};

namespace {

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

#define HIP_OR_FAIL(ctx, call)                                                                   \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail((ctx), RT_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_));         \
    } while (0)

void free_scene(rt_ctx *c) {
    void **ps[] = {&c->arr.nodes, &c->arr.nodes4, &c->arr.leaves, &c->arr.tris, &c->arr.sphs,
                   &c->arr.shade, &c->arr.mats,   &c->arr.lights, &c->arr.gates};
    for (void **p : ps) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    c->has_scene = false;
}

template <typename T>
hipError_t upload(void **dst, const std::vector<T> &v) {
    if (v.empty()) return hipSuccess;
    hipError_t e = hipMalloc(dst, v.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

rtm::f3 F3(const rt_float3 &v) { return rtm::mk(v.x, v.y, v.z); }

// Ordered-integer view of a float for bisection over representable values.
int32_t fkey(float f) {
    uint32_t b;
    std::memcpy(&b, &f, 4);
    return (b & 0x80000000u) ? -(int32_t)(b & 0x7fffffffu) : (int32_t)b;
}
float ffrom(int32_t k) {
    uint32_t b = k < 0 ? (0x80000000u | (uint32_t)(-k)) : (uint32_t)k;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

// The reference's specular back-face test (RayTracingSetup.cs:382-392):
//   degrees(acos(d)) > 90f,  acos = (float)System.Math.Acos((double)d),
//   degrees(x) = x * 57.29578f.
// It is monotone non-increasing in d, so it equals d < T for the smallest
// float T where it is false.  T is found here once with the host libm (the
// same double acos the CPU oracle uses) so the GPU never evaluates acos.
bool spec_backfacing(float d) { return (float)std::acos((double)d) * 57.29578f > 90.0f; }

float compute_spec_threshold() {
    int32_t lo = fkey(-1.0f), hi = fkey(1.0f);  // backfacing(lo) true, backfacing(hi) false
    while (hi - lo > 1) {
        int32_t mid = lo + (hi - lo) / 2;
        if (spec_backfacing(ffrom(mid)))
            lo = mid;
        else
            hi = mid;
    }
    return ffrom(hi);
}

float spec_threshold() {
    static const float T = compute_spec_threshold();
    return T;
}

bool mat_less(const rt_material &a, const rt_material &b) { return std::memcmp(&a, &b, sizeof a) < 0; }

rtd::DevMaterial to_dev(const rt_material &m) {
    rtd::DevMaterial d;
    d.kd_phong = make_float4(m.diffuse_reflectance.x, m.diffuse_reflectance.y, m.diffuse_reflectance.z,
                             m.phong_exponent);
    d.ka_mirror = make_float4(m.ambient_reflectance.x, m.ambient_reflectance.y, m.ambient_reflectance.z,
                              m.is_mirror ? 1.0f : 0.0f);
    d.km = make_float4(m.mirror_reflectance.x, m.mirror_reflectance.y, m.mirror_reflectance.z, 0.0f);
    // ks.w = 1: the specular term is an exact signed zero for every hit, so
    // the device may skip pow (shade.h light_term): SpecularReflectance is
    // +-0 and PhongExponent in [0, 1e6] keeps pow(cnh <= 1 + 2^-22, n) finite
    // and non-negative, hence (ks * pow) * E == (ks * 0) * E bit for bit.
    const bool no_spec = m.specular_reflectance.x == 0.0f && m.specular_reflectance.y == 0.0f &&
                         m.specular_reflectance.z == 0.0f && m.phong_exponent >= 0.0f && m.phong_exponent <= 1e6f;
    d.ks = make_float4(m.specular_reflectance.x, m.specular_reflectance.y, m.specular_reflectance.z,
                       no_spec ? 1.0f : 0.0f);
    return d;
}

int isqrt_exact(int v) {
    if (v <= 0) return -1;
    int n = 1;
    while (n * n < v) ++n;
    return n * n == v ? n : -1;
}

int32_t band_local_rows(int32_t res_y, int32_t band_count, int32_t band_rows) {
    if (res_y <= 0) return 0;
    if (band_count <= 1) return res_y;
    const int32_t blocks = (res_y + band_rows - 1) / band_rows;
    const int32_t slots = (blocks + band_count - 1) / band_count;
    return slots * band_rows;
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
void cut_setup(const rtd::SceneDev &S, rtd::FrameDev &F) {
    F.cut_test = 0;
    if (!S.cut || !S.bvh4 || !S.has_prims || F.res_x <= 0 || F.res_y <= 0) return;
    if (const char *e = std::getenv("RT_NO_CUT"))  // testing: every camera packet from the root
        if (*e && *e != '0') return;
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

// (Re)computes the top-level cut of the current 4-wide tree on the context's
// stream, after the kernels that built or refitted it (the caller
// synchronises the stream before any frame can read it).
int enqueue_cut(rt_ctx *ctx) {
    rtd::SceneDev &S = ctx->S;
    S.cut = nullptr;
    if (!S.bvh4 || !S.nodes4 || !S.has_prims) return RT_OK;
    if (!ctx->d_cut) HIP_OR_FAIL(ctx, hipMalloc((void **)&ctx->d_cut, sizeof(rtd::CutTable)));
    HIP_OR_FAIL(ctx, rtk::launch_build_cut(S.nodes4, ctx->d_cut, ctx->stream));
    S.cut = ctx->d_cut;
    return RT_OK;
}

// After a refit of the tree the cut was built for (same topology): the same
// subtrees with their new boxes.
int enqueue_cut_refresh(rt_ctx *ctx) {
    rtd::SceneDev &S = ctx->S;
    if (!S.cut || !S.bvh4 || !S.nodes4 || !S.has_prims) return enqueue_cut(ctx);
    HIP_OR_FAIL(ctx, rtk::launch_refresh_cut(S.nodes4, ctx->d_cut, ctx->stream));
    return RT_OK;
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
    const int tiles_y = (F.local_rows + th - 1) / th;
    F.num_tiles = F.res_x > 0 ? F.tiles_x * tiles_y : 0;
    const bool f8 = (prm->flags & RT_FLAG_OUT_RGBA8) != 0, f16 = (prm->flags & RT_FLAG_OUT_RGBA16F) != 0,
               f12 = (prm->flags & RT_FLAG_OUT_RGB32F) != 0;
    if ((int)f8 + (int)f16 + (int)f12 > 1)
        return fail(ctx, RT_E_INVALID, "RT_FLAG_OUT_RGBA8, RT_FLAG_OUT_RGBA16F and RT_FLAG_OUT_RGB32F are exclusive");
    F.out_format = f8 ? rtd::kOutRGBA8 : (f16 ? rtd::kOutRGBA16F : (f12 ? rtd::kOutRGB32F : rtd::kOutFloat4));
    out_bytes = (size_t)F.local_rows * F.res_x * rt_pixel_bytes(prm->flags);
    sky_setup(ctx->S, F);
    cut_setup(ctx->S, F);
    return RT_OK;
}

// The context's own device output buffer (rt_render), grow-only.
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
        HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
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

template <typename T>
hipError_t put(rt_ctx *ctx, GrowBuf &b, const T *src, size_t count) {
    hipError_t e = ensure(ctx, b, count * sizeof(T));
    if (e != hipSuccess || count == 0) return e;
    return hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
}

// Quarter-wave splitting of a frame's slowest tiles trades extra work (each
// quarter re-walks the BVH top) for a shorter critical path; it pays only
// when the frame (shard) is small enough for its slowest wave to set its
// time: measured with 3 frames in flight, a 1/8 C3 shard (16,200 tiles)
// +18 %, a 1/4 shard (32,400) -7 %, a whole frame (129,600) -7 %.  The very
// slowest of them (1/2048 of the tiles) go further, to sixteen waves of one
// pixel each: a 1/8 shard's single frame -14 % more, throughput with frames
// in flight +-1 % (1/512 or more: -5..-15 %).
constexpr int kSplit16Div = 2048;  // of those, 1/kSplit16Div of the tiles as sixteenth-waves; 0: off
constexpr int kSplitDiv = 256;  // 1/kSplitDiv of the tiles (the slowest) run as quarter-waves; 0: off
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
constexpr int kLptPeriod = 16;  // frames between longest-first re-sorts (one hipCUB sort ~46 us)
// rt_render's host-output pipeline: row slabs alternating over two streams, relative row counts
// kSlabsCopyBound when the PCIe copy is the longer part (float RGBA: 33 MB at 1080p, 0.59 ms against
// a 0.29 ms frame — small slabs first so the copy starts early, then slabs the render keeps ahead
// of), else kSlabsRenderBound (RGBA8 / RGBA16F: small last slab, little copy after the render);
// measured best of 9 / 10 weight vectors on C3 (tools/exp/e2e_weights.py, profiles/r03_e2e/).
// Frames under kSlabMinFrame go in one piece.
constexpr double kSlabsCopyBound[] = {1, 2, 2, 3, 3, 4};
constexpr double kSlabsRenderBound[] = {1, 2, 2, 1};
constexpr size_t kSlabMinFrame = (size_t)2 << 20;
constexpr int kMaxSlabs = 16;  // RT_SLABS / RT_SLAB_WEIGHTS (tuning) range

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
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
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
    HIP_OR_FAIL(ctx, hipDeviceSynchronize());
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

// Longest-first dispatch of a megakernel launch: picks the state of
// (stream, slab), points F at the last measured order and decides whether
// this launch measures costs (the caller sorts them after the launch).
int lpt_prepare(rt_ctx *ctx, rtd::FrameDev &F, const rt_render_params *prm, bool mega, bool count, int slab,
                LptSlot *&ls, bool &lpt_sort) {
    ls = nullptr;
    lpt_sort = false;
    F.tile_order = nullptr;
    F.tile_cost = nullptr;
    F.wave_counts = nullptr;
    if (!mega || (prm->flags & RT_FLAG_ROW_ORDER) != 0 || F.num_tiles <= 0) return RT_OK;
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
            F.split16_tiles = std::min(F.split_tiles, std::max(1, F.num_tiles / kSplit16Div));
            F.split_tiles -= F.split16_tiles;
        }
    } else if (F.tile_order && !count && !levels && kSplit16DivLarge > 0 && 4 % F.spp == 0 &&
               F.num_tiles <= kSplit16MaxTiles) {
        F.split16_tiles = std::max(1, F.num_tiles / kSplit16DivLarge);
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
    return RT_OK;
}

int lpt_sort_now(rt_ctx *ctx, const rtd::FrameDev &F, LptSlot *ls) {
    HIP_OR_FAIL(ctx, rtk::sort_tiles_by_cost((const unsigned *)ls->cost.p, (unsigned *)ls->cost_sorted.p,
                                             (const int *)ls->iota.p, (int *)ls->order.p, F.num_tiles,
                                             ls->scratch.p, ls->scratch.cap, ctx->stream));
    ls->valid = true;
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

// Enqueues the trace launch(es) of F on the context's stream.
int launch_frame(rt_ctx *ctx, rtd::FrameDev &F, const Path &P, const rtw::Args &A, int chunk_tiles) {
    if (P.packet)
        HIP_OR_FAIL(ctx, rtk::launch_render_packet(ctx->S, F, P.count, ctx->stream));
    else if (P.mega)
        HIP_OR_FAIL(ctx, rtk::launch_render_mega(ctx->S, F, P.count, ctx->stream));
    else if (P.wavefront && F.num_tiles > 0)
        HIP_OR_FAIL(ctx, rtk::launch_render_wavefront(ctx->S, F, A, chunk_tiles, P.count, ctx->stream));
    return RT_OK;
}

int run_frame(rt_ctx *ctx, rtd::FrameDev &F, const rt_render_params *prm, void *d_out, rt_stats *stats,
              std::chrono::steady_clock::time_point t_start, void *host_out, size_t out_bytes) {
    Range range("rt_frame");
    F.out = d_out;
    F.counters = ctx->d_counters;
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
    // host while the next ones render (the PCIe copy is the longer part)
    const bool slabs = host_out && out_bytes && F.band_count == 1 && !P.wavefront;
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
        const bool copy_bound = F.out_format == rtd::kOutFloat4 || F.out_format == rtd::kOutRGB32F;
        const double *w0 = copy_bound ? kSlabsCopyBound : kSlabsRenderBound;
        int nslab = out_bytes < kSlabMinFrame ? 1 : copy_bound ? 6 : 4;
        if (nslab > 1)
            for (int k = 0; k < nslab; ++k) wts[k] = w0[k];
        if (const char *e = std::getenv("RT_SLABS")) {  // tuning: equal slabs
            nslab = std::max(1, std::min(kMaxSlabs, std::atoi(e)));
            for (int k = 0; k < kMaxSlabs; ++k) wts[k] = 1.0;
        }
        if (const char *e = std::getenv("RT_SLAB_WEIGHTS")) {  // tuning: "1,1,2,4,8"
            nslab = 0;
            for (const char *q = e; *q && nslab < kMaxSlabs;) {
                wts[nslab++] = std::max(1e-3, std::atof(q));
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
            nslab = std::max(1, nslab);
        }
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
        int st = lpt_prepare(ctx, L.F, prm, P.mega, P.count, 0, L.ls, L.sort);
        if (st) return st;
        launches.push_back(L);
    }
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
        for (int k = 0; k < nslab; ++k) {
            ctx->stream = launches[k].stream;
            int st = launch_frame(ctx, launches[k].F, P, A, chunk_tiles);
            if (st) return st;
            HIP_OR_FAIL(ctx, hipEventRecord(ctx->slab_done[k], ctx->stream));
            // the copier thread copies slab k once its launch has ended, while
            // this thread enqueues the next launches
            const int r0 = launches[k].r0, r1 = launches[k].r1;
            if (r1 > r0)
                ctx->copier.post({ctx->slab_done[k], (char *)host_out + (size_t)r0 * row_bytes,
                                  (const char *)d_out + (size_t)r0 * row_bytes, (size_t)(r1 - r0) * row_bytes});
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
        HIP_OR_FAIL(ctx, ctx->copier.wait());  // every slab is in the caller's buffer
    } else {
        Launch &L = launches[0];
        int st = launch_frame(ctx, L.F, P, A, chunk_tiles);
        if (st) return st;
        if (async) {
            if (L.sort) {
                st = lpt_sort_now(ctx, L.F, L.ls);
                if (st) return st;
            }
            st = record_async_end(ctx);
            if (st) return st;
            if (ctx->async_frames++ == 0 && ctx->async_t0_set == false) {
                ctx->async_t0 = t_start;
                ctx->async_t0_set = true;
            }
            if (stats) std::memset(stats, 0, sizeof *stats);
            return RT_OK;
        }
        HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
        st = fold_counters(ctx, ctx->stream);
        if (st) return st;
        if (L.sort) {  // after the timed region: the order of the next frames
            st = lpt_sort_now(ctx, L.F, L.ls);
            if (st) return st;
        }
        if (host_out && out_bytes)
            HIP_OR_FAIL(ctx, hipMemcpyAsync(host_out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    unsigned long long counts[rtd::kCounterWords];
    read_folded(ctx, counts);
    if (stats) {
        float ms = 0.0f;
        HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        fill_stats(stats, counts, ms,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    }
    return RT_OK;
}


// Scene.CalculateAABB (Scene.cs:17-41) with Unity min/max semantics:
// mesh AABBs, then loose triangle vertices, then sphere boxes.
void scene_aabb(const rt_scene_desc *sc, rtm::f3 &smin_out, rtm::f3 &smax_out) {
    const int NS = sc->sphere_count, NL = sc->triangle_count;
    rtm::f3 smin = rtm::mk(FLT_MAX, FLT_MAX, FLT_MAX), smax = rtm::mk(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    auto enc_box = [&](rtm::f3 lo, rtm::f3 hi) {  // AABB.Encapsulate(AABB): min(Min, other.Min)
        smin = rtm::mk(rtm::umin(smin.x, lo.x), rtm::umin(smin.y, lo.y), rtm::umin(smin.z, lo.z));
        smax = rtm::mk(rtm::umax(smax.x, hi.x), rtm::umax(smax.y, hi.y), rtm::umax(smax.z, hi.z));
    };
    auto enc_pt = [&](rtm::f3 p) {  // AABB.Encapsulate(float3): min(point, Min)
        smin = rtm::mk(rtm::umin(p.x, smin.x), rtm::umin(p.y, smin.y), rtm::umin(p.z, smin.z));
        smax = rtm::mk(rtm::umax(p.x, smax.x), rtm::umax(p.y, smax.y), rtm::umax(p.z, smax.z));
    };
    for (int m = 0; m < sc->mesh_count; ++m) enc_box(F3(sc->meshes[m].aabb.min), F3(sc->meshes[m].aabb.max));
    for (int i = 0; i < NL; ++i) {
        enc_pt(F3(sc->triangles[i].vertex0));
        enc_pt(F3(sc->triangles[i].vertex1));
        enc_pt(F3(sc->triangles[i].vertex2));
    }
    for (int i = 0; i < NS; ++i) {  // Sphere.AABB, Sphere.cs:17-22
        const rtm::f3 c = F3(sc->spheres[i].center);
        const float r = sqrtf(sc->spheres[i].radius_squared);
        enc_box(rtm::mk(c.x - r, c.y - r, c.z - r), rtm::mk(c.x + r, c.y + r, c.z + r));
    }
    smin_out = smin;
    smax_out = smax;
}

// Absolute node-box padding: 2^-13 of the scene's coordinate scale.
float pad_abs_of(rtm::f3 smin, rtm::f3 smax) {
    float scale = 1.0f;
    for (float v : {smin.x, smin.y, smin.z, smax.x, smax.y, smax.z})
        if (std::isfinite(v)) scale = std::max(scale, std::fabs(v));
    return scale * 0x1p-13f;
}

// Runs the device build on inputs already resident (ctx->lb) and points the
// scene at its output.
int run_lbvh(rt_ctx *ctx, const rtl::LbvhInput &in, bool wide, rtd::SceneDev &S, int &nodes_count) {
    LbvhBufs &B = ctx->lb;
    const int P = in.mt + in.ns + in.nl;
    rtl::LbvhOutput out{};
    out.nodes = (rtd::BvhNode *)B.nodes.p;
    out.nodes4 = wide ? (rtd::BvhNode4 *)B.nodes4.p : nullptr;
    out.tris = (rtd::TriRec *)B.tris.p;
    out.sphs = (rtd::SphRec *)B.sphs.p;
    out.shade = (float4 *)B.shade.p;
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    HIP_OR_FAIL(ctx, rtl::build_lbvh_gpu(in, out, B.scratch.p, B.scratch.cap, ctx->stream));
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    float ms = 0.0f;
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->info.build_ms += ms;
    int binfo[3] = {0, 0, 0};  // 2-wide depth, 4-wide node count, 4-wide depth
    HIP_OR_FAIL(ctx, hipMemcpy(binfo, rtl::lbvh_info_ptr(B.scratch.p, P), sizeof(binfo), hipMemcpyDeviceToHost));
    ctx->last_bvh_depth = wide ? binfo[2] : binfo[0];
    // traversal stack: one entry per 2-wide level, three per 4-wide level
    const int need = wide ? 3 * (binfo[2] + 1) : binfo[0] + 1;
    if (need > rtd::kStackTotal)
        return fail(ctx, RT_E_SCENE, "LBVH %d-wide depth %d exceeds the traversal stack; use RT_BUILD_SAH_HOST",
                    wide ? 4 : 2, wide ? binfo[2] : binfo[0]);
    S.nodes = (const rtd::BvhNode *)B.nodes.p;
    S.nodes4 = wide ? (const rtd::BvhNode4 *)B.nodes4.p : nullptr;
    S.tris = (const rtd::TriRec *)B.tris.p;
    S.sphs = (const rtd::SphRec *)B.sphs.p;
    S.shade = (const float4 *)B.shade.p;
    S.bvh4 = wide ? 1 : 0;
    nodes_count = wide ? binfo[1] : std::max(1, P - 1);
    ctx->src.in = in;
    ctx->src.wide = wide;
    return RT_OK;
}

// GPU LBVH path of rt_set_scene_ex: uploads the caller's arrays as they are
// (no per-primitive host work beyond material ids) and builds on the device.
// geom_on_device: the mesh triangles/normals were produced on the device
// (rt_set_scene_source) and are already in ctx->lb.
template <typename MatId>
int set_scene_lbvh(rt_ctx *ctx, const rt_scene_desc *sc, int MT, int NS, int NL, rtm::f3 smin, rtm::f3 smax,
                   float pad_abs, MatId &mat_id, bool wide, bool geom_on_device, rtd::SceneDev &S,
                   int &nodes_count) {
    const int P = MT + NS + NL;
    std::vector<rtl::MeshDev> meshes((size_t)sc->mesh_count);
    for (int m = 0; m < sc->mesh_count; ++m) {
        meshes[m].rank_first = ctx->mesh_rank_first[m];
        meshes[m].geom_first = sc->meshes[m].first_triangle;
        meshes[m].count = sc->meshes[m].triangle_count;
        meshes[m].material = mat_id(sc->meshes[m].material);
    }
    std::vector<int> sph_mat((size_t)NS), loose_mat((size_t)NL);
    for (int i = 0; i < NS; ++i) sph_mat[i] = mat_id(sc->sphere_materials[i]);
    for (int i = 0; i < NL; ++i) loose_mat[i] = mat_id(sc->triangle_materials[i]);
    LbvhBufs &B = ctx->lb;
    HIP_OR_FAIL(ctx, put(ctx, B.meshes, meshes.data(), meshes.size()));
    if (!geom_on_device) {
        HIP_OR_FAIL(ctx, put(ctx, B.mesh_tris, sc->mesh_triangles, (size_t)sc->mesh_triangle_total));
        HIP_OR_FAIL(ctx, put(ctx, B.mesh_normals, sc->mesh_triangle_normals, (size_t)sc->mesh_triangle_total));
    }
    HIP_OR_FAIL(ctx, put(ctx, B.spheres, sc->spheres, (size_t)NS));
    HIP_OR_FAIL(ctx, put(ctx, B.sphere_mat, sph_mat.data(), sph_mat.size()));
    HIP_OR_FAIL(ctx, put(ctx, B.loose_tris, sc->triangles, (size_t)NL));
    HIP_OR_FAIL(ctx, put(ctx, B.loose_normals, sc->triangle_normals, (size_t)NL));
    HIP_OR_FAIL(ctx, put(ctx, B.loose_mat, loose_mat.data(), loose_mat.size()));
    HIP_OR_FAIL(ctx, ensure(ctx, B.nodes, sizeof(rtd::BvhNode) * (size_t)std::max(1, P - 1)));
    if (wide) HIP_OR_FAIL(ctx, ensure(ctx, B.nodes4, sizeof(rtd::BvhNode4) * (size_t)std::max(1, P - 1)));
    HIP_OR_FAIL(ctx, ensure(ctx, B.tris, sizeof(rtd::TriRec) * (size_t)(MT + NL + 1)));  // + sentinel
    HIP_OR_FAIL(ctx, ensure(ctx, B.sphs, sizeof(rtd::SphRec) * (size_t)std::max(1, NS)));
    HIP_OR_FAIL(ctx, ensure(ctx, B.shade, sizeof(float4) * (size_t)P));
    const size_t scratch = rtl::lbvh_scratch_bytes(P);
    HIP_OR_FAIL(ctx, ensure(ctx, B.scratch, scratch));
    rtl::LbvhInput in{};
    in.mesh_count = sc->mesh_count;
    in.mt = MT;
    in.ns = NS;
    in.nl = NL;
    in.meshes = (const rtl::MeshDev *)B.meshes.p;
    in.mesh_tris = (const float *)B.mesh_tris.p;
    in.mesh_normals = (const float *)B.mesh_normals.p;
    in.spheres = (const float *)B.spheres.p;
    in.sphere_mat = (const int *)B.sphere_mat.p;
    in.loose_tris = (const float *)B.loose_tris.p;
    in.loose_normals = (const float *)B.loose_normals.p;
    in.loose_mat = (const int *)B.loose_mat.p;
    in.scene_lo[0] = smin.x; in.scene_lo[1] = smin.y; in.scene_lo[2] = smin.z;
    in.scene_hi[0] = smax.x; in.scene_hi[1] = smax.y; in.scene_hi[2] = smax.z;
    in.pad_abs = pad_abs;
    in.gates = (const rtd::MeshGate *)ctx->arr.gates;
    in.mesh_bits = 0;
    while ((1ll << in.mesh_bits) <= (long long)sc->mesh_count) ++in.mesh_bits;  // ids 0 .. mesh_count
    in.key_bits = 64;
    return run_lbvh(ctx, in, wide, S, nodes_count);
}

int set_scene_impl(rt_ctx *ctx, const rt_scene_desc *sc, int32_t build, bool geom_on_device,
                   std::chrono::steady_clock::time_point t_start);
int warm_up(rt_ctx *ctx);

// Device mesh extraction from the resident sources (scene_xform.hip); returns
// the exact per-mesh AABBs on the host (they feed Scene.CalculateAABB).
rtx::XformArgs xform_args(rt_ctx *ctx) {
    LbvhBufs &B = ctx->lb;
    rtx::XformArgs a{};
    a.mesh_count = ctx->src.mesh_count;
    a.vertex_total = ctx->src.vertex_total;
    a.tri_total = ctx->src.tri_total;
    a.meshes = (const rtx::MeshSrcDev *)B.src_meshes.p;
    a.local = (const float *)B.src_local.p;
    a.indices = (const int *)B.src_indices.p;
    a.matrices = (const float *)B.src_matrices.p;
    a.world = (float *)B.src_world.p;
    a.tris = (float *)B.mesh_tris.p;
    a.normals = (float *)B.mesh_normals.p;
    a.aabbs = (rtd::MeshGate *)B.src_aabbs.p;
    a.part_total = ctx->src.part_total;
    a.parts = (rtd::MeshGate *)B.src_parts.p;
    return a;
}

int extract_meshes(rt_ctx *ctx, std::vector<rtd::MeshGate> &aabbs, float &ms) {
    LbvhBufs &B = ctx->lb;
    const rtx::XformArgs a = xform_args(ctx);
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    HIP_OR_FAIL(ctx, rtx::transform_meshes(a, ctx->stream));
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    aabbs.resize((size_t)a.mesh_count);
    if (a.mesh_count)
        HIP_OR_FAIL(ctx, hipMemcpyAsync(aabbs.data(), B.src_aabbs.p, sizeof(rtd::MeshGate) * aabbs.size(),
                                        hipMemcpyDeviceToHost, ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    return RT_OK;
}


}  // namespace

extern "C" {

int32_t rt_abi_version(void) { return RT_ABI_VERSION; }

float rt_spec_threshold(void) { return spec_threshold(); }

}  // extern "C"

namespace {

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
    ctx->copier.stop();
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
    if (ctx->slab_stream2) (void)hipStreamSynchronize(ctx->slab_stream2);
    free_scene(ctx);
    free_wavefront(ctx);
    ctx->lb.release();
    ctx->src.refit.release();
    for (LptSlot &l : ctx->lpt) l.release();
    if (ctx->wf_ctr) (void)hipFree(ctx->wf_ctr);
    if (ctx->d_out) (void)hipFree(ctx->d_out);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->d_cut) (void)hipFree(ctx->d_cut);
    if (ctx->h_counts) (void)hipHostFree(ctx->h_counts);
    if (ctx->h_update) (void)hipHostFree(ctx->h_update);
    if (ctx->ev_x) (void)hipEventDestroy(ctx->ev_x);
    if (ctx->d_rays) (void)hipFree(ctx->d_rays);
    if (ctx->d_hits) (void)hipFree(ctx->d_hits);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev_a0) (void)hipEventDestroy(ctx->ev_a0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->ev_slab0) (void)hipEventDestroy(ctx->ev_slab0);
    for (auto &se : ctx->async_end) (void)hipEventDestroy(se.second);
    for (hipEvent_t e : ctx->slab_done) (void)hipEventDestroy(e);
    if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->slab_stream2) (void)hipStreamDestroy(ctx->slab_stream2);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

int nmembers(const rt_ctx *c) { return 1 + (int)c->peers.size(); }
rt_ctx *member(rt_ctx *c, int i) { return i == 0 ? c : c->peers[(size_t)i - 1]; }

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
    for (auto &t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (st[(size_t)i] != RT_OK) {
            if (i) ctx->err = "device " + std::to_string(member(ctx, i)->device) + ": " + member(ctx, i)->err;
            return st[(size_t)i];
        }
    return RT_OK;
}

void release_group(rt_ctx *ctx) {
    if (!ctx->comms.empty()) {  // only an RCCL group ever loaded the library
        Rccl &R = rccl();
        for (ncclComm_t c : ctx->comms)
            if (c && R.ok) (void)R.comm_destroy(c);
        ctx->comms.clear();
    }
    const int n = nmembers(ctx);
    for (GroupSlot &g : ctx->gslots) {
        if (!g.used) continue;
        for (int i = 0; i < n && i < (int)g.member_stream.size(); ++i) {
            (void)hipSetDevice(member(ctx, i)->device);
            if (g.member_stream[(size_t)i]) {
                (void)hipStreamSynchronize(g.member_stream[(size_t)i]);
                (void)hipStreamDestroy(g.member_stream[(size_t)i]);
            }
            if (g.member_done[(size_t)i]) (void)hipEventDestroy(g.member_done[(size_t)i]);
            if (g.member_out[(size_t)i].p) (void)hipFree(g.member_out[(size_t)i].p);
        }
        (void)hipSetDevice(ctx->device);
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
        const ncclResult_t r = R.comm_init_all(root->comms.data(), n, devices);
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
        HIP_OR_FAIL(m, hipMemcpy2DAsync((char *)host + (size_t)band * R * row, (size_t)bands * R * row, band_buf,
                                        (size_t)R * row, (size_t)R * row, (size_t)mine, hipMemcpyDeviceToHost,
                                        m->stream));
    const int rest = res_y - full * R;  // rows of a last partial block
    if (rest > 0 && full % bands == band && row > 0)
        HIP_OR_FAIL(m, hipMemcpyAsync((char *)host + (size_t)full * R * row,
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
        st = run_frame(m, F[(size_t)i], &mp[(size_t)i], out, nullptr, t0, nullptr, 0);
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
            HIP_OR_FAIL(ctx, hipStreamSynchronize(m->stream));
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
        const ncclResult_t r2 = Rc.group_end();
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
        HIP_OR_FAIL(ctx, hipMemcpyAsync(host_out, d_out, full_bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (async) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    return group_stats(ctx, stash, stats, t0);
}

}  // namespace

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
        return create_one(dev, out_ctx);
    }
    if (num_gpus > count)
        return fail(nullptr, RT_E_NO_DEVICE, "num_gpus %d > %d visible devices", num_gpus, count);
    std::vector<int32_t> devs((size_t)num_gpus);
    for (int i = 0; i < num_gpus; ++i) devs[(size_t)i] = i;
    return create_group(devs.data(), num_gpus, 0, out_ctx);
}

int rt_create_devices(rt_ctx **out_ctx, const int32_t *devices, int32_t num_devices, int32_t gather) {
    if (!out_ctx) return fail(nullptr, RT_E_INVALID, "out_ctx is null");
    *out_ctx = nullptr;
    if (num_devices < 1 || !devices) return fail(nullptr, RT_E_INVALID, "need at least one device");
    return create_group(devices, num_devices, gather, out_ctx);
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

int rt_set_scene(rt_ctx *ctx, const rt_scene_desc *sc) { return rt_set_scene_ex(ctx, sc, RT_BUILD_SAH_HOST); }

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

namespace {

int set_scene_impl(rt_ctx *ctx, const rt_scene_desc *sc, int32_t build, bool geom_on_device,
                   std::chrono::steady_clock::time_point t_start) {
    if (!sc) return fail(ctx, RT_E_INVALID, "scene is null");
    if (build != RT_BUILD_SAH_HOST && build != RT_BUILD_LBVH_GPU && build != RT_BUILD_LBVH_GPU_BVH2)
        return fail(ctx, RT_E_INVALID, "unknown build %d", build);
    if (sc->triangle_count < 0 || sc->mesh_triangle_total < 0 || sc->mesh_count < 0 || sc->sphere_count < 0 ||
        sc->point_light_count < 0)
        return fail(ctx, RT_E_INVALID, "negative count in scene");
    if ((sc->triangle_count && (!sc->triangles || !sc->triangle_normals || !sc->triangle_materials)) ||
        (sc->mesh_count && !sc->meshes) ||
        (sc->mesh_triangle_total && !geom_on_device && (!sc->mesh_triangles || !sc->mesh_triangle_normals)) ||
        (sc->sphere_count && (!sc->spheres || !sc->sphere_materials)) ||
        (sc->point_light_count && !sc->point_lights))
        return fail(ctx, RT_E_INVALID, "null array with a non-zero count");
    int64_t mesh_ranks = 0;
    for (int m = 0; m < sc->mesh_count; ++m) {
        const rt_mesh &M = sc->meshes[m];
        if (M.triangle_count < 0 || M.first_triangle < 0 ||
            (int64_t)M.first_triangle + M.triangle_count > sc->mesh_triangle_total)
            return fail(ctx, RT_E_SCENE, "mesh %d range [%d, +%d) outside mesh_triangle_total %d", m,
                        M.first_triangle, M.triangle_count, sc->mesh_triangle_total);
        mesh_ranks += M.triangle_count;
    }
    if (mesh_ranks + sc->sphere_count + sc->triangle_count > (int64_t)(1 << rtd::kLeafFirstBits))
        return fail(ctx, RT_E_SCENE, "too many primitives (max %d)", 1 << rtd::kLeafFirstBits);
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    free_scene(ctx);
    ctx->info = rt_scene_info{};
    ++ctx->scene_version;

    const int MT = (int)mesh_ranks, NS = sc->sphere_count, NL = sc->triangle_count;
    const int P = MT + NS + NL;

    // Scene.CalculateAABB (Scene.cs:17-41) with Unity min/max semantics.
    rtm::f3 smin, smax;
    scene_aabb(sc, smin, smax);

    // Materials, deduplicated.
    std::map<rt_material, int, bool (*)(const rt_material &, const rt_material &)> mat_ids(mat_less);
    std::vector<rtd::DevMaterial> mats;
    auto mat_id = [&](const rt_material &m) {
        auto it = mat_ids.find(m);
        if (it != mat_ids.end()) return it->second;
        int id = (int)mats.size();
        mat_ids.emplace(m, id);
        mats.push_back(to_dev(m));
        return id;
    };
    const float pad_abs = pad_abs_of(smin, smax);

    ctx->mesh_rank_first.assign((size_t)sc->mesh_count + 1, 0);
    {
        int rk = 0;
        for (int m = 0; m < sc->mesh_count; ++m) {
            ctx->mesh_rank_first[m] = rk;
            rk += sc->meshes[m].triangle_count;
        }
        ctx->mesh_rank_first[sc->mesh_count] = rk;
    }
    std::vector<rtd::MeshGate> gates((size_t)sc->mesh_count);
    for (int m = 0; m < sc->mesh_count; ++m) {
        const rt_aabb &a = sc->meshes[m].aabb;
        gates[m].lo = make_float4(a.min.x, a.min.y, a.min.z, 0.0f);
        gates[m].hi = make_float4(a.max.x, a.max.y, a.max.z, 0.0f);
    }
    std::vector<rtd::DevLight> lights((size_t)sc->point_light_count);
    for (int l = 0; l < sc->point_light_count; ++l) {
        const rt_point_light &L = sc->point_lights[l];
        lights[l].pos = make_float4(L.position.x, L.position.y, L.position.z, 0.0f);
        lights[l].intensity = make_float4(L.intensity.x, L.intensity.y, L.intensity.z, 0.0f);
    }

    HIP_OR_FAIL(ctx, upload(&ctx->arr.gates, gates));  // before the build: the LBVH keys use the mesh boxes
    rtd::SceneDev &S = ctx->S;
    int nodes_count = 0;
    if ((build == RT_BUILD_LBVH_GPU || build == RT_BUILD_LBVH_GPU_BVH2) && P > 0) {
        const int st = set_scene_lbvh(ctx, sc, MT, NS, NL, smin, smax, pad_abs, mat_id,
                                      build == RT_BUILD_LBVH_GPU, geom_on_device, S, nodes_count);
        if (st) return st;
    } else {
        // Host binned-SAH build (bvh.cpp), collapsed to 4-wide nodes.
        struct TriSrc { rtm::f3 v0, v1, v2; };
        std::vector<TriSrc> tri_src((size_t)P);
        std::vector<float4> shade((size_t)P);
        std::vector<rtb::Prim> prims;
        prims.reserve((size_t)P);
        auto add_tri_prim = [&](int rank, const rt_triangle &t, int gate) {
            rtb::Prim p;
            const float *v[3] = {&t.vertex0.x, &t.vertex1.x, &t.vertex2.x};
            float ext = 0.0f;
            for (int a = 0; a < 3; ++a) {
                p.lo[a] = std::min(v[0][a], std::min(v[1][a], v[2][a]));
                p.hi[a] = std::max(v[0][a], std::max(v[1][a], v[2][a]));
                ext = std::max(ext, p.hi[a] - p.lo[a]);
            }
            const float pad = pad_abs + ext * 1e-4f;
            for (int a = 0; a < 3; ++a) {
                p.c[a] = 0.5f * (p.lo[a] + p.hi[a]);
                p.lo[a] -= pad;
                p.hi[a] += pad;
            }
            p.kind = rtd::kLeafTri;
            p.gate = gate;
            p.payload = rank;
            tri_src[rank] = {F3(t.vertex0), F3(t.vertex1), F3(t.vertex2)};
            prims.push_back(p);
        };
        auto put_shade = [&](int rank, float x, float y, float z, int mid) {
            shade[rank] = make_float4(x, y, z, 0.0f);
            std::memcpy(&shade[rank].w, &mid, 4);
        };
        int rank = 0;
        for (int m = 0; m < sc->mesh_count; ++m) {
            const rt_mesh &M = sc->meshes[m];
            const int mid = mat_id(M.material);
            for (int i = 0; i < M.triangle_count; ++i, ++rank) {
                const int g = M.first_triangle + i;
                add_tri_prim(rank, sc->mesh_triangles[g], m);
                const rt_float3 &nn = sc->mesh_triangle_normals[g];
                put_shade(rank, nn.x, nn.y, nn.z, mid);
            }
        }
        std::vector<rtd::SphRec> sph_src((size_t)NS);
        for (int i = 0; i < NS; ++i, ++rank) {
            const rt_sphere &s = sc->spheres[i];
            const float r = sqrtf(s.radius_squared);
            rtb::Prim p;
            const float c[3] = {s.center.x, s.center.y, s.center.z};
            const float pad = pad_abs + r * 1e-4f;
            for (int a = 0; a < 3; ++a) {
                p.c[a] = c[a];
                p.lo[a] = c[a] - r - pad;
                p.hi[a] = c[a] + r + pad;
            }
            p.kind = rtd::kLeafSphere;
            p.gate = -1;
            p.payload = rank;
            prims.push_back(p);
            sph_src[i].cr = make_float4(s.center.x, s.center.y, s.center.z, s.radius_squared);
            sph_src[i].misc = make_int4(rank, -1, 0, 0);
            put_shade(rank, s.center.x, s.center.y, s.center.z, mat_id(sc->sphere_materials[i]));
        }
        for (int i = 0; i < NL; ++i, ++rank) {
            add_tri_prim(rank, sc->triangles[i], -1);
            const rt_float3 &nn = sc->triangle_normals[i];
            put_shade(rank, nn.x, nn.y, nn.z, mat_id(sc->triangle_materials[i]));
        }

        rtb::BuildResult B = rtb::build_bvh(prims, 4);
        ctx->last_bvh_depth = B.max_depth;
        if (B.max_depth > rtd::kMaxTreeDepth)
            return fail(ctx, RT_E_INTERNAL, "BVH depth %d exceeds stack", B.max_depth);
        std::vector<rtd::BvhNode4> nodes4;
        const int sentinel = (int)B.tri_order.size();
        const int depth4 = rtb::collapse_bvh4(B, nodes4, rtd::encode_leaf(sentinel, 1, rtd::kLeafTri));
        if (3 * (depth4 + 1) > rtd::kStackTotal)
            return fail(ctx, RT_E_INTERNAL, "BVH4 depth %d exceeds stack", depth4);
        std::vector<int> tri_gate((size_t)P, -1);
        for (int m = 0; m < sc->mesh_count; ++m)
            for (int r = ctx->mesh_rank_first[m]; r < ctx->mesh_rank_first[m + 1]; ++r) tri_gate[r] = m;
        std::vector<rtd::TriRec> tris(B.tri_order.size());
        for (size_t i = 0; i < B.tri_order.size(); ++i) {
            const int rk = B.tri_order[i];
            const TriSrc &t = tri_src[rk];
            const rtm::f3 e1 = t.v1 - t.v0, e2 = t.v2 - t.v0;  // RMath.cs:34-35
            float rbits, gbits;
            std::memcpy(&rbits, &rk, 4);
            std::memcpy(&gbits, &tri_gate[rk], 4);
            tris[i].p0 = make_float4(t.v0.x, t.v0.y, t.v0.z, e1.x);
            tris[i].p1 = make_float4(e1.y, e1.z, e2.x, e2.y);
            tris[i].p2 = make_float4(e2.z, rbits, gbits, 0.0f);
        }
        tris.push_back(rtd::sentinel_tri());
        std::vector<rtd::SphRec> sphs(B.sph_order.size());
        for (size_t i = 0; i < B.sph_order.size(); ++i) sphs[i] = sph_src[B.sph_order[i] - MT];
        HIP_OR_FAIL(ctx, upload(&ctx->arr.nodes4, nodes4));
        HIP_OR_FAIL(ctx, upload(&ctx->arr.tris, tris));
        HIP_OR_FAIL(ctx, upload(&ctx->arr.sphs, sphs));
        HIP_OR_FAIL(ctx, upload(&ctx->arr.shade, shade));
        S.nodes = nullptr;
        S.nodes4 = (const rtd::BvhNode4 *)ctx->arr.nodes4;
        S.tris = (const rtd::TriRec *)ctx->arr.tris;
        S.sphs = (const rtd::SphRec *)ctx->arr.sphs;
        S.shade = (const float4 *)ctx->arr.shade;
        S.bvh4 = 1;
        nodes_count = (int)nodes4.size();
    }
    HIP_OR_FAIL(ctx, upload(&ctx->arr.mats, mats));
    HIP_OR_FAIL(ctx, upload(&ctx->arr.lights, lights));
    S.has_prims = P > 0;
    {
        const int st = enqueue_cut(ctx);
        if (st) return st;
    }
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));

    S.leaves = nullptr;
    S.mats = (const rtd::DevMaterial *)ctx->arr.mats;
    S.lights = (const rtd::DevLight *)ctx->arr.lights;
    S.gates = (const rtd::MeshGate *)ctx->arr.gates;
    S.num_lights = sc->point_light_count;
    S.mesh_tri_total = MT;
    S.sphere_count = NS;
    S.has_prims = P > 0;
    S.scene_lo[0] = smin.x; S.scene_lo[1] = smin.y; S.scene_lo[2] = smin.z;
    S.scene_hi[0] = smax.x; S.scene_hi[1] = smax.y; S.scene_hi[2] = smax.z;
    S.ambient[0] = sc->ambient_radiance.x;
    S.ambient[1] = sc->ambient_radiance.y;
    S.ambient[2] = sc->ambient_radiance.z;
    S.spec_threshold = spec_threshold();
    ctx->mesh_tri_ranks = MT;
    ctx->sphere_count = NS;
    ctx->loose_count = NL;
    ctx->info.build = build;
    ctx->info.bvh_width = P > 0 ? (S.bvh4 ? 4 : 2) : 0;
    ctx->info.nodes = P > 0 ? nodes_count : 0;
    ctx->info.primitives = P;
    ctx->info.total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    ctx->has_scene = true;
    return warm_up(ctx);
}

// The first launch of a kernel pays for loading its code object and for the
// queue's scratch (private segment) allocation — 16-17 ms of a context's first
// frame, i.e. of the first Update.  Once per context, right after its first
// scene: tiny frames (16 x 16) through every render-kernel instance a frame
// takes (1, 4 and 16 spp; twice each, so the split instance that needs a
// measured tile order runs too; the tile-count reduction, the tile sort).
int warm_up(rt_ctx *ctx) {
    if (ctx->warmed) return RT_OK;
    ctx->warmed = true;
    const rtd::SceneDev &S = ctx->S;
    rt_camera cam{};
    cam.position = {0.5f * (S.scene_lo[0] + S.scene_hi[0]), 0.5f * (S.scene_lo[1] + S.scene_hi[1]),
                    S.scene_lo[2] - 1.0f};
    if (!std::isfinite(cam.position.x) || !std::isfinite(cam.position.y) || !std::isfinite(cam.position.z))
        cam.position = {0.0f, 0.0f, -1.0f};
    cam.forward = {0.0f, 0.0f, 1.0f};
    cam.right = {1.0f, 0.0f, 0.0f};
    cam.up = {0.0f, 1.0f, 0.0f};
    rt_image_plane pl{};
    pl.resolution_x = 16;
    pl.resolution_y = 16;
    pl.distance_to_camera = 1.0f;
    pl.half_horizontal_length = 0.5f;
    pl.half_vertical_length = 0.5f;
    for (int spp : {1, 4, 16}) {
        for (int rep = 0; rep < 2; ++rep) {
            rt_render_params prm{};
            prm.max_reflection_bounces = 1;
            prm.samples_per_pixel = spp;
            prm.band_count = 1;
            prm.band_rows = 8;
            rtd::FrameDev F;
            size_t bytes = 0;
            int st = prepare_frame(ctx, &cam, &pl, &prm, F, bytes);
            if (st) return st;
            HIP_OR_FAIL(ctx, ensure_out(ctx, bytes));
            st = run_frame(ctx, F, &prm, ctx->d_out, nullptr, std::chrono::steady_clock::now(), nullptr, 0);
            if (st) return st;
        }
    }
    // rt_render's host-output pipeline (row slabs on two streams + a copy
    // stream): a frame of two slabs
    pl.resolution_x = 512;
    pl.resolution_y = 512;
    rt_render_params prm{};
    prm.max_reflection_bounces = 1;
    prm.samples_per_pixel = 4;
    prm.band_count = 1;
    prm.band_rows = 8;
    rtd::FrameDev F;
    size_t bytes = 0;
    int st = prepare_frame(ctx, &cam, &pl, &prm, F, bytes);
    if (st) return st;
    HIP_OR_FAIL(ctx, ensure_out(ctx, bytes));
    std::vector<unsigned char> host(bytes);
    return run_frame(ctx, F, &prm, ctx->d_out, nullptr, std::chrono::steady_clock::now(), host.data(), bytes);
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// ---- RT_BUILD_SAH_REFIT ------------------------------------------------

rtx::RefitArgs refit_args(rt_ctx *ctx) {
    RefitState &R = ctx->src.refit;
    LbvhBufs &B = ctx->lb;
    rtx::RefitArgs a{};
    a.ntri = R.ntri;
    a.nsph = R.nsph;
    a.nnodes = R.nnodes;
    a.tris = (rtd::TriRec *)ctx->S.tris;  // the host build's arrays or the LBVH's (B.*)
    a.sphs = ctx->S.sphs;
    a.shade = (float4 *)ctx->S.shade;
    a.mt = ctx->mesh_tri_ranks;
    a.ns = ctx->sphere_count;
    a.mesh_count = ctx->src.mesh_count;
    a.mesh_rank_first = (const int *)R.rank_first.p;
    a.mesh_geom_first = (const int *)R.geom_first.p;
    a.mesh_tris = (const float *)B.mesh_tris.p;
    a.mesh_normals = (const float *)B.mesh_normals.p;
    a.loose_tris = (const float *)R.loose.p;
    a.box = (const float *)B.scene_box.p;
    a.prim_lo = (float4 *)R.prim_lo.p;
    a.prim_hi = (float4 *)R.prim_hi.p;
    a.nodes = (rtd::BvhNode4 *)ctx->S.nodes4;
    a.parent_slot = (const int *)R.parent_slot.p;
    a.internal_children = (const int *)R.internal_children.p;
    a.arrivals = (int *)R.arrivals.p;
    a.empty_ref = rtd::encode_leaf(R.ntri, 1, rtd::kLeafTri);  // the sentinel record (both builders)
    a.quality = (float *)R.quality.p;
    return a;
}

// A full build of the current device geometry (world triangles as
// extracted, exact mesh AABBs `aabbs`): the host SAH tree (rt_set_scene_source_ex)
// or, when a refitted tree has degraded, the device LBVH (a host rebuild of a
// big scene would stall the Update for tens of ms); then the tree's refit
// tables and one refit of that same geometry for its reference surface area.
int refit_build(rt_ctx *ctx, const std::vector<rtd::MeshGate> &aabbs, bool host_sah,
                std::chrono::steady_clock::time_point t0) {
    RefitState &R = ctx->src.refit;
    LbvhBufs &B = ctx->lb;
    const int tt = ctx->src.tri_total, M = ctx->src.mesh_count;
    std::vector<rt_triangle> mtris;
    std::vector<rt_float3> mnorm;
    if (host_sah && tt) {
        mtris.resize((size_t)tt);
        mnorm.resize((size_t)tt);
        HIP_OR_FAIL(ctx, hipMemcpy(mtris.data(), B.mesh_tris.p, sizeof(rt_triangle) * (size_t)tt, hipMemcpyDeviceToHost));
        HIP_OR_FAIL(ctx, hipMemcpy(mnorm.data(), B.mesh_normals.p, sizeof(rt_float3) * (size_t)tt,
                                   hipMemcpyDeviceToHost));
    }
    for (int m = 0; m < M; ++m) {
        R.meshes[m].aabb.min = {aabbs[m].lo.x, aabbs[m].lo.y, aabbs[m].lo.z};
        R.meshes[m].aabb.max = {aabbs[m].hi.x, aabbs[m].hi.y, aabbs[m].hi.z};
    }
    rt_scene_desc d = R.base.desc;
    d.meshes = R.meshes.data();
    d.mesh_count = M;
    d.mesh_triangles = host_sah ? mtris.data() : nullptr;
    d.mesh_triangle_normals = host_sah ? mnorm.data() : nullptr;
    d.mesh_triangle_total = tt;
    int st = set_scene_impl(ctx, &d, host_sah ? RT_BUILD_SAH_HOST : RT_BUILD_LBVH_GPU, !host_sah, t0);
    if (st) return st;
    ctx->info.build = RT_BUILD_SAH_REFIT;
    R.nnodes = ctx->info.nodes;
    R.ntri = ctx->mesh_tri_ranks + ctx->loose_count;
    R.nsph = ctx->sphere_count;
    if (R.nnodes <= 0) return RT_OK;
    std::vector<int> rank_first((size_t)std::max(1, M)), geom_first((size_t)std::max(1, M));
    for (int m = 0; m < M; ++m) {
        rank_first[m] = ctx->mesh_rank_first[m];
        geom_first[m] = R.meshes[m].first_triangle;
    }
    const std::vector<rt_triangle> &lt = R.base.tris;
    HIP_OR_FAIL(ctx, ensure(ctx, R.parent_slot, sizeof(int) * (size_t)R.nnodes));
    HIP_OR_FAIL(ctx, ensure(ctx, R.internal_children, sizeof(int) * (size_t)R.nnodes));
    HIP_OR_FAIL(ctx, put(ctx, R.rank_first, rank_first.data(), rank_first.size()));
    HIP_OR_FAIL(ctx, put(ctx, R.geom_first, geom_first.data(), geom_first.size()));
    if (!lt.empty()) HIP_OR_FAIL(ctx, put(ctx, R.loose, lt.data(), lt.size()));
    HIP_OR_FAIL(ctx, ensure(ctx, R.arrivals, sizeof(int) * (size_t)R.nnodes));
    HIP_OR_FAIL(ctx, ensure(ctx, R.prim_lo, sizeof(float4) * (size_t)std::max(1, R.ntri + R.nsph)));
    HIP_OR_FAIL(ctx, ensure(ctx, R.prim_hi, sizeof(float4) * (size_t)std::max(1, R.ntri + R.nsph)));
    HIP_OR_FAIL(ctx, ensure(ctx, R.quality, 2 * sizeof(float)));
    // the reference area: a refit of the geometry just built (the scene box
    // and padding as an update computes them)
    HIP_OR_FAIL(ctx, ensure(ctx, B.scene_box, 8 * sizeof(float)));
    if (!ctx->h_update)
        HIP_OR_FAIL(ctx, hipHostMalloc((void **)&ctx->h_update, sizeof *ctx->h_update, hipHostMallocCoherent));
    HIP_OR_FAIL(ctx, rtx::scene_box((const rtd::MeshGate *)B.src_aabbs.p, M, ctx->src.rest_lo, ctx->src.rest_hi,
                                    (float *)B.scene_box.p, ctx->h_update->box, ctx->stream));
    const rtx::RefitArgs a = refit_args(ctx);
    HIP_OR_FAIL(ctx, rtx::refit_links(a, (int *)R.parent_slot.p, (int *)R.internal_children.p, ctx->stream));
    HIP_OR_FAIL(ctx, rtx::refit_tree(a, ctx->stream));
    {
        const int st = enqueue_cut(ctx);
        if (st) return st;
    }
    HIP_OR_FAIL(ctx, hipMemcpyAsync(ctx->h_update->quality, a.quality, 2 * sizeof(float), hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    const volatile float *q = ctx->h_update->quality;
    R.area_built = q[1] > 0.0f ? q[0] / q[1] : 0.0f;
    return RT_OK;
}

int set_scene_source_one(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count,
                         int32_t build, std::chrono::steady_clock::time_point t0) {
    ctx->src.active = false;
    if (!base) return fail(ctx, RT_E_INVALID, "base scene is null");
    if (build != RT_BUILD_LBVH_GPU && build != RT_BUILD_SAH_REFIT)
        return fail(ctx, RT_E_INVALID, "rt_set_scene_source_ex: build %d is neither RT_BUILD_LBVH_GPU nor "
                    "RT_BUILD_SAH_REFIT", build);
    if (mesh_count < 0 || (mesh_count && !meshes)) return fail(ctx, RT_E_INVALID, "bad mesh source array");
    if (base->mesh_count || base->mesh_triangle_total)
        return fail(ctx, RT_E_INVALID, "the base scene of rt_set_scene_source must not carry meshes");
    int64_t vt = 0, tt = 0;
    for (int m = 0; m < mesh_count; ++m) {
        const rt_mesh_source &M = meshes[m];
        if (M.vertex_count < 0 || M.index_count < 0 || M.index_count % 3)
            return fail(ctx, RT_E_SCENE, "mesh %d: vertex_count %d / index_count %d invalid", m, M.vertex_count,
                        M.index_count);
        if ((M.vertex_count && !M.vertices) || (M.index_count && !M.indices))
            return fail(ctx, RT_E_INVALID, "mesh %d: null array with a non-zero count", m);
        vt += M.vertex_count;
        tt += M.index_count / 3;
    }
    if (vt > (1ll << 28) || tt > (1ll << rtd::kLeafFirstBits))
        return fail(ctx, RT_E_SCENE, "too many mesh vertices / triangles");
    std::vector<rtx::MeshSrcDev> md((size_t)mesh_count);
    std::vector<float> local((size_t)vt * 3), mats((size_t)mesh_count * 16);
    std::vector<int> idx((size_t)tt * 3);
    int parts = 0;  // AABB-reduction parts (scene_xform.hip k_aabb_parts)
    {
        int v = 0, t = 0;
        for (int m = 0; m < mesh_count; ++m) {
            const rt_mesh_source &M = meshes[m];
            md[m] = {v, M.vertex_count, t, M.index_count / 3, parts};
            parts += std::max(1, (M.vertex_count + rtx::kAabbPart - 1) / rtx::kAabbPart);
            if (M.vertex_count) std::memcpy(&local[(size_t)v * 3], M.vertices, sizeof(rt_float3) * M.vertex_count);
            std::memcpy(&mats[(size_t)m * 16], M.local_to_world, sizeof(float) * 16);
            for (int i = 0; i < M.index_count; ++i) {
                const int k = M.indices[i];
                if (k < 0 || k >= M.vertex_count)
                    return fail(ctx, RT_E_SCENE, "mesh %d: index %d = %d outside [0, %d)", m, i, k, M.vertex_count);
                idx[(size_t)t * 3 + i] = v + k;
            }
            v += M.vertex_count;
            t += M.index_count / 3;
        }
    }
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    LbvhBufs &B = ctx->lb;
    HIP_OR_FAIL(ctx, put(ctx, B.src_meshes, md.data(), md.size()));
    HIP_OR_FAIL(ctx, put(ctx, B.src_local, local.data(), local.size()));
    HIP_OR_FAIL(ctx, put(ctx, B.src_indices, idx.data(), idx.size()));
    HIP_OR_FAIL(ctx, put(ctx, B.src_matrices, mats.data(), mats.size()));
    HIP_OR_FAIL(ctx, ensure(ctx, B.src_world, sizeof(float) * 3 * (size_t)vt));
    HIP_OR_FAIL(ctx, ensure(ctx, B.src_aabbs, sizeof(rtd::MeshGate) * (size_t)mesh_count));
    HIP_OR_FAIL(ctx, ensure(ctx, B.src_parts, sizeof(rtd::MeshGate) * (size_t)std::max(parts, 1)));
    HIP_OR_FAIL(ctx, ensure(ctx, B.mesh_tris, sizeof(rt_triangle) * (size_t)tt));
    HIP_OR_FAIL(ctx, ensure(ctx, B.mesh_normals, sizeof(rt_float3) * (size_t)tt));
    ctx->src.mesh_count = mesh_count;
    ctx->src.vertex_total = (int)vt;
    ctx->src.tri_total = (int)tt;
    ctx->src.part_total = parts;
    std::vector<rtd::MeshGate> aabbs;
    float xform_ms = 0.0f;
    int st = extract_meshes(ctx, aabbs, xform_ms);
    if (st) return st;
    std::vector<rt_mesh> dm((size_t)mesh_count);
    for (int m = 0; m < mesh_count; ++m) {
        dm[m].first_triangle = md[m].tri_first;
        dm[m].triangle_count = md[m].tri_count;
        dm[m].material = meshes[m].material;
        dm[m].aabb.min = {aabbs[m].lo.x, aabbs[m].lo.y, aabbs[m].lo.z};
        dm[m].aabb.max = {aabbs[m].hi.x, aabbs[m].hi.y, aabbs[m].hi.z};
    }
    rt_scene_desc rest = *base;  // loose triangles and spheres only
    rtm::f3 lo, hi;
    scene_aabb(&rest, lo, hi);
    ctx->src.rest_lo[0] = lo.x; ctx->src.rest_lo[1] = lo.y; ctx->src.rest_lo[2] = lo.z;
    ctx->src.rest_hi[0] = hi.x; ctx->src.rest_hi[1] = hi.y; ctx->src.rest_hi[2] = hi.z;
    ctx->src.build = build;
    if (build == RT_BUILD_SAH_REFIT) {
        RefitState &R = ctx->src.refit;
        R.base.set(*base);
        R.meshes = dm;
        R.rebuilds = 0;
        st = refit_build(ctx, aabbs, true, t0);
        if (st) return st;
        ctx->info.build_ms += xform_ms;
        ctx->src.active = true;
        return RT_OK;
    }
    rt_scene_desc d = *base;
    d.meshes = dm.data();
    d.mesh_count = mesh_count;
    d.mesh_triangles = nullptr;
    d.mesh_triangle_normals = nullptr;
    d.mesh_triangle_total = (int32_t)tt;
    st = set_scene_impl(ctx, &d, RT_BUILD_LBVH_GPU, true, t0);
    if (st) return st;
    ctx->info.build_ms += xform_ms;
    ctx->src.active = true;
    return RT_OK;
}

// Refit half of an update (RT_BUILD_SAH_REFIT), after the extraction, the
// scene box and the gates are enqueued: the tree refitted on the device, one
// synchronisation; a full host rebuild when the refitted tree's relative
// surface area has grown past kRefitRebuild x that of its last build (or is
// not finite).
int refit_update(rt_ctx *ctx, std::chrono::steady_clock::time_point t0) {
    RefitState &R = ctx->src.refit;
    const rtx::RefitArgs a = refit_args(ctx);
    HIP_OR_FAIL(ctx, rtx::refit_tree(a, ctx->stream));
    {
        const int st = enqueue_cut_refresh(ctx);
        if (st) return st;
    }
    if (R.nnodes > 0)
        HIP_OR_FAIL(ctx, hipMemcpyAsync(ctx->h_update->quality, a.quality, 2 * sizeof(float), hipMemcpyDeviceToHost,
                                        ctx->stream));
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    float xform_ms = 0.0f, refit_ms = 0.0f;
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&xform_ms, ctx->ev0, ctx->ev_x));
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&refit_ms, ctx->ev_x, ctx->ev1));
    const volatile float *hb = ctx->h_update->box;
    rtd::SceneDev &S = ctx->S;
    for (int c = 0; c < 3; ++c) {
        S.scene_lo[c] = hb[c];
        S.scene_hi[c] = hb[3 + c];
    }
    ctx->info.build_ms = xform_ms + refit_ms;
    if (R.nnodes > 0) {
        const volatile float *q = ctx->h_update->quality;
        const float area = q[1] > 0.0f ? q[0] / q[1] : 0.0f;
        static const float limit = [] {  // tuning override
            const char *e = std::getenv("RT_REFIT_REBUILD");
            return e ? (float)std::atof(e) : kRefitRebuild;
        }();
        if (!(area <= limit * R.area_built)) {
            std::vector<rtd::MeshGate> aabbs((size_t)ctx->src.mesh_count);
            if (!aabbs.empty())
                HIP_OR_FAIL(ctx, hipMemcpy(aabbs.data(), ctx->lb.src_aabbs.p, sizeof(rtd::MeshGate) * aabbs.size(),
                                           hipMemcpyDeviceToHost));
            const double build_ms = ctx->info.build_ms;
            const int st = refit_build(ctx, aabbs, false, t0);
            if (st) {
                ctx->has_scene = false;
                return st;
            }
            ++R.rebuilds;
            ctx->info.build_ms = build_ms;
        }
    }
    ctx->info.total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

// The shim's per-Update path: one host synchronisation.  Matrices up,
// extraction, the scene box (device fold of the mesh AABBs), the mesh gates
// and the LBVH build are enqueued back to back; the host then reads the box
// (for the frame's kernel arguments) and the build's depth (the traversal
// stack check) from page-locked words.
int update_mesh_transforms_one(rt_ctx *ctx, const float *local_to_world, int32_t mesh_count,
                              std::chrono::steady_clock::time_point t0) {
    if (!ctx->has_scene || !ctx->src.active)
        return fail(ctx, RT_E_STATE, "rt_update_mesh_transforms needs a scene from rt_set_scene_source");
    if (mesh_count != ctx->src.mesh_count || (mesh_count && !local_to_world))
        return fail(ctx, RT_E_INVALID, "expected %d matrices, got %d", ctx->src.mesh_count, mesh_count);
    HIP_OR_FAIL(ctx, hipSetDevice(ctx->device));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    LbvhBufs &B = ctx->lb;
    if (!ctx->h_update)
        HIP_OR_FAIL(ctx, hipHostMalloc((void **)&ctx->h_update, sizeof *ctx->h_update, hipHostMallocCoherent));
    if (!ctx->ev_x) HIP_OR_FAIL(ctx, hipEventCreate(&ctx->ev_x));
    HIP_OR_FAIL(ctx, ensure(ctx, B.scene_box, 8 * sizeof(float)));
    ++ctx->scene_version;
    if (mesh_count)  // pageable source: staged before the call returns
        HIP_OR_FAIL(ctx, hipMemcpyAsync(B.src_matrices.p, local_to_world, sizeof(float) * 16 * (size_t)mesh_count,
                                        hipMemcpyHostToDevice, ctx->stream));
    const rtx::XformArgs a = xform_args(ctx);
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    HIP_OR_FAIL(ctx, rtx::transform_meshes(a, ctx->stream));
    // Scene.CalculateAABB: mesh AABBs, then the (unchanged) loose triangles and spheres
    HIP_OR_FAIL(ctx, rtx::scene_box(a.aabbs, mesh_count, ctx->src.rest_lo, ctx->src.rest_hi, (float *)B.scene_box.p,
                                    ctx->h_update->box, ctx->stream));
    if (mesh_count)  // the exact mesh gates (Scene.cs:67)
        HIP_OR_FAIL(ctx, hipMemcpyAsync(ctx->arr.gates, a.aabbs, sizeof(rtd::MeshGate) * (size_t)mesh_count,
                                        hipMemcpyDeviceToDevice, ctx->stream));
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev_x, ctx->stream));
    if (ctx->src.build == RT_BUILD_SAH_REFIT) return refit_update(ctx, t0);
    const int P = ctx->src.in.mt + ctx->src.in.ns + ctx->src.in.nl;
    LbvhBufs &L = ctx->lb;
    const bool wide = ctx->src.wide;
    if (P > 0) {
        rtl::LbvhInput in = ctx->src.in;
        in.box_dev = (const float *)B.scene_box.p;
        rtl::LbvhOutput out{};
        out.nodes = (rtd::BvhNode *)L.nodes.p;
        out.nodes4 = wide ? (rtd::BvhNode4 *)L.nodes4.p : nullptr;
        out.tris = (rtd::TriRec *)L.tris.p;
        out.sphs = (rtd::SphRec *)L.sphs.p;
        out.shade = (float4 *)L.shade.p;
        HIP_OR_FAIL(ctx, rtl::build_lbvh_gpu(in, out, L.scratch.p, L.scratch.cap, ctx->stream));
        HIP_OR_FAIL(ctx, hipMemcpyAsync(ctx->h_update->binfo, rtl::lbvh_info_ptr(L.scratch.p, P), 3 * sizeof(int),
                                        hipMemcpyDeviceToHost, ctx->stream));
        const int st = enqueue_cut(ctx);
        if (st) return st;
    }
    HIP_OR_FAIL(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    float xform_ms = 0.0f, build_ms = 0.0f;
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&xform_ms, ctx->ev0, ctx->ev_x));
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&build_ms, ctx->ev_x, ctx->ev1));
    const volatile float *hb = ctx->h_update->box;
    float box[7];
    for (int i = 0; i < 7; ++i) box[i] = hb[i];
    rtd::SceneDev &S = ctx->S;
    ctx->info.build_ms = xform_ms;
    if (P > 0) {
        const volatile int *bi = ctx->h_update->binfo;
        const int binfo[3] = {bi[0], bi[1], bi[2]};
        ctx->info.build_ms += build_ms;
        ctx->last_bvh_depth = wide ? binfo[2] : binfo[0];
        const int need = wide ? 3 * (binfo[2] + 1) : binfo[0] + 1;  // as run_lbvh
        if (need > rtd::kStackTotal) {
            ctx->has_scene = false;
            return fail(ctx, RT_E_SCENE, "LBVH %d-wide depth %d exceeds the traversal stack; use RT_BUILD_SAH_HOST",
                        wide ? 4 : 2, wide ? binfo[2] : binfo[0]);
        }
        ctx->info.nodes = wide ? binfo[1] : std::max(1, P - 1);
        for (int c = 0; c < 3; ++c) {
            ctx->src.in.scene_lo[c] = box[c];
            ctx->src.in.scene_hi[c] = box[3 + c];
        }
        ctx->src.in.pad_abs = box[6];
    }
    for (int c = 0; c < 3; ++c) {
        S.scene_lo[c] = box[c];
        S.scene_hi[c] = box[3 + c];
    }
    ctx->info.total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

}  // namespace

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
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
    for (const GroupSlot &g : ctx->gslots)
        for (size_t i = 1; g.used && i < g.member_stream.size(); ++i) {
            HIP_OR_FAIL(ctx, hipSetDevice(member(ctx, (int)i)->device));
            HIP_OR_FAIL(ctx, hipStreamSynchronize(g.member_stream[i]));
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
    HIP_OR_FAIL(ctx, hipMemcpyAsync(ctx->d_rays, rays, (size_t)n * sizeof(rt_ray), hipMemcpyHostToDevice,
                                    ctx->stream));
    HIP_OR_FAIL(ctx, rtk::launch_intersect(ctx->S, ctx->d_rays, n, ctx->d_hits, ctx->stream));
    std::vector<int4> hits((size_t)n);
    HIP_OR_FAIL(ctx, hipMemcpyAsync(hits.data(), ctx->d_hits, (size_t)n * sizeof(int4), hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_OR_FAIL(ctx, hipStreamSynchronize(ctx->stream));
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

}  // extern "C"
