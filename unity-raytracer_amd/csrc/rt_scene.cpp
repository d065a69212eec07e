// rt_scene.cpp — scenes: validation, Scene.CalculateAABB (Scene.cs:17-41),
// material deduplication, the host SAH build or the device LBVH, the HBM
// layout (rt_device.h), the top-level cut, device mesh extraction
// (SceneMesh.cs:11-53) and the per-Update refit / rebuild.
#include "rt_host.h"

namespace rti {

int warm_up(rt_ctx *ctx);

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
    const rti::Wait w("upload: hipMalloc + hipMemcpy");
    hipError_t e = hipMalloc(dst, v.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

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

template <typename T>
hipError_t put(rt_ctx *ctx, GrowBuf &b, const T *src, size_t count) {
    hipError_t e = ensure(ctx, b, count * sizeof(T));
    if (e != hipSuccess || count == 0) return e;
    const rti::Wait w("put: hipMemcpyAsync from pageable host memory");
    return hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    float ms = 0.0f;
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->info.build_ms += ms;
    int binfo[3] = {0, 0, 0};  // 2-wide depth, 4-wide node count, 4-wide depth
    HIP_WAIT(ctx, hipMemcpy(binfo, rtl::lbvh_info_ptr(B.scratch.p, P), sizeof(binfo), hipMemcpyDeviceToHost));
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
        HIP_WAIT(ctx, hipMemcpyAsync(aabbs.data(), B.src_aabbs.p, sizeof(rtd::MeshGate) * aabbs.size(),
                                        hipMemcpyDeviceToHost, ctx->stream));
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
    HIP_OR_FAIL(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    return RT_OK;
}


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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));

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
        HIP_WAIT(ctx, hipMemcpy(mtris.data(), B.mesh_tris.p, sizeof(rt_triangle) * (size_t)tt, hipMemcpyDeviceToHost));
        HIP_WAIT(ctx, hipMemcpy(mnorm.data(), B.mesh_normals.p, sizeof(rt_float3) * (size_t)tt,
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
    HIP_OR_FAIL(ctx, ensure(ctx, R.quality, 4 * sizeof(float)));  // + the fixed-point sum (scene_xform.hip)
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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
#ifdef RT_EXP_REFIT_REBUILD
        constexpr float limit = RT_EXP_REFIT_REBUILD;  // measuring builds (tools/exp/refit_sweep.sh)
#else
        constexpr float limit = kRefitRebuild;
#endif
        // a NaN quality (a degenerate or non-finite scene box: scene_xform.hip
        // quality_scale) keeps the tree — the refit stays exact, only a
        // measure of its speed is missing (it rebuilt every update)
        if (area > limit * R.area_built) {
            std::vector<rtd::MeshGate> aabbs((size_t)ctx->src.mesh_count);
            if (!aabbs.empty())
                HIP_WAIT(ctx, hipMemcpy(aabbs.data(), ctx->lb.src_aabbs.p, sizeof(rtd::MeshGate) * aabbs.size(),
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
    // the update rewrites the tree, the primitive records and the cut in
    // place: RT_FLAG_ASYNC frames still pending on other streams (rt_set_stream
    // between frames) must have ended first, not only this stream's
    if (ctx->async_frames > 0) {
        const int st = settle_async(ctx);
        if (st) return st;
    }
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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
    HIP_WAIT(ctx, hipStreamSynchronize(ctx->stream));
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

}  // namespace rti
