/*
 * rt_mi355.h — C-ABI of the MI355X (gfx950) trace path.
 *
 * This is the drop-in boundary for the per-pixel trace loop of
 * vectorized-runner/unity-raytracer (reference @ v1).  The reference has no
 * native code and no `Render(Scene, Camera)` method; its frame-level seam is
 *
 *     RayTracingSetup.CastPixelRays(CameraData)
 *         Assets/RayTracer/Demo-RayTracing/RayTracingSetup.cs:275-302
 *
 * which reads the implicit inputs `Scene` (Data/Objects/Scene.cs:8-15),
 * `ImagePlane` (:21), `BackgroundColor` (:22), `MaxReflectionBounces` (:23)
 * and writes `Color[] PixelColors` (:40).  The entry points below replace
 * that method (and, for batch ray queries, `Scene.IntersectRay`,
 * Data/Objects/Scene.cs:43-122).  A Unity C# host binds them with
 * [DllImport]; the stub is in INTEGRATION.md.
 *
 * Conventions
 *   - Plain C types only; every struct is blittable (C# bool → int32).
 *   - Every call returns 0 (RT_OK) or a negative rt_status; the message of
 *     the last failure is available from rt_last_error().  No C++ exception
 *     crosses this boundary.
 *   - Calls on one context are synchronous and not thread-safe (the
 *     reference calls CastPixelRays once per frame from Update() on Unity's
 *     main thread, RayTracingSetup.cs:171-199).
 *   - The caller owns every input array and output buffer; the library
 *     copies what it needs and retains no caller pointer.
 *   - All arithmetic is IEEE float32 with the operation order of the
 *     reference (see DESIGN.md "Arithmetic contract").
 */
#ifndef RT_MI355_H
#define RT_MI355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6

/* ---- status codes ------------------------------------------------------ */
typedef enum rt_status {
    RT_OK = 0,
    RT_E_INVALID = -1,   /* bad argument (null pointer, negative size, spp not n*n ...)   */
    RT_E_SCENE = -2,     /* malformed scene (index out of range, mesh range overflow ...) */
    RT_E_HIP = -3,       /* a HIP runtime call failed (message carries hipGetErrorString) */
    RT_E_NO_DEVICE = -4, /* no gfx950 device visible                                      */
    RT_E_STATE = -5,     /* call order (e.g. rt_render before rt_set_scene)                */
    RT_E_INTERNAL = -6   /* internal invariant broken; reference analog: the
                            ArgumentOutOfRangeException of a None hit type,
                            RayTracingSetup.cs:432-434                              */
} rt_status;

/* ---- POD types mirroring the reference's structs ----------------------- */

/* Unity.Mathematics.float3 */
typedef struct rt_float3 { float x, y, z; } rt_float3;

/* Triangle, Data/Objects/Triangle.cs:7-11 (36 B) */
typedef struct rt_triangle { rt_float3 vertex0, vertex1, vertex2; } rt_triangle;

/* Sphere, Data/Objects/Sphere.cs:7-10 (16 B) — stores the SQUARED radius */
typedef struct rt_sphere { rt_float3 center; float radius_squared; } rt_sphere;

/* AABB, Data/Collision/AABB.cs:5-8 (24 B) */
typedef struct rt_aabb { rt_float3 min, max; } rt_aabb;

/* MaterialData, Data/Shading/MaterialData.cs:7-15 (56 B; C# bool → int32) */
typedef struct rt_material {
    rt_float3 diffuse_reflectance;
    rt_float3 ambient_reflectance;
    rt_float3 mirror_reflectance;
    rt_float3 specular_reflectance;
    float phong_exponent;
    int32_t is_mirror;
} rt_material;

/* PointLightData, Data/Lights/PointLightData.cs:7-11 (24 B) */
typedef struct rt_point_light { rt_float3 position, intensity; } rt_point_light;

/* CameraData, Data/Camera/CameraData.cs:5-11 (48 B).  Forward/Right/Up are
 * the already-normalised basis built in RayTracingSetup.Update() :175-181. */
typedef struct rt_camera { rt_float3 position, forward, right, up; } rt_camera;

/* ImagePlane, Data/Camera/ImagePlane.cs:11-45 (Resolution inlined, 20 B) */
typedef struct rt_image_plane {
    int32_t resolution_x, resolution_y;
    float distance_to_camera;
    float half_horizontal_length;
    float half_vertical_length;
} rt_image_plane;

/* Mesh, Data/Objects/Mesh.cs:7-13, flattened: its Triangles[] and
 * TriangleNormals[] are the range [first_triangle, first_triangle +
 * triangle_count) of rt_scene_desc.mesh_triangles / mesh_triangle_normals. */
typedef struct rt_mesh {
    int32_t first_triangle;
    int32_t triangle_count;
    rt_material material;
    rt_aabb aabb;   /* Mesh.AABB over ALL transformed vertices, SceneMesh.cs:22-31 */
} rt_mesh;

/* Scene, Data/Objects/Scene.cs:8-15.  Order inside every array is the order
 * of the reference's List<>s and fixes the closest-hit tie winner
 * (meshes by index then triangle index, then spheres, then loose
 * triangles; first wins, Scene.cs:75,93,108). */
typedef struct rt_scene_desc {
    /* TriangleData, Data/Objects/TriangleData.cs:8-13 */
    const rt_triangle *triangles;
    const rt_float3 *triangle_normals;      /* Triangle.Normal, Triangle.cs:13-21   */
    const rt_material *triangle_materials;
    int32_t triangle_count;
    /* MeshData, Data/Objects/MeshData.cs:7-9 */
    const rt_triangle *mesh_triangles;
    const rt_float3 *mesh_triangle_normals; /* -Triangle.Normal, SceneMesh.cs:43    */
    int32_t mesh_triangle_total;
    const rt_mesh *meshes;
    int32_t mesh_count;
    /* SphereData, Data/Objects/SphereData.cs:7-10 */
    const rt_sphere *spheres;
    const rt_material *sphere_materials;
    int32_t sphere_count;
    /* PointLights / AmbientLight, Scene.cs:12-13 */
    const rt_point_light *point_lights;
    int32_t point_light_count;
    rt_float3 ambient_radiance;             /* AmbientLightData.Radiance            */
} rt_scene_desc;

/* Frame parameters: the serialized fields of RayTracingSetup (:22-23) plus
 * the build's documented extensions (DESIGN.md "Extensions"). */
typedef struct rt_render_params {
    float background_color[4];      /* UnityEngine.Color (0..1); alpha ignored, Rgb.cs:15-18 */
    int32_t max_reflection_bounces; /* MaxReflectionBounces (:23)                  */
    int32_t samples_per_pixel;      /* n*n stratified samples; 1 == reference        */
    int32_t band_index;             /* block-cyclic row sharding: this shard          */
    int32_t band_count;             /*   number of shards (1 = whole image)           */
    int32_t band_rows;              /*   rows per block (0 → 8)                       */
    int32_t flags;                  /* RT_FLAG_*                                      */
} rt_render_params;

#define RT_FLAG_COUNT_TESTS 1   /* fill rt_stats box/triangle/sphere counters (slower) */
#define RT_FLAG_WAVEFRONT   2   /* per-level wavefront passes instead of the default megakernel */
#define RT_FLAG_PACKET      4   /* wave-synchronous megakernel with per-wave packet traversal */
/* Output pixel format (default: float RGBA = the reference's Color, 16 B).
 * Encoding happens in the render kernel's final store, so the HBM write,
 * the shard gather and the D2H copy shrink 4x / 2x. */
#define RT_FLAG_OUT_RGBA8   8   /* Color32: round-half-even(clamp01(c) * 255), alpha 255; 4 B */
#define RT_FLAG_OUT_RGBA16F 16  /* IEEE half RGBA (round to nearest even), alpha 1, unclamped; 8 B */
/* Float RGB without the constant alpha (Rgb.Color's a is always 1): the
 * Color values bit for bit in 12 B — a shard transport format that cuts the
 * framebuffer gather by a quarter. */
#define RT_FLAG_OUT_RGB32F  128
/* rt_render_device only: enqueue the frame on the context's stream and return
 * without waiting (a frame loop that keeps the GPU fed; switching the stream
 * with rt_set_stream between frames lets consecutive frames overlap).  The
 * stats argument is zeroed; rt_finish waits for the device and returns the
 * counters and device time of all asynchronous frames since the previous
 * rt_finish.  The first frame of a (stream, layout) waits once for the
 * device after its launch: its measured longest-first order's sky tail is
 * read back (frames in flight beside it render that tail in batches). */
#define RT_FLAG_ASYNC       32
/* Megakernel frames normally dispatch their tiles longest-first, ordered by
 * the per-tile cost an earlier frame of the same layout and scene measured on
 * the same stream (the frame's tail is its slowest tiles; re-measured every
 * few frames).  This flag keeps row-major order.  Results never depend on the
 * order. */
#define RT_FLAG_ROW_ORDER   64
/* Camera packets start at the root instead of below the tree's top-level cut
 * (DESIGN.md §5): the reference ordering of node visits, for testing that the
 * cut changes no result.  Results never depend on it. */
#define RT_FLAG_NO_CUT      256

/* Work counters and timings of the last render. */
typedef struct rt_stats {
    uint64_t primary_rays;     /* camera samples traced                          */
    uint64_t shadow_rays;      /* one per (hit, point light), :327-333           */
    uint64_t reflection_rays;  /* mirror bounces, :358-363                        */
    uint64_t box_tests;        /* BVH node/AABB slab tests   (RT_FLAG_COUNT_TESTS) */
    uint64_t triangle_tests;   /* Möller–Trumbore tests      (RT_FLAG_COUNT_TESTS) */
    uint64_t sphere_tests;     /* ray/sphere tests           (RT_FLAG_COUNT_TESTS) */
    uint64_t shading_fetches;  /* closest hits shaded (normal + material fetch)    */
    double kernel_ms;          /* device time of the trace kernel(s); a multi-GPU
                                  frame: the slowest device's                      */
    double total_ms;           /* wall time of the whole call                     */
    uint64_t primary_scene_misses; /* camera samples rejected by the Scene.AABB gate
                                      (Scene.cs:54) before any object test
                                      (RT_FLAG_COUNT_TESTS frames of the default
                                      megakernel path only; 0 when the frame also
                                      sets RT_FLAG_PACKET or RT_FLAG_WAVEFRONT)      */
    uint64_t shadow_rays_moot; /* shadow rays (counted in shadow_rays) whose answer
                                  cannot change the pixel — the light's unoccluded
                                  term leaves the colour's bits unchanged, e.g. a
                                  light behind the surface — so they were not
                                  traversed (0 in RT_FLAG_COUNT_TESTS frames).
                                  Which moot rays are skipped depends on how the
                                  frame was dispatched: every packet traversal
                                  skips them, the per-lane mirror chains only in
                                  split tiles — so a frame that splits its slowest
                                  tiles may report more than the same frame
                                  unsplit; pixels and every other count are
                                  the same                                         */
} rt_stats;

/* Closest-hit record, IntersectionResult (Data/Collision/IntersectionResult.cs:3-7)
 * with ObjectId (Data/Objects/ObjectId.cs:5-9) inlined.  type: 0 None,
 * 1 Sphere, 2 Triangle, 3 MeshTriangle (ObjectType.cs:3-9). */
typedef struct rt_hit {
    int32_t type;
    int32_t index;
    int32_t mesh_index;
    float distance;
} rt_hit;

/* Ray, Data/Collision/Ray.cs:7-10 (24 B) */
typedef struct rt_ray { rt_float3 origin, direction; } rt_ray;

/* ---- entry points ------------------------------------------------------- */

typedef struct rt_ctx rt_ctx;

/* ABI version of the loaded library (== RT_ABI_VERSION it was built with). */
int32_t rt_abi_version(void);

/* Create a context.  num_gpus == 1: on the calling thread's current HIP
 * device.  num_gpus == N > 1: one context driving devices 0..N-1 of this
 * process from the calling thread (a Unity-loaded .so cannot launch one
 * process per GPU): the scene is replicated on every device
 * and each rt_render / rt_render_device frame is split into block-cyclic
 * row bands (8-row blocks, block b -> device b mod N, the pixels are
 * independent: RayTracingSetup.cs:288-301), rendered concurrently, gathered
 * to device 0 over xGMI by RCCL (ncclSend/ncclRecv in one group; peer copies
 * when RCCL is unavailable), put back in row order on device 0 and, for
 * rt_render, copied to the caller's Color[].  Frames are bit-identical to a
 * one-device frame. */
int rt_create(rt_ctx **out_ctx, int32_t num_gpus);

/* Transport of a multi-device context's band gather. */
#define RT_GATHER_NONE 0       /* one device                                            */
#define RT_GATHER_PEER_COPY 1  /* hipMemcpyPeerAsync from every device into device 0   */
#define RT_GATHER_RCCL 2       /* ncclSend/ncclRecv (one ncclGroupStart/End per frame)   */

/* rt_create with an explicit device list (devices[0] is the root that
 * receives the frame).  A device may appear more than once: its entries are
 * separate logical shards on that GPU (testing the multi-device path on one
 * GPU; the gather then uses peer copies).  gather: RT_GATHER_RCCL (default
 * for distinct devices when 0 is passed) or RT_GATHER_PEER_COPY.  With
 * RT_GATHER_RCCL even a one-device context routes its band through an RCCL
 * self send/receive. */
int rt_create_devices(rt_ctx **out_ctx, const int32_t *devices, int32_t num_devices, int32_t gather);

/* What a context drives. */
typedef struct rt_device_info {
    int32_t num_devices;      /* members (shards per frame)                    */
    int32_t gather;           /* RT_GATHER_*                                   */
    int32_t devices[16];      /* HIP device ids of the first 16 members         */
} rt_device_info;

int rt_get_device_info(const rt_ctx *ctx, rt_device_info *info);

/* Destroy a context (null is a no-op). */
void rt_destroy(rt_ctx *ctx);

/* Message of the last failed call on ctx (or of the last failed rt_create
 * when ctx is null).  Never null; valid until the next call on ctx. */
const char *rt_last_error(const rt_ctx *ctx);

/* Use this HIP stream (hipStream_t passed as void*) for all device work
 * (a multi-device context: device 0's work; the other devices use streams of
 * their own, one per stream device 0 is given, so frames in flight stay
 * independent);
 * null selects the context's own stream (created non-blocking, so NOT the
 * legacy null stream: a caller working on the null stream — e.g. torch's
 * default stream, whose handle is 0 — must pass a created stream to order
 * its own work with the library's). */
int rt_set_stream(rt_ctx *ctx, void *hip_stream);

/* Upload a scene: copies every array to HBM, computes Scene.AABB exactly as
 * Scene.CalculateAABB (Scene.cs:17-41) and builds the BVH — on the device
 * (RT_BUILD_LBVH_GPU; the host SAH when that tree would be too deep for the
 * traversal stack).  Replaces RayTracingSetup.UpdateScene()'s result
 * (:120-128).  rt_set_scene_ex chooses the builder. */
int rt_set_scene(rt_ctx *ctx, const rt_scene_desc *scene);

/* BVH builders for rt_set_scene_ex. */
#define RT_BUILD_SAH_HOST 0   /* binned SAH on the host, collapsed to 4-wide nodes */
#define RT_BUILD_LBVH_GPU 1   /* linear BVH built on the GPU (Morton + radix sort + Karras), collapsed
                                 to 4-wide nodes on the GPU (rt_set_scene's default; also for
                                 per-frame scene rebuilds, RayTracingSetup.cs:120-128) */
#define RT_BUILD_LBVH_GPU_BVH2 2  /* the same tree left 2-wide (comparison / diagnostics) */
#define RT_BUILD_SAH_REFIT 3  /* rt_set_scene_source_ex only: the host SAH tree once, then every
                                 rt_update_mesh_transforms refits it on the device (same topology and
                                 leaf order, new boxes) and rebuilds it only when the refitted tree's
                                 surface area has grown past 1.1x that of its last build
                                 (then on the device: the GPU LBVH, refitted from there on) */

/* rt_set_scene with a choice of BVH builder.  Results are identical for every
 * builder (the BVH only accelerates Scene.IntersectRay). */
int rt_set_scene_ex(rt_ctx *ctx, const rt_scene_desc *scene, int32_t build);

/* What the last rt_set_scene(_ex) built. */
typedef struct rt_scene_info {
    int32_t build;       /* RT_BUILD_* */
    int32_t bvh_width;   /* 4 or 2 (0: empty scene) */
    int32_t nodes;
    int32_t primitives;
    double build_ms;     /* device time of the GPU build (RT_BUILD_LBVH_GPU), else 0 */
    double total_ms;     /* wall time of the whole rt_set_scene(_ex) call */
} rt_scene_info;

int rt_get_scene_info(const rt_ctx *ctx, rt_scene_info *info);

/* Inspection: the scene's 4-wide BVH exactly as it lies in HBM — 128-B nodes
 * (child boxes plane by plane, child refs: >= 0 node, < 0 inline leaf
 * ~(first | (count-1) << 27 | kind << 29)), 48-B triangle records in leaf
 * order (v0, v1 - v0, v2 - v0, reference rank, mesh gate; one sentinel record
 * last), 32-B sphere records (center, r^2, rank) — copied into caller
 * buffers.  For tools and the CPU baseline that traverses the very tree the
 * GPU does (bench.py cpu_baseline).  Null buffers: only *info is filled.
 * RT_E_STATE without a scene or for a 2-wide (RT_BUILD_LBVH_GPU_BVH2) tree. */
typedef struct rt_bvh_export_info {
    int32_t nodes;           /* 128-B node records   */
    int32_t triangle_records;/* 48-B triangle records (incl. the sentinel) */
    int32_t sphere_records;  /* 32-B sphere records  */
    int32_t reserved;
} rt_bvh_export_info;

int rt_export_bvh(const rt_ctx *ctx, void *nodes, void *triangle_records, void *sphere_records,
                  rt_bvh_export_info *info);

/* One mesh as the reference holds it before extraction: SceneMesh's
 * MeshFilter.sharedMesh (vertices, index buffer) and Transform
 * (SceneMesh.cs:11-53).  The device applies localToWorldMatrix with
 * MultiplyPoint3x4, takes Mesh.AABB over all transformed vertices, builds the
 * triangles in index-buffer order and their normals (-Triangle.Normal). */
typedef struct rt_mesh_source {
    const rt_float3 *vertices;  /* local space, vertex_count */
    int32_t vertex_count;
    const int32_t *indices;     /* triangle list, index_count = 3 x triangles, each in [0, vertex_count) */
    int32_t index_count;
    float local_to_world[16];   /* Transform.localToWorldMatrix, row-major: m[row * 4 + col] */
    rt_material material;       /* SceneMesh.MaterialData */
} rt_mesh_source;

/* Scene whose meshes are extracted on the device (the replacement of
 * UpdateScene's per-frame FetchMeshes, RayTracingSetup.cs:120-128,159-169).
 * `base` carries the loose triangles, spheres, point lights and ambient light;
 * its mesh fields must be empty.  Vertices and index buffers stay resident on
 * the device; the BVH is built on the device (RT_BUILD_LBVH_GPU).  Results
 * equal rt_set_scene with the same meshes extracted on the host. */
int rt_set_scene_source(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count);

/* rt_set_scene_source with a choice of per-update BVH strategy: build =
 * RT_BUILD_LBVH_GPU (rt_set_scene_source's: a device rebuild every update) or
 * RT_BUILD_SAH_REFIT (a host SAH build here — tens of ms for 100k triangles —
 * then device refits; for rigid per-mesh motion, the Unity Update case).
 * Results are identical either way. */
int rt_set_scene_source_ex(rt_ctx *ctx, const rt_scene_desc *base, const rt_mesh_source *meshes, int32_t mesh_count,
                           int32_t build);

/* Per-frame update of a scene set by rt_set_scene_source: new
 * localToWorld matrices (mesh_count x 16 floats, rt_mesh_source layout),
 * re-extraction and BVH rebuild on the device.  Only the matrices cross
 * PCIe. */
int rt_update_mesh_transforms(rt_ctx *ctx, const float *local_to_world, int32_t mesh_count);

/* Render one frame: the MI355X replacement of CastPixelRays (:275-302).
 * out_rgba is a caller-owned HOST buffer of resolution_x*resolution_y pixels
 * of rt_pixel_bytes(flags) bytes — by default 4 floats (row-major, y = 0 is
 * the top row, alpha = 1), i.e. PixelColors.  When band_count > 1, only this
 * shard's rows are rendered and out_rgba receives the shard's compact
 * buffer (rt_band_rows_local rows); on a multi-device context such a frame
 * runs on device 0 only.  Copy-bound formats (float RGBA frames of 2 MB or
 * more) overlap the device-to-host copy with the rendering: row slabs
 * alternating over two streams, each finished slab copied while later slabs
 * render; other frames render in one piece with the copy right behind. */
int rt_render(rt_ctx *ctx, const rt_camera *camera, const rt_image_plane *plane,
              const rt_render_params *params, void *out_rgba, rt_stats *stats);

/* Waits for the asynchronous frames (RT_FLAG_ASYNC) and returns their summed
 * counters; kernel_ms is their summed device time, total_ms the wall time
 * since the first of them was enqueued. */
int rt_finish(rt_ctx *ctx, rt_stats *stats);

/* Bytes per output pixel for rt_render_params.flags: 16, 12, 8 or 4. */
int32_t rt_pixel_bytes(int32_t flags);

/* Same as rt_render but the output stays in HBM: d_out_rgba is a DEVICE
 * pointer on the context's GPU of at least out_bytes bytes.  The call
 * returns after the frame is complete on the device. */
int rt_render_device(rt_ctx *ctx, const rt_camera *camera, const rt_image_plane *plane,
                     const rt_render_params *params, void *d_out_rgba, size_t out_bytes,
                     rt_stats *stats);

/* Up to RT_MAX_BATCH frames of one layout (plane, params) from their own
 * cameras, as one device launch: the throughput path for frames in flight
 * whose frames are small — e.g. the frames of one gather group of a rank's
 * row band (band_count > 1), each far too small to fill the GPU alone.  Frame
 * i is rendered exactly as rt_render_device(cameras[i]) would render it (same
 * bits, same ray counts; the stats are summed) into the device buffer at
 * d_out + i * frame_stride_bytes (frame_stride_bytes >= one frame's bytes).
 * The frames' tiles form one longest-first order, so one frame's slowest tiles
 * overlap the others' work.  RT_FLAG_ASYNC as for rt_render_device.  Frames
 * the batch launch does not cover (other than 4 spp, MaxReflectionBounces >
 * 32, RT_FLAG_COUNT_TESTS / _WAVEFRONT / _PACKET, multi-device contexts) are
 * rendered one by one with the same results.  No reference counterpart:
 * RayTracingSetup.Update (RayTracingSetup.cs:171-199) renders one frame per
 * call. */
#define RT_MAX_BATCH 8
int rt_render_device_batch(rt_ctx *ctx, int32_t num_frames, const rt_camera *cameras,
                           const rt_image_plane *plane, const rt_render_params *params, void *d_out,
                           size_t frame_stride_bytes, rt_stats *stats);

/* Rows of the compact per-shard buffer for (resolution_y, band_index,
 * band_count, band_rows): the same for every shard, so the last shards of a
 * ragged split end in padding rows (blocks past the image).  Padding rows
 * are not part of the image: no render writes them (rt_render's host buffer
 * may hold whatever the device buffer held) and rt_assemble_bands skips them. */
int32_t rt_band_rows_local(int32_t resolution_y, int32_t band_index, int32_t band_count,
                           int32_t band_rows);

/* Reassemble an image from band_count gathered shard buffers laid out
 * back to back (each rt_band_rows_local(max) rows, padded) into row order.
 * Both pointers are DEVICE pointers on the context's GPU. */
int rt_assemble_bands(rt_ctx *ctx, const float *d_gathered, int32_t resolution_x,
                      int32_t resolution_y, int32_t band_count, int32_t band_rows,
                      float *d_image);

/* rt_assemble_bands for any output format: pixel_bytes = rt_pixel_bytes(flags).
 * Stream-ordered: returns once the kernel is enqueued on the context's stream
 * (rt_assemble_bands waits for it). */
int rt_assemble_bands_ex(rt_ctx *ctx, const void *d_gathered, int32_t resolution_x,
                         int32_t resolution_y, int32_t band_count, int32_t band_rows,
                         int32_t pixel_bytes, void *d_image);

/* Waits for all work enqueued on the context's stream. */
int rt_synchronize(rt_ctx *ctx);

/* Batch closest-hit query: Scene.IntersectRay (Scene.cs:43-122) for n host
 * rays; writes n host rt_hit records. */
int rt_intersect_rays(rt_ctx *ctx, const rt_ray *rays, int32_t n, rt_hit *out_hits);

/* Diagnostic: the float threshold T with  d < T  <=>  degrees(acos(d)) > 90f
 * (RayTracingSetup.cs:384-392), which the kernels use instead of acos so the
 * discrete specular branch matches the host libm bit for bit. */
float rt_spec_threshold(void);

/* Testing only (fault injection; no reference counterpart): what = 
 * RT_DEBUG_FAIL_SLAB makes rt_render's host-output pipeline fail before row
 * slab `value` (-1: off), so the error path's cleanup — every copy posted
 * for the earlier slabs finished before rt_render returns — can be tested. */
#define RT_DEBUG_FAIL_SLAB 1
/* Measuring only: RT_DEBUG_WAVE_CLOCKS (value 1: on, 0: off) makes every
 * render_kernel launch record, per wave, its start and duration on the GPU's
 * constant 100 MHz clock; rt_debug_read(ctx, RT_DEBUG_WAVE_CLOCKS, ...) returns
 * the last launch's records (waits for the device).  A record is 4 uint32:
 * start (low, high word), duration, tile | (part + 1) << 24 (part: -1 whole
 * tile, else the split tile's quarter / sixteenth); a zero record is a wave
 * slot that did no tile.  The product build does not record (RT_E_STATE); a
 * measuring build is compiled with -DRT_WAVE_CLOCK.  One
 * frame in flight at a time: every launch overwrites the records. */
#define RT_DEBUG_WAVE_CLOCKS 2
/* Testing only: RT_DEBUG_GROUP_SAMPLE_WAVES (value 0: off, 1: on, the
 * default) — whether the bands of this multi-device context's frames may run
 * a lone band's slowest pixels as one-sample waves (rt_frame.cpp
 * lpt_prepare), as a single-device frame's small shards do; the stall probe
 * (tools/stall_probe.py) and A/B runs switch it. */
#define RT_DEBUG_GROUP_SAMPLE_WAVES 3
/* Diagnostics: rt_debug_read(ctx, RT_DEBUG_HOST_WAITS, out, cap, &n) writes
 * a text report (NUL-terminated, truncated to cap) of every host thread that
 * is inside one of the library's blocking runtime calls right now (the call,
 * its device and for how long) and, for a non-NULL ctx, whether each stream of
 * the context and its members still has work pending.  Safe to call from
 * another thread while a call of the context is blocked; ctx may be NULL. */
#define RT_DEBUG_HOST_WAITS 4
/* Diagnostics: rt_debug_read(ctx, RT_DEBUG_LAST_LAUNCH, out, cap, &n) writes
 * the kernel instance the context's last render launch ran and its split
 * shape (tiles, split16 / split tiles, one-sample shift, rows, band), as
 * NUL-terminated text — which instance a frame took (tests, bench.py). */
#define RT_DEBUG_LAST_LAUNCH 5
/* Testing only: RT_DEBUG_SAMPLE_WAVE_STACK (value n >= 0; 0, the default:
 * the whole area) limits the one-sample waves' whole-wave traversal to n
 * stack entries for its 16-entries-a-step wide steps; above that it walks
 * depth-first, one entry a step (csrc/coop.h) — a small n exercises that
 * mode (same answers either way). */
#define RT_DEBUG_SAMPLE_WAVE_STACK 6
/* Diagnostics: rt_debug_read(ctx, RT_DEBUG_COUNTERS, out, cap, &n) writes the
 * 16 64-bit counter words of the last synchronous frame or rt_finish (words
 * 0-8: rt_stats' counts; word 9: in a -DRT_FETCH_COUNT measuring build, the
 * bytes those frames' traversal and shading requested; 0 otherwise). */
#define RT_DEBUG_COUNTERS 7
int rt_debug_set(rt_ctx *ctx, int32_t what, int32_t value);
int rt_debug_read(rt_ctx *ctx, int32_t what, void *out, int64_t capacity_bytes, int64_t *bytes_written);

#ifdef __cplusplus
}
#endif

#endif /* RT_MI355_H */
