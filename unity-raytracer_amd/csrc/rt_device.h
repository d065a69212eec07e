// rt_device.h — HBM layout of an uploaded scene and the kernel parameter
// blocks.  Shared by the host (rt_abi.cpp, bvh.cpp) and the kernels.
//
// Layout (DESIGN.md "Data layout in HBM"):
//   nodes   BvhNode[]   64 B  BVH2 node holding BOTH children's boxes (one
//                             coalesced 64-B fetch tests two boxes)
//   leaves  LeafDesc[]  16 B  {first, count, kind, gate}
//   tris    TriRec[]    48 B  v0, edge1, edge2, rank — leaf order (Möller–
//                             Trumbore inputs only; 3 x 16-B loads)
//   sphs    SphRec[]    32 B  center, r^2, rank — leaf order
//   shade   float4[]    16 B  per reference rank: normal (or sphere center),
//                             material id — fetched once per shaded hit
//   mats    DevMaterial 64 B  deduplicated MaterialData
//   lights  DevLight    32 B
//   gates   MeshGate    32 B  exact (unpadded) Mesh.AABB of every mesh
// A "rank" is the primitive's position in the reference's scan order
// (Scene.cs:64-115): mesh triangles (mesh by mesh), then spheres, then loose
// triangles.  Equal distances resolve to the lowest rank, which is exactly
// the reference's "first wins" (strict '>', Scene.cs:75,93,108).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace rtd {

// LDS traversal stack entries per lane (deeper entries: the private
// overflow).  16 keeps a one-wave workgroup of the megakernel at 4.8 KB of
// LDS, so six waves per SIMD fit a CU (trace.hip kMkMinWaves); 24 capped it
// at 23 waves per CU.  Only per-lane traversals use it (mirror chains, the
// counting launch, rt_intersect_rays).
#ifdef RT_EXP_STACK
constexpr int kStackSize = RT_EXP_STACK;  // measuring builds only
#else
constexpr int kStackSize = 16;
#endif
constexpr int kStackTotal = 128;         // + private (scratch) overflow: >= 3 * BVH4 depth, >= LBVH depth
constexpr int kMaxTreeDepth = 31;         // builder guarantees BVH2 internal depth <= 31
constexpr int kMaxBounces = 32;     // per-lane mirror fold stack
constexpr int kWaveSize = 64;
constexpr int kBlockThreads = 256;  // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlockThreads / kWaveSize;

// Ray/test counters are sharded: slot = block % kCounterSlots, 8 x u64 (one
// 64-B line) per slot; the host sums the slots.  One shared word would
// serialise every wave's atomics (a single word saturates near 88 atomics/us).
constexpr int kCounterSlots = 256;
constexpr int kCounterWords = 16;  // one 128-B slot: words 0-8 used (rt_stats order)

constexpr int kHintLights = 4;  // lights whose first shadow packets keep an occluder hint (FrameDev::shadow_hint)

constexpr int kLeafTri = 0;
constexpr int kLeafSphere = 1;

// Output pixel formats (rt_render_params.flags RT_FLAG_OUT_*).
constexpr int kOutFloat4 = 0;   // Color, 16 B (the reference's Color[])
constexpr int kOutRGBA8 = 1;    // Color32, 4 B
constexpr int kOutRGBA16F = 2;  // half RGBA, 8 B
constexpr int kOutRGB32F = 3;   // float RGB (alpha 1 implied), 12 B

struct alignas(16) BvhNode {
    float4 a;  // child0 lo.x, hi.x, lo.y, hi.y
    float4 b;  // child1 lo.x, hi.x, lo.y, hi.y
    float4 c;  // child0 lo.z, hi.z, child1 lo.z, hi.z
    int4 d;    // child0, child1 (>= 0 internal node, < 0 inline leaf ref), unused
};

// 4-wide node (BVH2 collapsed, 128 B = one L2 line): the four child boxes
// stored plane by plane so one lane tests four boxes from 6 float4 loads.
// Child refs: >= 0 internal node; < 0 leaf, ~ref = first | (count-1) << 27 |
// kind << 29 (first indexes tris[] or sphs[]); empty slots have +inf boxes.
struct alignas(16) BvhNode4 {
    float4 lox, hix, loy, hiy, loz, hiz;
    int4 child;
    int4 pad;
};

constexpr int kLeafFirstBits = 27;
__host__ __device__ __forceinline__ int encode_leaf(int first, int count, int kind) {
    return ~(first | ((count - 1) << kLeafFirstBits) | (kind << (kLeafFirstBits + 2)));
}

struct alignas(16) LeafDesc {
    int first;  // into tris[] or sphs[]
    int count;
    int kind;   // kLeafTri / kLeafSphere
    int gate;   // mesh index whose exact AABB gates this leaf, -1 = none
};

struct alignas(16) TriRec {
    float4 p0;  // v0.x v0.y v0.z e1.x
    float4 p1;  // e1.y e1.z e2.x e2.y
    float4 p2;  // e2.z rank(bits) gate(bits: mesh index or -1) -
};

// Every scene's triangle array ends with a sentinel record: all-zero edges
// and gate -1, so Moller-Trumbore rejects it for every ray (det == 0, or NaN
// for a NaN ray).  Unused BVH child slots (+inf boxes) point at it: a NaN or
// zero-direction ray that "enters" such a slot reaches a harmless leaf
// instead of cycling back to the root.
__host__ __device__ __forceinline__ TriRec sentinel_tri() {
    TriRec t;
    t.p0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    t.p1 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int rank = 0x7fffffff, gate = -1;
    float rb, gb;
    __builtin_memcpy(&rb, &rank, 4);
    __builtin_memcpy(&gb, &gate, 4);
    t.p2 = make_float4(0.0f, rb, gb, 0.0f);
    return t;
}

struct alignas(16) SphRec {
    float4 cr;  // center.xyz, radius_squared
    int4 misc;  // rank, gate (-1), -, -
};

struct alignas(16) DevMaterial {
    float4 kd_phong;   // DiffuseReflectance.xyz, PhongExponent
    float4 ka_mirror;  // AmbientReflectance.xyz, IsMirror (0/1 as float)
    float4 km;         // MirrorReflectance.xyz, -
    float4 ks;         // SpecularReflectance.xyz, 1 = specular term is always +-0 (pow skipped)
};

struct alignas(16) DevLight {
    float4 pos;        // Position.xyz
    float4 intensity;  // Intensity.xyz
};

struct alignas(16) MeshGate {
    float4 lo;
    float4 hi;
};

// A cut of the 4-wide tree: up to kCutMax subtrees (internal nodes or leaf
// refs) such that every leaf lies below exactly one of them, with their padded
// boxes (SoA, one entry per lane).  A camera packet starts from the entries
// its tile's frustum touches instead of walking the top levels node by node
// (packet.h cut_start).  Built on the device from nodes4 after every tree
// change (trace.hip build_cut_kernel); count 0 = no cut (start at the root).
constexpr int kCutMax = 64;
struct CutBox {  // one entry whole (32 B): the popped-marker test's scalar loads
    float4 lo;     // lo.xyz, ref (bits)
    float4 hi;     // hi.xyz, -
};
struct CutTable {
    float lo_x[kCutMax], lo_y[kCutMax], lo_z[kCutMax];
    float hi_x[kCutMax], hi_y[kCutMax], hi_z[kCutMax];
    int ref[kCutMax];
    int count;
    int pad[3];
    CutBox box[kCutMax];
};

// Everything a kernel needs to read the scene.
struct SceneDev {
    const BvhNode *nodes;
    const BvhNode4 *nodes4;
    const LeafDesc *leaves;
    const TriRec *tris;
    const SphRec *sphs;
    const float4 *shade;
    const DevMaterial *mats;
    const DevLight *lights;
    const MeshGate *gates;
    int num_lights;
    int mesh_tri_total;  // ranks [0, mesh_tri_total) are mesh triangles
    int sphere_count;    // ranks [mesh_tri_total, +sphere_count) are spheres
    int has_prims;       // 0 → every ray misses after the scene gate
    int bvh4;            // 1: nodes4 (host SAH build), 0: nodes (BVH2, GPU LBVH build)
    float scene_lo[3];   // Scene.AABB (Scene.CalculateAABB)
    float scene_hi[3];
    float ambient[3];    // AmbientLight.Radiance
    float spec_threshold;  // d < spec_threshold  <=>  degrees(acos(d)) > 90f
    const CutTable *cut;   // bvh4 scenes: the top-level cut (null: none)
};

// Longest-first dispatch key of one tile (render_kernel): its shader-clock
// cost on a log scale (4 mantissa bits, < 512, one cheap radix-sort pass set).
// A tile split into 64 >> pshift parts is measured on its first part and
// charged that part's cost times the number of parts.
__host__ __device__ __forceinline__ unsigned tile_cost_key(unsigned long long c64, int part, int pshift) {
    if (part == 0) c64 <<= 6 - pshift;  // parts = 64 >> pshift
    const unsigned c = (unsigned)(c64 < 0xffffffffull ? c64 : 0xffffffffull);
    const unsigned e = c ? 31u - (unsigned)__builtin_clz(c) : 0u;  // floor(log2 c)
    return e < 4 ? c : (((e - 3u) << 4) | ((c >> (e - 4u)) & 15u));
}

// Camera samples a launch of F traces: every pixel of its rows that lies in
// the image (slot_pixel's test), spp samples each.
__host__ __device__ inline unsigned long long active_samples(int res_x, int res_y, int local_rows, int row0,
                                                             int band_index, int band_count, int band_rows,
                                                             int spp) {
    long long rows = 0;
    if (band_count > 1) {
        for (int ly = 0; ly < local_rows; ly += band_rows) {
            const int blk = ly / band_rows;
            const long long gy0 = ((long long)blk * band_count + band_index) * band_rows;
            const long long n = (long long)(local_rows - ly < band_rows ? local_rows - ly : band_rows);
            rows += gy0 >= res_y ? 0 : (gy0 + n <= res_y ? n : res_y - gy0);
        }
    } else {
        const long long end = (long long)row0 + local_rows;
        rows = end <= res_y ? local_rows : (row0 < res_y ? res_y - row0 : 0);
    }
    return (unsigned long long)(rows > 0 ? rows : 0) * (unsigned long long)(res_x > 0 ? res_x : 0) * spp;
}

// Per-frame constants of CastPixelRays (RayTracingSetup.cs:277-284).
struct FrameDev {
    float cam_pos[3];
    float right[3];
    float up[3];
    float top_left[3];       // ImagePlane.GetRect(camera).TopLeft
    float hl, vl;            // HorizontalLength, VerticalLength
    float bg255[3];          // new Rgb(BackgroundColor).Value
    int res_x, res_y;
    int spp, spp_n;          // samples per pixel = spp_n * spp_n
    int max_bounces;
    int band_index, band_count, band_rows;
    unsigned band_rows_magic;  // floor(2^32 / band_rows) (0xffffffff for 1): shade.h band_block
    int lv_zs;                 // render_levels_kernel: tiles per XCD stripe, and floor(2^32 / lv_zs)
    unsigned lv_zs_magic;      // (set by launch_render_levels for the instance it launches)
    int local_rows;          // rows of the compact output buffer
    int row0;                // band_count == 1: first image row of this launch (a row slab of rt_render)
    int tile_w, tile_h;      // pixels of one wave's tile
    int tiles_x, num_tiles;
    unsigned tiles_x_magic;  // floor(2^32 / tiles_x) (0xffffffff for 1): tile -> (tx, ty) without a division
    int *shadow_hint;        // render_kernel: per tile x light (< kHintLights) the leaf that occluded the most
                             // lanes of the tile's first shadow packet last time (0: none); null: off
    void *out;               // local_rows x res_x pixels in out_format
    const int *tile_order;   // megakernel dispatch order (null: row-major)
    unsigned *tile_cost;     // per-tile cost of this frame (shader clock), null: not recorded
    int out_format;          // kOutFloat4 / kOutRGBA8 / kOutRGBA16F / kOutRGB32F
    int split16_tiles;       // render_kernel: the first split16_tiles of tile_order run as 16 sixteenth-waves each,
    int split_tiles;         // ... the next split_tiles as 4 quarter-waves each
    int sky_batch_tiles;     // ... and the last sky_batch_tiles (the last measurement's sky tiles) rtk::kSkyBatch a wave
    unsigned long long *counters;  // kCounterSlots x kCounterWords u64, rt_stats order
    // Conservative sky test (render_kernel, non-counting instances): a wave
    // whose every sample ray, approximated (relative error ~1e-6), misses the
    // padded Scene.AABB (pad 2^-10 of the camera-relative scene scale, far
    // above the approximation and rounding errors) is background without its
    // exact rays: each of them misses the exact Scene.AABB gate (Scene.cs:54),
    // so Shade returns the background (RayTracingSetup.cs:310-311).
    unsigned long long primary_total;  // render_kernel (non-counting): camera samples of this launch, added once
    uint4 *wave_counts;      // render_kernel (non-counting): per-wave {shadow, reflection, moot, tag} tallies,
                             // one uint4 per wave of the launch, reduced after it; null: per-wave atomics
    unsigned count_tag;      // this launch's tag in wave_counts (unique per context launch, never 0)
    float inv_spp;           // 1 / spp, exact when spp is a power of two (x * inv_spp == x / spp then)
    int sky_test;            // 1: on (camera outside the padded box, all inputs finite)
    float sky_tlc[3];        // top_left - cam_pos
    float sky_hx, sky_vy;    // HorizontalLength / res_x, VerticalLength / res_y
    float sky_lo[3], sky_hi[3];  // padded Scene.AABB - cam_pos
    // Tile frustum of the camera packets (packet.h cut_start): the camera ray
    // of image point (x, y) (pixel units, y down) runs along D(x, y) = A + x R
    // + y U with A = TopLeft - Position, R = right * hl / res_x, U = -up * vl /
    // res_y (RayTracingSetup.cs:291-296).  The plane through Position bounding
    // the tile on the side x >= xa has the normal cut_ax + xa * cut_bx (the
    // side x <= xb: its negation at xb), likewise y with cut_ay / cut_by;
    // signs make the tile's side positive.  cut_test 0: start at the root.
    int cut_test;
    float cut_ax[3], cut_bx[3], cut_ay[3], cut_by[3];
    float cut_a[3], cut_r[3], cut_u[3];  // A, R, U (the central ray's direction orders the entries)
    uint4 *wave_clock;  // measuring builds only (RT_WAVE_CLOCK): per-wave {start lo, start hi, duration, tile}
    // finely split tiles: 64 >> s16_shift waves each (2: a pixel per wave; 0: a
    // sample per wave, whose pixel sums meet here — per split tile its 64
    // samples as float4 and its 16 pixels' arrival counts)
    int s16_shift;
    float *split_samples;
    int *split_count;
    // one-sample waves (trace.hip render_sample_wave): the stack depth up to
    // which their traversal takes wide steps (coop.h), 0 = as deep as the
    // wave's LDS stack area allows (testing knob: a small value makes every
    // step depth-first, rt_debug_set)
    int sample_wave_stack;
    int in_flight;  // 1: other frames of the context are in flight beside this one (rt_frame.cpp overlapped_frame)
    // measuring builds only (RT_EXP_PERSIST): a whole frame's non-split launch
    // as persist_waves resident waves pulling longest-first tiles from eight
    // per-XCD tile counters (persist_ctr, 16 ints apart, zeroed per launch)
    int persist_waves;
    int *persist_ctr;
};

// The frames of one batch launch (trace.hip render_batch_kernel,
// rt_render_device_batch): frames of one layout from their own cameras, whose
// tiles form one index space — batch tile f * frame_tiles + t is tile t of
// frame f.  Every f[i] carries the batch's dispatch fields (num_tiles = frames
// x frame_tiles, tile_order / tile_cost over batch tiles, splits, sky tail,
// tallies, counters); its camera-derived constants and output are its own.
// Passed by value (kernel arguments, scalar loads): kMaxBatch x 408 B.
constexpr int kMaxBatch = 8;
struct FrameBatch {
    FrameDev f[kMaxBatch];
    int frames;                  // 1 .. kMaxBatch
    int frame_tiles;             // tiles of one frame
    unsigned frame_tiles_magic;  // floor(2^32 / frame_tiles) (0xffffffff for 1)
};

}  // namespace rtd
