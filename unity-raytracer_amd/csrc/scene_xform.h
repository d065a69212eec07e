// scene_xform.h — mesh extraction on the device.
//
// The reference re-extracts every mesh on every Update()
// (RayTracingSetup.cs:120-128,159-169 → SceneMesh.Mesh, SceneMesh.cs:11-53):
//   * every local vertex goes through localToWorldMatrix.MultiplyPoint3x4
//     (m00*x + m01*y + m02*z + m03 per row, left to right, no FMA);
//   * Mesh.AABB = Encapsulate over ALL transformed vertices (SceneMesh.cs:22-31);
//   * triangles come from the index buffer in order; the mesh normal of each
//     is -Triangle.Normal = -(v / length(v)), v = cross(v2 - v0, v1 - v0)
//     (Triangle.cs:13-21, SceneMesh.cs:43).
// Here the local vertices and index buffers stay resident in HBM and a frame
// only uploads the mesh_count 4x4 matrices; the world-space triangles and
// normals land directly in the LBVH builder's input arrays.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_device.h"

namespace rtx {

struct MeshSrcDev {
    int vertex_first;  // into the concatenated local vertex array
    int vertex_count;
    int tri_first;     // geometry index of the mesh's first triangle
    int tri_count;
    int part_first;    // first of the mesh's AABB parts (max(1, ceil(vertex_count / kAabbPart)) each)
};

constexpr int kAabbPart = 2048;  // vertices per AABB-reduction wave

struct XformArgs {
    int mesh_count, vertex_total, tri_total;
    const MeshSrcDev *meshes;  // mesh_count
    const float *local;        // vertex_total x 3
    const int *indices;        // tri_total x 3, global vertex indices (validated on the host)
    const float *matrices;     // mesh_count x 16, row-major m[row * 4 + col]
    float *world;              // vertex_total x 3 (scratch)
    float *tris;               // tri_total x 9 (rt_triangle layout)
    float *normals;            // tri_total x 3
    rtd::MeshGate *aabbs;      // mesh_count: exact Mesh.AABB
    int part_total;            // AABB parts over all meshes
    rtd::MeshGate *parts;      // part_total (scratch): per-part partial AABBs
};

hipError_t transform_meshes(const XformArgs &a, hipStream_t stream);

// Scene.CalculateAABB of an animated scene on the device: the mesh AABBs in
// order, then the fixed box of the loose triangles and spheres (rest_lo/hi,
// from the host), with the host's Unity min/max and its absolute node padding
// (rt_abi.cpp pad_abs_of).  Writes {lo[3], hi[3], pad_abs} to box (device,
// read by the LBVH build) and to host_box (page-locked, read after the
// stream's synchronisation).
hipError_t scene_box(const rtd::MeshGate *aabbs, int mesh_count, const float rest_lo[3], const float rest_hi[3],
                     float *box, float *host_box, hipStream_t stream);

// Refit of a fixed 4-wide tree after the meshes moved (rt_set_scene_source_ex
// with RT_BUILD_SAH_REFIT): the topology and the leaf order of the host SAH
// build are kept; every mesh triangle record (v0, v1 - v0, v2 - v0) and
// shading normal is rewritten from the extracted world triangles, every
// primitive's padded box recomputed with the frame's padding (the builders'
// rule), and the node boxes rebuilt bottom-up (one thread per leaf-only node
// climbing while it is its parent's last internal child to arrive; slots
// handed over with write-through stores, like lbvh.hip k_bounds).  Also sums
// the internal slots' half areas and the root's, the tree-quality measure the
// host compares with the last full build's.
struct RefitArgs {
    int ntri, nsph, nnodes;         // triangle records (sentinel excluded), sphere records, 4-wide nodes
    rtd::TriRec *tris;              // leaf order; mesh triangle records rewritten
    const rtd::SphRec *sphs;
    float4 *shade;                  // rank-indexed; mesh triangle normals rewritten (.w kept)
    int mt, ns;                     // ranks: [0, mt) mesh triangles, [mt, mt + ns) spheres, then loose
    int mesh_count;
    const int *mesh_rank_first;     // mesh_count
    const int *mesh_geom_first;     // mesh_count
    const float *mesh_tris;         // geometry-indexed world triangles (9 floats)
    const float *mesh_normals;      // geometry-indexed (3 floats)
    const float *loose_tris;        // loose-triangle vertices (9 floats each)
    const float *box;               // {scene lo, hi, pad_abs} (k_scene_box)
    float4 *prim_lo, *prim_hi;      // ntri + nsph padded boxes (scratch)
    rtd::BvhNode4 *nodes;
    const int *parent_slot;         // per node: parent * 4 + slot, -1 for the root
    const int *internal_children;   // per node
    int *arrivals;                  // per node, zeroed by refit_tree
    int empty_ref;                  // the unused slots' ref (+inf boxes, left alone)
    float *quality;                 // [0] sum of internal slots' half areas, [1] root half area; [2..3]: the
                                    // sum's 64-bit fixed-point accumulator (16 B, zeroed by refit_tree)
};

hipError_t refit_tree(const RefitArgs &a, hipStream_t stream);
// fills a tree's parent_slot / internal_children tables (a.nodes, a.nnodes)
hipError_t refit_links(const RefitArgs &a, int *parent_slot, int *internal_children, hipStream_t stream);

}  // namespace rtx
