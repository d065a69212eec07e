// lbvh.h — on-device BVH build (the reference rebuilds
// its scene every Update(), RayTracingSetup.cs:120-128,171-199, so a drop-in
// must absorb per-frame scene changes without a host rebuild).
//
// Linear BVH (Karras 2012) built entirely on the GPU:
//   1. per rank: the primitive's reference record (v0, edge1, edge2 / centre,
//      r^2), its shading record, its padded bounds and a 64-bit key
//      30-bit Morton code of the mesh centre (or the primitive's own centroid)
//      | mesh id + 1 | Morton code of the centroid inside its mesh's AABB;
//   2. radix sort of (key, rank) (hipCUB);
//   3. leaf-order primitive arrays + inline leaf refs (one primitive per leaf,
//      so leaves are trivially homogeneous in kind and mesh gate);
//   4. Karras hierarchy: n-1 internal nodes in parallel;
//   5. bottom-up padded boxes, second arrival continues (write-through sc1
//      stores and sc1 loads: per-XCD L2s are not coherent on MI355X);
//   6. 2-wide depth (climb to the root; 2-wide output); small homogeneous subtrees marked
//      as multi-primitive leaves; which 2-wide nodes stay as 4-wide nodes
//      (walk from the root over the greedy slots below) -> scan;
//   7. optional collapse to 4-wide nodes: each kept node expands, twice, its
//      internal child slot of largest surface area (the host builder's rule).
// Output: 2-wide nodes (rtd::BvhNode) and, when requested, 4-wide nodes
// (rtd::BvhNode4), both with inline leaf refs and traversed by the same
// kernels (SceneDev.bvh4).  Same padding rules as the host builder, so
// results still equal the brute-force reference.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_device.h"

namespace rtl {

struct MeshDev {
    int rank_first;  // first reference rank of the mesh's triangles
    int geom_first;  // rt_mesh.first_triangle
    int count;
    int material;
};

struct LbvhInput {
    int mesh_count, mt, ns, nl;       // mesh triangle ranks, spheres, loose triangles
    const MeshDev *meshes;            // mesh_count
    const float *mesh_tris;           // geometry-indexed, 9 floats
    const float *mesh_normals;        // geometry-indexed, 3 floats
    const float *spheres;             // ns x 4 (center, r^2)
    const int *sphere_mat;            // ns
    const float *loose_tris;          // nl x 9
    const float *loose_normals;       // nl x 3
    const int *loose_mat;             // nl
    float scene_lo[3], scene_hi[3];   // Scene.AABB (quantisation box)
    float pad_abs;                    // same padding as the host builder
    const float *box_dev;             // non-null: {scene_lo, scene_hi, pad_abs} from device memory instead
    const rtd::MeshGate *gates;       // mesh_count exact mesh AABBs (Mesh.AABB, the gates)
    int mesh_bits;                    // bits of (mesh id + 1) in the sort key
    int key_bits;                     // 64: 30-bit Morton | mesh id + 1 | in-mesh Morton
};

struct LbvhOutput {
    rtd::BvhNode *nodes;    // max(1, n-1)
    rtd::BvhNode4 *nodes4;  // max(1, n-1) or null (no collapse)
    rtd::TriRec *tris;    // mt + nl leaf order, + the sentinel (rt_device.h)
    rtd::SphRec *sphs;    // ns, leaf order
    float4 *shade;        // n, rank order
};

// Scratch owned by the caller (grown with lbvh_scratch_bytes).
size_t lbvh_scratch_bytes(int n);

// Three device ints written by build_lbvh_gpu: the depth of the 2-wide tree
// (levels, leaves included; 2-wide output only), the 4-wide node count and
// the depth of the deepest 4-wide node (root 0) (4-wide output only).
const int *lbvh_info_ptr(const void *scratch, int n);

// Builds on `stream`; returns the first HIP error.  n = mt + ns + nl >= 1.
hipError_t build_lbvh_gpu(const LbvhInput &in, const LbvhOutput &out, void *scratch, size_t scratch_bytes,
                          hipStream_t stream);

}  // namespace rtl
