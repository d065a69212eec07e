// bvh.h — host BVH builder (binned SAH) for the MI355X trace kernels.
//
// The reference has no working BVH (Assets/RayTracer/Data/Collision/BVH.cs is
// an unfinished stub: Subdivide throws at :79 and nothing calls it), its
// closest-hit is the brute-force scan of Scene.IntersectRay (Scene.cs:43-122).
// This builder exists so the GPU can answer the SAME query faster; it must
// never change an answer:
//   * leaves are homogeneous in (kind, gate mesh) so the reference's exact,
//     unpadded per-mesh AABB gate (Scene.cs:67) is applied per leaf;
//   * child boxes are padded outward so the (approximate) node test never
//     culls a primitive the exact Möller–Trumbore / sphere test accepts;
//   * BVH2 internal depth <= 31, so the traversal stack (kStackTotal entries,
//     >= 3 per BVH4 level) cannot overflow.
#pragma once

#include <cstdint>
#include <vector>

#include "rt_device.h"

namespace rtb {

struct Prim {
    float lo[3], hi[3];  // padded bounds
    float c[3];          // centroid
    int kind;            // rtd::kLeafTri / kLeafSphere
    int gate;            // mesh index (-1 = loose / sphere)
    int payload;         // index into the kind's source array
};

struct BuildResult {
    std::vector<rtd::BvhNode> nodes;
    std::vector<rtd::LeafDesc> leaves;
    std::vector<int> tri_order;  // payloads of triangle leaves, leaf order
    std::vector<int> sph_order;  // payloads of sphere leaves, leaf order
    int max_depth = 0;
    double build_ms = 0.0;
};

// Collapse a BVH2 into 4-wide nodes (largest-area internal child expanded
// first), leaves inlined into the child refs.  Returns the max depth.
// empty_ref: the ref stored in unused slots (their boxes are +inf and are
// only "entered" by NaN / zero-direction rays): a sentinel leaf, never a
// node, so such rays cannot cycle.
int collapse_bvh4(const BuildResult &B, std::vector<rtd::BvhNode4> &out, int empty_ref);

// Build over prims (reordered in place).  Always produces >= 1 internal node
// when prims is non-empty (a lone leaf hangs off the root beside an empty child).
BuildResult build_bvh(std::vector<Prim> &prims, int max_leaf = 4);

}  // namespace rtb
