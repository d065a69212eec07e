// wavefront.h — HBM work queues of the wavefront render path (trace_wf.hip).
//
// A frame is processed in chunks of tiles (64 sample slots per tile).  Each
// chunk runs levels k = 0..max_bounces of the reference's Shade recursion
// (RayTracingSetup.cs:304-366) as separate passes over compact queues:
//
//   trace_closest(k)  persistent, wave-level dynamic ray fetch   -> hit[e]
//   shade(k)          surface, shadow rays, mirror rays(k+1)     -> shadow queue, ray(k+1)
//   trace_any(k)      persistent, dynamic fetch over shadow rays -> occ[i]
//   finish(k)         ambient + unoccluded light terms in order  -> col[e]
//   fold(k)           col[e] = c + km * col[child]  (k = deepest-1 .. 0)
//   resolve           sum samples per pixel in order, /spp, /255 -> out
//
// Pool entries of level k are contiguous: [begin_k, begin_k + n_k) with
// begin_k = n_0 + ... + n_{k-1}; level 0 entry e is slot (tile0 + e/64, e%64)
// and its ray is regenerated, never stored.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_device.h"

namespace rtw {

constexpr int kMaxLevels = rtd::kMaxBounces + 1;

struct Counters {
    int n[kMaxLevels];         // entries per level (n[0] = chunk slots)
    int shadow_n[kMaxLevels];  // shadow rays emitted by shade(k)
    int head_c[kMaxLevels];    // dynamic-fetch heads, closest-hit pass
    int head_a[kMaxLevels];    // dynamic-fetch heads, any-hit pass
};

struct Args {
    Counters *ctr;
    float4 *ray_o;  // level >= 1: origin.xyz
    float4 *ray_d;  // level >= 1: direction.xyz
    int4 *hit;      // rank (-2 inactive slot, -1 miss), t bits, shadow base, -
    float4 *col;    // colour .xyz (Rgb.Value units), child entry in .w (int bits, -1 none)
    float4 *sh_o;   // shadow ray origin.xyz
    float4 *sh_d;   // shadow ray direction.xyz, lightDistanceSq in .w
    unsigned char *occ;
    int tile0;      // first tile of the chunk
    int n0;         // slots in the chunk (tiles * 64)
    int max_level;  // max(0, max_reflection_bounces)
};

}  // namespace rtw
