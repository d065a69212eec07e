// kernels.h — host-side launchers of the gfx950 kernels in trace.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "wavefront.h"

namespace rtk {

// Measuring builds (-DRT_WAVE_CLOCK): render_kernel records per-wave clocks
// into F.wave_clock (rt_debug_set RT_DEBUG_WAVE_CLOCKS); the product build
// compiles no such store.
#ifdef RT_WAVE_CLOCK
constexpr bool kWaveClockBuild = true;
#else
constexpr bool kWaveClockBuild = false;
#endif

// Sky tiles per wave at the end of a longest-first order (FrameDev
// sky_batch_tiles): a tile whose every sample surely misses the scene box is
// a background store, too little work for a wave of its own (60 % of a C3
// frame's waves, 12 % of its wave time: wclk_r05s).
#ifdef RT_EXP_SKYBATCH
constexpr int kSkyBatch = RT_EXP_SKYBATCH;  // measuring builds only (1: off)
#else
constexpr int kSkyBatch = 32;  // C3 in flight: 16 -> 32 +1.2 % / +0.2 % on two boxes, C4 +-0 (r06b, r05w)
#endif
// Count of the tiles before the sorted order's sky tail (cost key 0) into
// host-mapped memory, one 64-bit store tagged with the sort's sequence number:
// (seq << 32) | count.
hipError_t launch_sky_count(const unsigned *cost_sorted, int n, unsigned seq, unsigned long long *out,
                            hipStream_t stream);

// Frames (row shards) of at most this many tiles launch render_kernel's
// 5-wave instances (trace.hip), the only ones with the one-sample split path.
constexpr int kShardTilesMax = 70000;

// One frame (or one row shard of it): CastPixelRays + Shade, RayTracingSetup.cs:275-366.
// Megakernel: one lane per sample, whole Whitted chain in one launch (trace.hip).
// Longest-first tile order for the next frame (trace.hip).
size_t tile_sort_scratch_bytes(int n);
// waves of a render_kernel launch of F (tiles + the extra waves of split tiles)
int render_mega_waves(const rtd::FrameDev &F);
// Sums the kCounterSlots sharded counter slots into kCounterWords words at out.
hipError_t launch_fold_counters(const unsigned long long *counters, unsigned long long *out, hipStream_t stream);
hipError_t launch_iota(int *p, int n, hipStream_t stream);
hipError_t sort_tiles_by_cost(const unsigned *cost, unsigned *cost_sorted, const int *iota, int *order, int n,
                              void *scratch, size_t scratch_bytes, hipStream_t stream);

// The top-level cut of a 4-wide tree (rtd::CutTable), after every tree build
// or refit, on the stream of that build.
hipError_t launch_build_cut(const rtd::BvhNode4 *nodes, rtd::CutTable *out, hipStream_t stream);
// the same cut with its boxes re-read from the (refitted) tree
hipError_t launch_refresh_cut(const rtd::BvhNode4 *nodes, rtd::CutTable *out, hipStream_t stream);

// *instance (nullable): the name of the kernel instance launched (static
// storage; null when nothing was launched) — rt_debug_read RT_DEBUG_LAST_LAUNCH.
hipError_t launch_render_mega(const rtd::SceneDev &S, const rtd::FrameDev &F, bool count_tests,
                              hipStream_t stream, const char **instance = nullptr);

// The frames of a batch (rtd::FrameBatch: whole 4-spp frames of one layout)
// in one launch: render_batch_kernel, then the batch's sky tail and tallies
// (sky_batch_batch_kernel) or its tallies alone.
hipError_t launch_render_batch(const rtd::SceneDev &S, const rtd::FrameBatch &B, hipStream_t stream,
                               const char **instance = nullptr);

// Level-synchronous all-packet megakernel (trace_levels.hip), chosen by
// launch_render_mega for >= 16 spp on a 4-wide BVH.
hipError_t launch_render_levels(const rtd::SceneDev &S, const rtd::FrameDev &F, hipStream_t stream);

// Packet megakernel: wave-synchronous levels, coherent rays traced one BVH
// path per wave (packet.h).
hipError_t launch_render_packet(const rtd::SceneDev &S, const rtd::FrameDev &F, bool count_tests,
                                hipStream_t stream);

// Wavefront: per-level queues in HBM, persistent traversal with dynamic ray
// fetch (trace_wf.hip); chunk_tiles tiles (64 slots each) per pass sequence.
hipError_t launch_render_wavefront(const rtd::SceneDev &S, const rtd::FrameDev &F, const rtw::Args &A,
                                   int chunk_tiles, bool count_tests, hipStream_t stream);

// Batch closest hit, Scene.IntersectRay (Scene.cs:43-122): rays are 6 floats
// (origin, direction); out[i] = {rank or -1, distance bits, rank of the closest
// mesh-triangle hit or -1 (the reference's stale MeshIndex), -}.
hipError_t launch_intersect(const rtd::SceneDev &S, const float *rays, int n, int4 *out,
                            hipStream_t stream);

// Row-order reassembly of block-cyclic shards gathered back to back.
hipError_t launch_assemble(const void *gathered, int res_x, int res_y, int band_count, int band_rows,
                           int local_rows, int pixel_bytes, void *image, hipStream_t stream);

}  // namespace rtk
