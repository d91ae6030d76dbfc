// kernels.h — host-side launch interface of the gfx950 kernels.
//
// kernels.hip is compiled twice:
//   mrt::precise  — parity build: -ffp-contract=off, IEEE div/sqrt, sin/cos
//                   evaluated in double and rounded (bit-matches the oracle);
//   mrt::fast     — production build: FMA contraction, v_rcp/v_rsq/v_sqrt,
//                   native v_sin/v_cos.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrt_layout.h"

namespace mrt {

// Ray queue: SoA of four float4 planes, one record per ray slot:
//   plane 0: (origin.xyz, bits(slot | prevDiffuse << 31))    = Ray.origin, params.y
//            slot = frame_in_batch * num_slots + owned slot (the pixel's
//            radiance index; the pixel is decoded from it, kernels.hip)
//   plane 1: (direction.xyz, 0)                            = Ray.direction
//   plane 2: (throughput.rgb, material pdf)                = Ray.throughput, params.x
//   plane 3: (radiance.rgb, ior)                           = Ray.radiance, params.w
// Planes 0-1 are all the traversal needs; planes 2-3 are loaded after the
// hit so they do not occupy registers during traversal.
// The bounce index (Ray.params.z) is uniform per launch and not stored.
constexpr int kQueuePlanes = 4;
struct RayQueue {
  float4* plane[kQueuePlanes];
};

// Frame batching: one launch carries the rays of `batch` consecutive frames
// (frame_index .. frame_index + batch - 1): about 2^24 rays per launch, so a
// GPU that owns a small share of the tiles (1/8 of 1080p: 64 frames per
// launch) still issues launches of the same size as a whole 1080p GPU.
constexpr uint32_t kMaxBatch = 64;

// Dynamic work distribution inside a bounce launch: the dense input is split
// into kGrabRanges contiguous ranges, each with its own grab counter (one
// 128-B line apart, so the atomics do not serialise on one word); a wave
// takes kGrab rays at a time from its home range, then steals from the next
// ranges.  A block's output segment holds chunk + kSegSlack rays, where
// kSegSlack >= (waves per block + 1) * kGrab keeps at least one block able to
// grab until the input is exhausted (see bounce_kernel).
#ifndef MRT_GRAB   // r5, alternating in one call: 64 / 192 lose 1.1-2.6 % / 1.0 % on C2, 2.1 / 0.5 % on C4
#define MRT_GRAB 128
#endif
constexpr uint32_t kGrab = MRT_GRAB;
static_assert(kGrab % 64 == 0 && (4 + 1) * kGrab <= 1024, "kGrab: whole waves, within kSegSlack");
constexpr uint32_t kGrabRanges = 16;   // <= 31: the probe's open mask is one 32-bit ballot word
static_assert(kGrabRanges <= 31, "kGrabRanges");
#ifndef MRT_GRAB_STRIDE
#define MRT_GRAB_STRIDE 32
#endif
constexpr uint32_t kGrabStride = MRT_GRAB_STRIDE;    // uint32 words between counters
constexpr uint32_t kSegSlack = 1024;

// Wave-local streaming wavefront (stream_kernel): every bounce of a batch in
// one launch with no inter-wave hand-off.  Each wave keeps its own queue of
// kStreamCap ray slots per bounce level 1..L-1 (SoA planes of RayQueue a.in_q,
// level k of wave w at slots ((w * (L - 1)) + k - 1) * kStreamCap) and always
// runs 64 rays of one bounce: the deepest level holding >= 64 rays, else 64
// new camera rays; survivors go to the next level (< 2 * 64 rays each).
constexpr uint32_t kStreamCap = 128;
constexpr uint32_t kStreamMaxL = 64;
inline size_t stream_slots(uint32_t L, uint32_t G) { return (size_t)G * 4 * (L > 1 ? L - 1 : 1) * kStreamCap; }

// n / d for every n < 2^31 as mulhi(n, m) >> sh (m = 0: d = 1), with
// l = ceil(log2 d), m = ceil(2^(31 + l) / d) < 2^32, sh = l - 1: the error
// m d - 2^(31+l) < d <= 2^l, so n (m d - 2^(31+l)) < 2^(31+l) and the
// floor is exact (Granlund & Montgomery 1994, N = 31).  Wave-uniform kernel
// arguments: the quotient costs one v_mul_hi_u32 and a shift instead of the
// compiler's per-lane reciprocal sequence and its three VGPRs.
struct MagicDiv {
  uint32_t m, sh;
};
inline MagicDiv magic_div(uint32_t d) {
  if (d <= 1) return {0u, 0u};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const unsigned long long p = 1ull << (31 + l);
  return {(uint32_t)((p + d - 1) / d), l - 1};
}
// The kernels' quotient (kernels.hip mdiv: __umulhi(n, m) >> sh) restated on
// the host, and the check draw_n runs on every launch's divisors: m = 0 means
// d = 1, so a multiplier left zero for a divisor d > 1 (or one computed for
// another d) fails at the floor steps below instead of dividing by 1.
inline uint32_t mdiv_host(uint32_t n, MagicDiv m) {
  return m.m ? (uint32_t)(((unsigned long long)n * m.m) >> 32) >> m.sh : n;
}
inline bool magic_ok(MagicDiv m, uint32_t d) {
  if (d == 0) return false;
  const uint32_t top = 0x7FFFFFFFu, ns[5] = {0u, d - 1u, d < top ? d : top, top - top % d, top};
  for (uint32_t n : ns)
    if (mdiv_host(n, m) != n / d) return false;
  return true;
}

struct BounceArgs {
  uint32_t width, height;
  uint32_t frame_index;        // SharedData.frameIndex of the batch's first frame
  uint32_t batch;              // frames in this launch (1..kMaxBatch)
  uint32_t bounce;             // loop iteration i (renderer/Renderer.mm:517)
  uint32_t max_path_length;    // MAX_PATH_LENGTH
  uint32_t shard_rank, shard_count, tiles_x;
  uint32_t num_slots;          // per frame: owned tiles * 4096 pixel slots (bounce 0 input = num_slots * batch)
  uint32_t flags;              // kShadeDebugMaterial: DEBUG_MATERIAL (renderer/Shaders.metal:7,142-147)
  uint32_t debug;              // ablation bits for profiling (0 in production, env MRT_DEBUG):
                               //   1 = skip shadow traversal, 2 = skip shading, 4 = no queue writes,
                               //   8 = static interleaved work assignment (no grab counters),
                               //   16 = no material partition of the survivors, 32 = no occlusion traversal
                               //   of light samples, 64 = no occlusion query of last-bounce light hits,
                               //   128 = no origin-triangle test (stream / bounce kernels),
                               //   256 = the accumulate touches no pixel (renderer.cpp draw_n),
                               //   512 = no convex-occluder test, 1024 = no other-light test (occluder-tree
                               //   shadow queries, stream / bounce kernels)
  // segmented queues: block g of a launch appends its class-0 survivors
  // (left a diffuse surface) to [g*cap, g*cap + c0_g) and its class-1
  // survivors to [g*cap + cap - c1_g, g*cap + cap) of the output queue
  // (cap = chunk + kSegSlack); counts are [c0 of all blocks][c1 of all blocks]
  uint32_t in_segments;        // bounce > 0: number of input segments (2 classes x previous grid size)
  const uint32_t* in_seg_count;
  const uint32_t* in_chunk;    // previous launch's chunk (segment stride in slots)
  uint32_t* out_seg_count;     // [grid]
  uint32_t* out_chunk;
  uint32_t* out_total;         // survivors of this launch (stats)
  uint32_t* grab;              // [kGrabRanges * kGrabStride] zeroed grab counters of this launch
  RayQueue in_q, out_q;
  // noise: the table of frame g (T_g, or the initial table for g < 0) is
  // noise_window[(noise_offset + g - frame_index) * 4096 ...]; raygen reads
  // T_f, iteration i reads T_{f - c(i)} (noise.h); noise_offset >= 2
  const float4* noise_window;
  uint32_t noise_offset;
  float4* radiance;            // [batch][num_slots] path radiance by owned slot, written once per
                               // owned pixel when its path ends (accumulated by launch_accumulate_frame)
  uint32_t* stack_spill;       // traversal stack entries beyond the LDS capacity:
                               // [grid * 256][max_stack] uint32 (null if none)
  uint32_t* bounce_counts;     // path / stream kernel: [max_path_length] rays alive at the start of bounce b + 1
  unsigned long long* span;    // [2] of the frame batch, zeroed: ~(earliest block start), latest wave end
                               // (wall_clock64 ticks; null = not recorded)
  const uint32_t* primary;     // camera-ray candidate lists per 8x8 pixel block (primary.h; null = traverse)
  uint32_t primary_bx;         // blocks per row of `primary`
  // exact division by the launch's runtime divisors without per-lane
  // reciprocals (magic_div): tiles_x, num_slots, batch
  MagicDiv div_tiles, div_slots, div_batch;
};

// running-mean accumulation of one frame over the owned tiles
struct AccumArgs {
  uint32_t width, height;
  uint32_t frame_index;        // first frame of the batch; frames are applied in order
  uint32_t batch;
  uint32_t shard_rank, shard_count, tiles_x;
  uint32_t num_slots;          // owned tiles * 4096
  const float4* radiance;      // [batch][num_slots]
  float4* image;
  uint32_t accumulate;         // ACCUMULATE_IMAGE (renderer/Raytracing.h:14); 0: the last frame alone
  // the last batch of a draw: block 0 copies the draw's statistics words
  // ([0, copy_words) and [span_word, span_word + span_words)) to the host's
  // pinned copy and zeroes all zero_words of `counters` for the ring entry's
  // next draw (no memset and no copy-engine hop per draw); null otherwise
  uint32_t* counters;
  uint32_t* host_counters;
  uint32_t copy_words, span_word, span_words, zero_words;
};

constexpr uint32_t kShadeDebugMaterial = 1u;   // BounceArgs::flags / launch_shade flags

#define MRT_DECLARE_LAUNCHERS(NS)                                                                         \
  namespace NS {                                                                                          \
  hipError_t launch_raygen(uint32_t W, uint32_t H, const float* noise, RefRay* rays, hipStream_t s);      \
  /* spill: >= (max_stack - 32) * kIntersectSpillGrid * 256 uint32 when sc.max_stack > kMaxStack */       \
  hipError_t launch_intersect(const DeviceScene& sc, const void* rays, uint32_t stride, uint32_t count,   \
                              RefIntersection* out, uint32_t* spill, hipStream_t s);                      \
  hipError_t launch_shade(const DeviceScene& sc, uint32_t W, uint32_t H, uint32_t frame_index,            \
                          uint32_t max_path_length, const float* noise, const RefIntersection* isect,     \
                          RefRay* rays, RefShadowRay* srays, uint32_t flags, hipStream_t s);              \
  hipError_t launch_resolve(uint32_t count, const RefIntersection* isect, RefRay* rays,                   \
                            const RefShadowRay* srays, hipStream_t s);                                    \
  hipError_t launch_accumulate(uint32_t W, uint32_t H, uint32_t frame_index, const RefRay* rays,          \
                               float* image, bool accumulate, hipStream_t s);                             \
  /* persistent grid size of the fused bounce kernel for this scene */                                    \
  hipError_t bounce_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t blocks_per_cu,          \
                         uint32_t* grid);                                                                \
  /* fused wavefront bounce over `grid` blocks (the same grid for every launch of a renderer);          \
     stack_entries = LDS stack capacity 8/16/24/32, deeper entries go to a.stack_spill */                 \
  hipError_t launch_bounce(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries,           \
                           uint32_t grid, hipStream_t s);                                                 \
  /* path megakernel: every bounce of a batch of frames in one launch (a.bounce unused, no ray queues) */ \
  hipError_t launch_paths(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries,            \
                          uint32_t grid, hipStream_t s);                                                  \
  hipError_t path_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t* grid);                   \
  /* wave-local streaming wavefront: all bounces of a batch in one launch, per-wave ray queues     \
     (whole-scene-in-LDS scenes; hipErrorNotSupported otherwise)     */                          \
  hipError_t launch_stream(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries,           \
                           uint32_t grid, hipStream_t s);                                                 \
  bool stream_supported(const DeviceScene& sc, uint32_t stack_entries);                                   \
  /* the stream kernel's persistent grid (its LDS has no per-block segment scratch) */                    \
  hipError_t stream_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t* grid);                  \
  /* the scene's LDS staging mode is not "whole scene in LDS": the path kernel is the faster one */      \
  bool path_preferred(const DeviceScene& sc);                                                             \
  /* accumulateImage over the owned tiles of a batch of frames (in frame order) */                        \
  hipError_t launch_accumulate_frame(const AccumArgs& a, hipStream_t s);                                  \
  /* blitFragment (Shaders.metal:33-70): tone map / sRGB / golden comparison of the RGBA32F image */     \
  hipError_t launch_display(const float4* image, const float4* reference, float4* out, uint32_t n,        \
                            uint32_t flags, float compare_scale, hipStream_t s);                          \
  /* owned-tile exchange: pack a shard's tiles of a W x H RGBA32F image into                             \
     [owned tile][64 x 64] float4 (zeros outside the image), or unpack them back (bitwise moves) */     \
  hipError_t launch_tiles_move(const float4* src, float4* dst, uint32_t W, uint32_t H, uint32_t rank,    \
                               uint32_t count, bool pack, hipStream_t s);                                 \
  /* diagnostic phase stamps (MRT_STAMPS builds; zeros otherwise) */                                      \
  hipError_t read_stamps(unsigned long long* out8, bool reset);                                          \
  /* per-wave timeline {start, exit, iterations} of the last launch of each bounce % 4 (stamp builds) */   \
  hipError_t read_wave_times(unsigned long long* out, size_t n);                                         \
  /* diagnostic lane statistics (MRT_LANESTATS builds; zeros otherwise) */                                 \
  hipError_t read_lane_stats(unsigned long long* out, size_t n, bool reset);                             \
  }

MRT_DECLARE_LAUNCHERS(precise)
MRT_DECLARE_LAUNCHERS(fast)

}  // namespace mrt
