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
//   plane 0: (origin.xyz, material pdf)          = Ray.origin, Ray.params.x
//   plane 1: (direction.xyz, ior)                = Ray.direction, Ray.params.w
//   plane 2: (throughput.rgb, bits(pixel | prevDiffuse << 31))
//   plane 3: (radiance.rgb, 0)
// The bounce index (Ray.params.z) is uniform per launch and not stored.
struct RayQueue {
  float4* plane[4];
};

struct BounceArgs {
  uint32_t width, height;
  uint32_t frame_index;        // SharedData.frameIndex
  uint32_t bounce;             // loop iteration i (renderer/Renderer.mm:517)
  uint32_t max_path_length;    // MAX_PATH_LENGTH
  uint32_t shard_rank, shard_count, tiles_x;
  uint32_t num_slots;          // bounce 0: owned tiles * 4096 pixel slots
  const uint32_t* in_count;    // bounce > 0: live rays produced by the previous bounce
  uint32_t* out_count;         // live rays produced by this bounce (atomic)
  RayQueue in_q, out_q;
  const float4* noise_raygen;  // slot f%3  = T_f
  const float4* noise_shade;   // slot (f+i)%3
  float4* image;               // RGBA32F accumulation image (row 0 = bottom)
};

#define MRT_DECLARE_LAUNCHERS(NS)                                                                         \
  namespace NS {                                                                                          \
  hipError_t launch_raygen(uint32_t W, uint32_t H, const float* noise, RefRay* rays, hipStream_t s);      \
  hipError_t launch_intersect(const DeviceScene& sc, const void* rays, uint32_t stride, uint32_t count,   \
                              RefIntersection* out, hipStream_t s);                                       \
  hipError_t launch_shade(const DeviceScene& sc, uint32_t W, uint32_t H, uint32_t frame_index,            \
                          uint32_t max_path_length, const float* noise, const RefIntersection* isect,     \
                          RefRay* rays, RefShadowRay* srays, hipStream_t s);                              \
  hipError_t launch_resolve(uint32_t count, const RefIntersection* isect, RefRay* rays,                   \
                            const RefShadowRay* srays, hipStream_t s);                                    \
  hipError_t launch_accumulate(uint32_t W, uint32_t H, uint32_t frame_index, const RefRay* rays,          \
                               float* image, hipStream_t s);                                              \
  /* fused wavefront bounce; grid = 0 -> persistent grid from occupancy */                               \
  hipError_t launch_bounce(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries,           \
                           hipStream_t s);                                                                \
  }

MRT_DECLARE_LAUNCHERS(precise)
MRT_DECLARE_LAUNCHERS(fast)

}  // namespace mrt
