// bvh_gpu.h — device-side acceleration-structure build: the MI355X
// replacement for MPSTriangleAccelerationStructure.rebuild
// (renderer/Renderer.mm:456-462), which builds from the GPU-resident
// vertex/index buffers without a host round trip.
//
// Both builders start from one device radix sort (rocPRIM) of the triangles
// by the 63-bit Morton code of their centroids, then build a binary tree:
//   * LBVH (Karras 2012): the radix tree in one pass (one thread per internal
//     node), boxes refitted bottom-up with arrival counters;
//   * PLOC (Meister & Bittner 2018): clusters in Morton order repeatedly merge
//     with their mutual nearest neighbour (smallest merged-box surface area)
//     within +-16 positions — SAH-like quality, still O(n) work per round;
// then a level-synchronous top-down collapse
// into the BVH4 node layout of mrt_layout.h (largest-area child opened first,
// subtrees of <= max_leaf triangles become leaves; every subtree is given the
// contiguous range of the leaf-ordered triangle array its triangles fill, in
// child order, so a leaf is a contiguous run).  Nodes are emitted level by level, i.e.
// in breadth-first order, so any prefix is the top levels (LDS staging).
// Boxes are padded outward like the host builder's, so traversal returns the
// exact brute-force nearest hit on this tree too.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace mrt {

enum class GpuBvhAlgo {
  kLbvh,   // Karras radix tree: fastest build, weakest tree
  kPloc,   // PLOC clustering over the Morton order: SAH-like tree quality
};

struct GpuBvhResult {
  float* nodes = nullptr;      // hipMalloc'd, 32 floats per BVH4 node (caller frees)
  float* tris = nullptr;       // hipMalloc'd, 12 floats per triangle, leaf order (caller frees)
  size_t nodes_bytes = 0, tris_bytes = 0;
  int32_t root = 0;            // node index, or a leaf ref for scenes of <= max_leaf triangles
  uint32_t num_nodes = 0;
  uint32_t num_leaves = 0;
  uint32_t levels = 0;         // BVH4 interior levels
  uint32_t max_stack = 0;      // traversal stack entries a ray can need
  uint32_t binary_depth = 0;   // deepest leaf of the binary radix tree
  uint32_t build_iterations = 0;   // PLOC merge rounds
  double build_ms = 0.0;       // device time of the build (HIP events)
};

// positions: 3 floats at `stride_bytes` per vertex, device memory;
// indices: 3 uint32 per triangle, device memory.  Synchronous on `stream`.
hipError_t build_bvh_gpu(const float* positions, uint32_t stride_bytes, const uint32_t* indices,
                         uint32_t num_triangles, uint32_t max_leaf, GpuBvhAlgo algo, hipStream_t stream,
                         GpuBvhResult& out, std::string& error);

}  // namespace mrt
