// bvh.h — acceleration-structure build, the replacement for
// MPSTriangleAccelerationStructure.rebuild (renderer/Renderer.mm:456-462).
//
// CPU binned-SAH BVH2 over the flattened triangles (vertex stride 24 B,
// uint32 indices, triangleCount = indices/3 exactly as the reference feeds
// MPS), emitted in the MI355X node layout documented in mrt_layout.h:
//   * interior nodes carry both child boxes (one 64-B line per visit);
//   * the first `lds_nodes` interior nodes are in breadth-first order (the
//     top levels, staged into LDS by the traversal kernels), the rest in
//     depth-first order (parent and nearer child share lines/pages);
//   * leaves (<= 16 triangles) reference a contiguous run of the leaf-ordered
//     triangle array {v0|prim, e1, e2}.
// Boxes are padded outward so the slab test is conservative under rounding:
// traversal then returns exactly the brute-force nearest hit.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "mrt_layout.h"

namespace mrt {

struct BvhBuildOptions {
  uint32_t max_leaf_size = 2;     // <= kMaxLeafSize; 2 measured best (C2 +9.5 % over 4, C3 +0.9 %, C4 =)
  uint32_t lds_node_budget = 256; // interior nodes placed first in BFS order
  uint32_t bins = 32;             // SAH bins: 32 measured C3 +1.9 % over 16 (C2, C4 =), 64 C2 -2 %
  uint32_t exact_sah_below = 0;   // ranges of fewer triangles use the exact sweep SAH (0 = never; measured C2 -2 %)
  bool full_sweep = false;        // exact sweep SAH at every node (presorted, O(n log n)); opt-in (MRT_FULL_SWEEP=1)
  float traversal_cost = 1.0f;    // relative to one triangle test
  uint32_t width = 2;             // 2 = the binary SAH tree itself, 4 = BVH4 (128-B nodes, collapsed; what the kernels traverse)
  int collapse_dp = -1;           // BVH4: 1 = the collapse that minimises the summed area of the wide interior nodes
                                  // (dynamic programming over the binary tree), 0 = greedy largest-area opening,
                                  // -1 = by size: DP below kGreedyCollapseTriangles, greedy above (measured r4:
                                  // C2 +0.8 %, C3 +1.9 % with DP; the 1M-triangle C4 -1.2 %); MRT_COLLAPSE=0/1
                                  // overrides -1 in every build path (scenes, mrt_accel_*, tools)
};

struct BvhResult {
  std::vector<float> nodes;       // 16 (BVH2) or 32 (BVH4) floats per interior node
  std::vector<float> tris;        // 12 floats per leaf-ordered triangle
  int32_t root = 0;
  uint32_t num_nodes = 0;
  uint32_t num_leaves = 0;
  uint32_t max_depth = 0;         // deepest leaf (root = 0); traversal needs <= max_depth stack entries
  uint32_t lds_nodes = 0;         // top BFS-ordered nodes (min(budget, num_nodes))
  uint32_t width = 2;
  uint32_t max_stack = 0;         // traversal stack entries needed (push all hit children but one)
  uint32_t wide_depth = 0;        // interior levels of the emitted tree
  double sah_cost = 0.0;
};

// positions: 3 floats per vertex at `stride_bytes` stride (24 for RefVertex).
bool build_bvh(const float* positions, size_t stride_bytes, const uint32_t* indices, uint32_t num_triangles,
               const BvhBuildOptions& opt, BvhResult& out, std::string& error);

inline int32_t leaf_ref(uint32_t first, uint32_t count) {
  return (int32_t)~((first << kLeafCountBits) | (count - 1));
}

}  // namespace mrt
