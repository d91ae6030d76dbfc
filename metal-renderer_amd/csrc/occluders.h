// occluders.h — the shadow-ray occluder tree.
//
// lightSamplingHandler (renderer/Shaders.metal:214-231) adds a light sample
// iff the nearest hit of the shadow ray (MPS intersect, renderer/Renderer.mm:
// 545-553) is the target light triangle.  A triangle can only stand in front
// of the target if the segment from the shadow origin p to the light point q
// crosses the triangle's plane.  For a plane with every light vertex strictly
// on one side of it, no triangle in that plane can occlude a shadow ray whose
// origin is on the same side (by a margin covering the float error of the
// ray-triangle test, occluders.cpp): such rays may traverse a second BVH
// built over the other triangles only.
//
// The culled planes are the scene's supporting planes (all vertices on one
// side): the walls, floor and ceiling of a room, which every shadow origin
// inside the room satisfies.  The kernels test the origin against the culled
// planes (a few FMAs, wave-uniform plane data) and traverse the occluder tree
// when it passes, the full tree otherwise; both give the same answer.
#pragma once
#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "mrt_layout.h"

namespace mrt {

struct OccluderSet {
  std::vector<uint32_t> keep;                  // triangles that stay in the occluder tree (ascending)
  std::vector<std::array<float, 4>> planes;    // culled planes (n, w): inside is n.x - w <= -margin
  float margin = 0.0f;                         // runtime inside margin (scene units)
  float cos_min = 0.0f;                        // shadow rays with |cos| to the light's normal below this
                                               //   traverse the main tree (grazing guard, occluders.cpp)
  uint32_t culled = 0;                         // triangles left out
};

// positions: 3 floats per vertex at `stride_bytes`; light_vertices and
// light_normals: 9 floats (three positions / vertex normals) per light
// triangle.  Returns false (no culling) when the
// scene is too large to classify or the qualifying planes hold less than an
// eighth of the triangles (then `out` is empty).
bool find_occluders(const float* positions, size_t stride_bytes, uint32_t num_vertices, const uint32_t* indices,
                    uint32_t num_triangles, const float* light_vertices, const float* light_normals,
                    uint32_t num_lights, OccluderSet& out);

// Convex occluders (r6).  When every triangle of the occluder tree lies on
// a convex six-faced solid — a connected set of triangles on the faces of
// the polyhedron their planes bound, three pairs of nearly opposite faces (a
// face in a culled plane may have no triangles, e.g. a block's bottom on the
// floor), bounded by the three slabs its corners span along one face normal
// of each pair —
// a shadow ray through the occluder tree can be answered without the walk:
//   * the segment [o, o + t_T d] misses the solid's three bounding slabs
//     pushed out by `delta`: no triangle of the solid can report a hit (the same
//     padded-volume argument as the BVH's padded boxes, with a margin 16x
//     theirs);
//   * the ray leaves the solid's face it starts on, not toward the face's
//     plane (d . n_face >= 0 over the face's own unit normal, `face_normal`):
//     the plane — a supporting plane of the convex solid — keeps the whole
//     segment ~1e-4 outside the solid, beyond the leaf test's reach;
//   * otherwise the leaf test of the triangles of the face the segment enters
//     (or leaves) the padded solid through, with the leaf test's arithmetic
//     and acceptance rule, certifies "occluded" exactly; if it does not, the
//     lane walks the occluder tree as before.
// Per solid: obb = (n0, n1, n2: unit axis normals, 9 floats; lo_a - delta,
// hi_a + delta for a = 0..2: 6 floats; 0), face_tris[2a + side] (side 0: the
// face opposite n_a's, 1: n_a's own face) = its two primitive ids
// (16 bits each, 0xFFFF = none).  `prim_face[t]` = solid * 8 + 2a + side + 1
// for the solids' triangles (0 elsewhere): the kernels read it from the
// primitive's shading record (p2.w).
struct ConvexSet {
  uint32_t count = 0;                              // solids (<= kMaxConvex)
  std::vector<std::array<float, 16>> obb;          // per solid, see above
  std::vector<std::array<uint32_t, 8>> face_tris;  // per solid: 6 faces (+2 unused, 0xFFFFFFFF)
  std::vector<std::array<float, 18>> face_normal;  // per solid: face k's outward unit normal at [3k, 3k+3)
  std::vector<uint32_t> prim_face;                 // per scene primitive, see above
  float delta = 0.0f;
};

bool find_convex_occluders(const float* vertices, size_t stride_bytes, uint32_t num_vertices, const uint32_t* indices,
                           uint32_t num_triangles, const std::vector<uint32_t>& keep, const OccluderSet& occ,
                           ConvexSet& out);

}  // namespace mrt
