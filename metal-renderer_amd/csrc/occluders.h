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

}  // namespace mrt
