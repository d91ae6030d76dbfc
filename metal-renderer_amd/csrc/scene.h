// scene.h — host-side scene import and flattening (the input contract of the
// hot path).  Mirrors initRaytracing (renderer/Renderer.mm:255-454): SceneKit
// OBJ/MTL import is replaced by our own parser with the same mapping
// (one geometry element per `usemtl`, Ka -> emission, Ks = (roughness,
// metalness, ior)), followed by the reference's element loop that builds
// TriangleReference / LightTriangle records and the light CDF + sentinel.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "mrt_layout.h"

namespace mrt {

struct SceneElement {
  uint32_t material = 0;               // index into materials (one SCNMaterial per element)
  std::vector<uint32_t> indices;       // 3 per triangle (uint32, SCNGeometryPrimitiveTypeTriangles)
};

struct HostScene {
  // import result (before flattening)
  std::vector<RefVertex> vertices;
  std::vector<RefMaterial> materials;
  std::vector<SceneElement> elements;
  // flattened (renderer/Renderer.mm:372-448)
  std::vector<uint32_t> indices;
  std::vector<RefTriangleReference> references;
  std::vector<RefLightTriangle> lights;   // light triangles + sentinel
  uint32_t light_count = 0;
};

// Parse an OBJ (+ its mtllib, or `mtl_override` when non-empty).  Handles CRLF,
// tabs, v / v/t / v//n / v/t/n corners, negative indices.
bool import_obj(const std::string& obj_path, const std::string& mtl_override, HostScene& scene,
                std::string& error);

// Material classification — renderer/Renderer.mm:278-329.
RefMaterial classify_material(const float kd[3], const float ka[3], const float ks[3]);

// Append a seeded, displaced lat-long sphere of exactly `triangles` triangles
// (rounded down to an even count) as one more diffuse element (BASELINE
// configs C4/C5: 1,048,576 triangles).  Deterministic for a given seed.
void append_procedural_mesh(HostScene& scene, uint32_t triangles, uint64_t seed);

// Run the element loop and light CDF (renderer/Renderer.mm:372-448).
void flatten(HostScene& scene);

}  // namespace mrt
