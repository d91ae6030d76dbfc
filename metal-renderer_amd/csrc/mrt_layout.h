// mrt_layout.h — data layouts shared by the host orchestration (C++) and the
// gfx950 kernels (HIP).  Plain structs of plain pointers; no torch types.
//
// Two families of layouts live here:
//   1. the REFERENCE AoS records (renderer/Raytracing.h:47-123), used only by
//      the stage-level C ABI (mrt_raygen / mrt_intersect / mrt_shade / ...)
//      so reference-layout buffers can be replayed for parity;
//   2. the MI355X-native layouts used by the fused wavefront path:
//        * ray queue: SoA of four float4 planes (16-B lane loads, 1 KiB per
//          wave instruction, fully coalesced);
//        * BVH4 nodes: 128-B component-major records (four child boxes +
//          refs) so one node visit is seven 16-B loads from one 128-B line;
//        * leaf triangles: {v0|prim, e1, e2} float4 triples in leaf order;
//        * per-primitive shading records (positions, normals, material and
//          light ids) in primitive order so a hit gathers 6 x 16 B with no
//          dependent index loads.
#pragma once
#include <stdint.h>

namespace mrt {

// ---- renderer/Raytracing.h:11-33 ------------------------------------------
constexpr float kDistanceEpsilon = 0.0001f;          // DISTANCE_EPSILON
constexpr float kAngleEpsilon = 0.00003807693583f;   // ANGLE_EPSILON
constexpr float kPi = 3.1415926f;                    // PI (truncated, as in the reference)
// rayGenerator's fixed camera origin up - view * 2.35 (renderer/Shaders.metal:75-103),
// shared by the kernels' camera_ray and the candidate-list builder (primary.cpp)
constexpr float kCameraX = 0.0f, kCameraY = 1.0f, kCameraZ = 2.35f;
constexpr unsigned kNoiseDim = 64;                   // NOISE_DIMENSIONS
constexpr unsigned kNoiseFloats = kNoiseDim * kNoiseDim * 4;
constexpr unsigned kTile = 64;                       // shard tile edge (== NOISE_DIMENSIONS)

// ---- renderer/Raytracing.h:35-43 ------------------------------------------
enum MaterialType : uint32_t { kDiffuse = 0, kMirror = 1, kPlastic = 2, kDielectric = 3 };

// ---- reference AoS records (renderer/Raytracing.h:47-123) -----------------
struct RefRay {               // Ray, 80 B (vector_float4 params is 16-B aligned)
  float origin[3]; float minDistance;
  float direction[3]; float maxDistance;
  float throughput[3]; float radiance[3];
  float pad_[2];
  float params[4];            // (material pdf, prev-is-diffuse, bounce, ior)
};
struct RefShadowRay {         // LightSamplingRay, 48 B
  float origin[3]; float minDistance;
  float direction[3]; float maxDistance;
  float throughput[3]; uint32_t targetIndex;
};
struct RefIntersection { float distance; uint32_t triangleIndex; float coordinates[2]; };  // 16 B
struct RefVertex { float v[3]; float n[3]; };                                              // 24 B
struct RefMaterial { float diffuse[3]; float emissive[3]; float ior; uint32_t materialType; };  // 32 B
struct RefTriangleReference { uint32_t tri[3]; uint32_t materialIndex; uint32_t lightTriangleIndex; };  // 20 B
struct RefLightTriangle {     // 100 B
  float emissive[3]; RefVertex v1, v2, v3; float area, pdf, cdf; uint32_t index;
};
static_assert(sizeof(RefRay) == 80, "RefRay");
static_assert(sizeof(RefShadowRay) == 48, "RefShadowRay");
static_assert(sizeof(RefIntersection) == 16, "RefIntersection");
static_assert(sizeof(RefVertex) == 24, "RefVertex");
static_assert(sizeof(RefMaterial) == 32, "RefMaterial");
static_assert(sizeof(RefTriangleReference) == 20, "RefTriangleReference");
static_assert(sizeof(RefLightTriangle) == 100, "RefLightTriangle");

// ---- device scene (MI355X layout) -----------------------------------------
// ref >= 0: interior node index; ref < 0: leaf, ~ref = (first << 4) | (count-1)
//
// BVH4 node i = nodes[8i .. 8i+7] (128 B, two 64-B lines), component-major so
// one 16-B load yields one box component for all four children:
//   [0] = lo.x[0..3]  [1] = hi.x[0..3]  [2] = lo.y[0..3]  [3] = hi.y[0..3]
//   [4] = lo.z[0..3]  [5] = hi.z[0..3]  [6] = bits(ref[0..3])  [7] = 0
// Unused child slots carry ref == kEmptyChild and an inverted box (lo = +inf,
// hi = -inf), which no slab test with the rows in ray order hits; traversals
// with rows in (lo, hi) order mask them by ref.

constexpr int32_t kEmptyChild = 0x7FFFFFFF;
constexpr int kLeafCountBits = 4;
constexpr int kMaxLeafSize = 1 << kLeafCountBits;   // 16
constexpr int kMaxBvhDepth = 32;                    // builder forces leaves below this binary depth
constexpr int kMaxStack = 64;                       // LDS traversal stack of the stage intersect kernel (host SAH BVH4 < 1.5 x depth)
constexpr int kMaxTraversalStack = 256;             // deepest supported tree (stack entries beyond LDS spill to global memory)
constexpr uint32_t kIntersectSpillGrid = 1024;      // persistent grid of the stage intersect kernel's spill variant

// Device-resident scene, passed to kernels by value.  Every pointer is
// 16-B aligned device memory; float pointers documented as "float4" hold
// 4 floats per record.
struct DeviceScene {
  const float* nodes;        // float4 x 8 per BVH4 node (see above)
  const float* tris;         // float4 x 3 per leaf-ordered triangle: (v0, bits(prim)), (e1, 0), (e2, 0)
  const float* prims;        // float4 x 6 per primitive (original order):
                             //   (p0, bits(material)), (p1, bits(light index or ~0u)), (p2, 0),
                             //   (n0, 0), (n1, 0), (n2, 0)
  const float* materials;    // float4 x 2 per material: (diffuse, ior), (emissive, bits(type))
  const float* lights;       // float4 x 7 per light entry (incl. sentinel):
                             //   (emissive, area), (v1.p, pdf), (v1.n, cdf), (v2.p, bits(index)),
                             //   (v2.n, 0), (v3.p, 0), (v3.n, 0)
  int32_t root;              // root node ref (may be a leaf ref for tiny scenes)
  uint32_t num_nodes;
  uint32_t num_triangles;
  uint32_t num_materials;
  uint32_t num_lights;       // light triangles, excluding the sentinel (SharedData.lightTrianglesCount)
  uint32_t lds_nodes;        // number of top nodes (BFS order) staged in LDS by the kernels
  uint32_t width;            // node width: 4 (BVH4; the only layout the kernels traverse)
  uint32_t max_stack;        // traversal stack entries a ray can need (<= kMaxTraversalStack; both trees)
  uint32_t light_shortcut;   // last-bounce nearest queries test the light triangles and then run one
                             // occlusion query (kernels.hip last_bounce_light_hit): <= kLightShortcutMax lights
  uint32_t origin_test;      // shadow rays test the triangle they leave before traversing (kernels.hip
                             // origin_occludes): on for deep trees (>= kOriginTestTriangles triangles)
  uint32_t region_grabs;     // path kernel: grab ranges are image bands over all frames (kernels.hip
                             // path_kernel refill): on for deep trees (>= kRegionGrabTriangles)
  // shadow-ray occluder tree (occluders.h): the BVH4 over the triangles that
  // are not in a culled plane, stored after the main tree — its nodes are
  // nodes [num_nodes, num_nodes + occ_nodes), its leaf triangles follow the
  // num_triangles main ones.  occ_planes == 0: none (shadow rays traverse
  // the main tree).  A shadow ray whose origin x has n.x - w <= -occ_margin
  // for every culled plane (n, w) traverses it from occ_root (kEmptyChild:
  // no triangle can occlude such a ray).
  int32_t occ_root;
  uint32_t occ_nodes;
  uint32_t occ_tris;
  uint32_t occ_planes;
  uint32_t occ_lights;       // the occluder tree holds no light triangle: queries through it test the
                             // other light triangles in a loop instead (kernels.hip lights_occlude)
  float occ_margin;
  float occ_cos_min;         // ... and whose cosine to the target light's (interpolated) normal is at least
                             // this (grazing guard for the light's own t error, occluders.cpp)
  float occ_plane[8][4];
  float occ_cos_min2;        // occ_cos_min squared (host-computed: a loop-invariant VALU product the stream kernel spilled)
  // convex occluders (occluders.h ConvexSet): when every triangle of the
  // occluder tree lies on one of conv_count parallelepiped solids, shadow rays
  // through it are answered by a segment-vs-solid test (kernels.hip
  // convex_occlusion): conv_obb[c] = three unit axis normals, then each
  // axis's padded slab (lo, hi); conv_face_tris[c][2a + side] = the face's
  // two primitive ids (16 bits each, 0xFFFF = none).  A primitive's shading
  // record carries (c * 8 + 2a + side + 1) in p2.w (0: not on a solid) and
  // its face's outward unit normal in n0.w, n1.w, n2.w.
  uint32_t conv_count;
  float conv_obb[4][16];             // [kMaxConvex]
  uint32_t conv_face_tris[4][8];
};
constexpr uint32_t kMaxOccPlanes = 8;
// convex occluders (DeviceScene::conv_*): at most this many solids, and the
// least d . n (n: the outward normal of the face a shadow ray starts on) for
// the ray to skip that face's solid (kernels.hip convex_occlusion)
constexpr uint32_t kMaxConvex = 4;
constexpr float kConvexLeaveDot = 1e-3f;
// the origin-triangle early-out pays where a shadow ray's descent to its own
// leaf goes through global memory: measured C4 (1M triangles) +2.6 %, C3
// (7 K) +0.5 % (with the path kernel's inline shadow finishes), C2 (36, the
// whole scene in LDS) 9747 / 9755 with it vs 9597 / 9859 and 9860 x 4
// without (r4, alternating A/B in one call)
constexpr uint32_t kOriginTestTriangles = 4096;
// block-major grab ranges (path kernel): measured (r4, alternating in one
// call) C4 +1.0 / +0.6 %, C5 1/8 share +0.2 / +0.4 %, C3 (7 K) -2.6 %
constexpr uint32_t kRegionGrabTriangles = 65536;
// the area-optimal BVH4 collapse (bvh.cpp) below this many triangles, the
// greedy one above (measured in renderer.cpp mrt_scene_create)
constexpr uint32_t kGreedyCollapseTriangles = 65536;
// light triangles tested per last-bounce ray by last_bounce_light_hit
constexpr uint32_t kLightShortcutMax = 16;
// occluder trees leave the light triangles out (tested in a loop per
// occlusion query, kernels.hip lights_occlude) up to this many lights
constexpr uint32_t kOccLightsMax = 8;

// camera-ray candidate lists (primary.h): header (offset << 8) | count per
// 8x8 pixel block; count kPrimaryFallback = traverse the BVH
constexpr uint32_t kPrimaryFallback = 0xFFu;
constexpr uint32_t kPrimaryBlock = 8;

// float4s per node record of a BVH width
#if defined(__HIPCC__)
#define MRT_HD __host__ __device__
#else
#define MRT_HD
#endif
MRT_HD constexpr uint32_t node_float4s(uint32_t width) { return 2u * width; }

}  // namespace mrt
