// ============================================================================
// mrt_oracle — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the metal-renderer hot path (serhii-rieznik/metal-renderer,
// read at /root/reference) used as the parity checker for the MI355X path
// tracer.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load this library; the product (metal-renderer_amd/) never links it.
//
// Provenance / pinning:
//   * The reference kernels are Metal Shading Language and need Apple's
//     <metal_stdlib>, MPS and SceneKit, none of which exist in this image, so
//     the reference is UNBUILDABLE here (no stand-in headers are written).
//   * This file restates, function by function, the reference's algorithm,
//     each function citing the file:line it follows.  Two closed-source pieces
//     are restated from their documented contract, and are "parity unpinned"
//     by the reference itself:
//       - MPSRayIntersector nearest-hit (renderer/Renderer.mm:464-469,519-523,
//         545-553): brute-force Moller-Trumbore, cull none, t in
//         [minDistance, maxDistance], distance = -1 on miss or maxDistance<0,
//         ties -> lowest primitive index, coordinates (u,v) = weights of
//         (V0,V1) (the convention interpolate() assumes,
//         renderer/KernelHelpers.h:39-42).
//       - SceneKit OBJ import (renderer/Renderer.mm:265-268): own OBJ/MTL
//         parser, one geometry element per `usemtl`, Ka -> emission.
//   * Pinned against the reference's only fixtures: the Mitsuba golden EXRs
//     in renderer/Media/reference (statistical: tests/test_oracle.py:22-48)
//     plus known-answer values derived from the reference source.
//   * The clock-seeded noise (renderer/Renderer.mm:109-112,486-490) is replaced
//     by the deterministic serialized schedule of SURVEY.md Appendix A.3.
//
// Arithmetic: IEEE binary32, built with -O2 -ffp-contract=off (no FMA
// contraction), correctly rounded sqrt/div; sin/cos are evaluated in double
// and rounded to float (correctly rounded in practice).  MSL float literals
// are single precision (all constants below carry an f suffix).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>
#include <fstream>
#include <sstream>
#include <atomic>
#include <mutex>

namespace {

// ---- renderer/Raytracing.h:11-33 (compile-time config) ---------------------
constexpr float kDistanceEpsilon = 0.0001f;          // Raytracing.h:16
constexpr float kAngleEpsilon = 0.00003807693583f;   // Raytracing.h:17
constexpr float kPi = 3.1415926f;                    // Raytracing.h:18
constexpr unsigned kNoiseDim = 64;                   // Raytracing.h:19

// ---- renderer/Raytracing.h:35-43 (material enum) ---------------------------
enum : uint32_t { MAT_DIFFUSE = 0, MAT_MIRROR = 1, MAT_PLASTIC = 2, MAT_DIELECTRIC = 3 };

// ---- renderer/Raytracing.h:47-123 (reference AoS records, same byte layout) -
struct SharedData { uint32_t frameIndex; uint32_t lightTrianglesCount; float time; };
struct Ray {                      // Raytracing.h:54-69 — 80 bytes
  float origin[3]; float minDistance;
  float direction[3]; float maxDistance;
  float throughput[3]; float radiance[3];
  float _pad[2];                  // vector_float4 params is 16-B aligned
  float params[4];                // (material pdf, prev-is-diffuse, bounce, ior)
};
struct LightSamplingRay {         // Raytracing.h:71-83 — 48 bytes
  float origin[3]; float minDistance;
  float direction[3]; float maxDistance;
  float throughput[3]; uint32_t targetIndex;
};
struct Intersection { float distance; uint32_t triangleIndex; float coordinates[2]; };  // :85-90
struct Vertex { float v[3]; float n[3]; };                                              // :92-96
struct Material { float diffuse[3]; float emissive[3]; float ior; uint32_t materialType; };  // :98-104
struct TriangleReference { uint32_t tri[3]; uint32_t materialIndex; uint32_t lightTriangleIndex; };  // :106-111
struct LightTriangle {            // :113-123 — 100 bytes
  float emissive[3]; Vertex v1, v2, v3; float area, pdf, cdf; uint32_t index;
};
static_assert(sizeof(Ray) == 80, "Ray layout");
static_assert(sizeof(LightSamplingRay) == 48, "LightSamplingRay layout");
static_assert(sizeof(Intersection) == 16, "Intersection layout");
static_assert(sizeof(Vertex) == 24, "Vertex layout");
static_assert(sizeof(Material) == 32, "Material layout");
static_assert(sizeof(TriangleReference) == 20, "TriangleReference layout");
static_assert(sizeof(LightTriangle) == 100, "LightTriangle layout");

// ---- small float3 helper with explicit evaluation order --------------------
struct F3 { float x, y, z; };
static inline F3 f3(const float* p) { return {p[0], p[1], p[2]}; }
static inline void st3(float* p, F3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
static inline F3 add(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline F3 mul(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline F3 neg(F3 a) { return {-a.x, -a.y, -a.z}; }
static inline float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline F3 cross(F3 a, F3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline float length(F3 a) { return std::sqrt(dot(a, a)); }
// normalize(x) = x * (1/sqrt(dot(x,x)))  (MSL normalize; IEEE form)
static inline F3 normalize(F3 a) { float inv = 1.0f / std::sqrt(dot(a, a)); return mul(a, inv); }
// MSL reflect(I, N) = I - 2 * dot(N, I) * N
static inline F3 reflect(F3 i, F3 n) { float k = 2.0f * dot(n, i); return sub(i, mul(n, k)); }
static inline float clampf(float x, float lo, float hi) { return std::fmin(std::fmax(x, lo), hi); }
static inline float sin_cr(float x) { return (float)std::sin((double)x); }
static inline float cos_cr(float x) { return (float)std::cos((double)x); }
// MSL mix(x, y, a) = x + (y - x) * a
static inline float mixf(float x, float y, float a) { return x + (y - x) * a; }

// ============================================================================
// Scene flattening — renderer/Renderer.mm:255-454 (initRaytracing), with the
// SceneKit OBJ import restated (parity unpinned, see header).
// ============================================================================
struct Scene {
  std::vector<Vertex> vertices;
  std::vector<uint32_t> indices;
  std::vector<Material> materials;
  std::vector<TriangleReference> references;
  std::vector<LightTriangle> lightTriangles;   // includes the sentinel
  uint32_t lightTrianglesCount = 0;
  std::string error;
  // Triangle planes (v0, e1 = v1 - v0, e2 = v2 - v0) in SoA form for the
  // packet brute force of large scenes (built on first use; see
  // intersect_packet).  The same float values tri_hit derives per test.
  mutable std::once_flag soa_once;
  mutable std::vector<float> soa;   // [9][T]
  // A binary SAH BVH over the same triangles for the CPU baseline (SURVEY.md
  // 8(d): "same BVH" as the GPU path rather than brute force), built on first
  // use (see build_cpu_bvh / intersect_bvh).
  mutable std::once_flag bvh_once;
  mutable std::vector<struct CpuBvhNode> bvh;
  mutable std::vector<uint32_t> bvh_prims;
};

// BVH node of the CPU baseline: a padded box and either two children
// (count == 0: left child = node + 1, right = `right`) or a leaf of `count`
// triangles bvh_prims[first .. first + count).
struct CpuBvhNode {
  float lo[3], hi[3];
  uint32_t right_or_first;
  uint32_t count;
};

struct MtlColor { float r = 0, g = 0, b = 0; bool set = false; };
struct MtlEntry { MtlColor kd, ka, ks; };

static std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r' || s[a] == '\n')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r' || s[b - 1] == '\n')) --b;
  return s.substr(a, b - a);
}

static bool parse_mtl(const std::string& path, std::unordered_map<std::string, MtlEntry>& out,
                      std::string& err) {
  std::ifstream f(path);
  if (!f) { err = "cannot open mtl " + path; return false; }
  std::string line, cur;
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ss(line);
    std::string key; ss >> key;
    if (key == "newmtl") { ss >> cur; out[cur]; continue; }
    if (cur.empty()) continue;
    auto readc = [&](MtlColor& c) {
      std::string a, b, d; ss >> a >> b >> d;
      c.r = std::strtof(a.c_str(), nullptr); c.g = std::strtof(b.c_str(), nullptr);
      c.b = std::strtof(d.c_str(), nullptr); c.set = true;
    };
    if (key == "Kd") readc(out[cur].kd);
    else if (key == "Ka") readc(out[cur].ka);
    else if (key == "Ks") readc(out[cur].ks);
    // any other key (Kx, illum, ...) is ignored, as by the reference
  }
  return true;
}

// Material classification — renderer/Renderer.mm:278-329.
static Material classify(const MtlEntry& m) {
  Material mtl{};
  mtl.diffuse[0] = m.kd.r; mtl.diffuse[1] = m.kd.g; mtl.diffuse[2] = m.kd.b;   // :286-288
  mtl.emissive[0] = m.ka.r; mtl.emissive[1] = m.ka.g; mtl.emissive[2] = m.ka.b; // :289-291 (Ka->emission)
  mtl.ior = m.ks.b;                                                               // :292
  float roughness = m.ks.r, metallness = m.ks.g;                                  // :294-295
  mtl.materialType = MAT_DIFFUSE;  // value-initialised (rough conductor, :305)
  if (metallness > 0.0f) {                                                        // :297-307
    if (roughness == 0.0f) mtl.materialType = MAT_MIRROR;
  } else if (roughness == 1.0f) {                                                 // :308-311
    mtl.materialType = MAT_DIFFUSE;
  } else if (mtl.ior <= 0.0f) {                                                   // :312-316
    mtl.ior = std::fabs(mtl.ior);
    mtl.materialType = (roughness == 0.0f) ? MAT_PLASTIC : MAT_DIFFUSE;
  } else {                                                                        // :317-320
    mtl.materialType = (roughness == 0.0f) ? MAT_DIELECTRIC : MAT_DIFFUSE;
  }
  return mtl;
}

static bool load_scene(const char* obj_path, const char* mtl_override, Scene& sc) {
  std::ifstream f(obj_path);
  if (!f) { sc.error = std::string("cannot open obj ") + obj_path; return false; }
  std::string dir(obj_path);
  size_t slash = dir.find_last_of('/');
  dir = (slash == std::string::npos) ? std::string() : dir.substr(0, slash + 1);

  std::unordered_map<std::string, MtlEntry> mtls;
  std::vector<F3> pos, nrm;
  struct Elem { std::string mtl; std::vector<uint32_t> idx; };
  std::vector<Elem> elems;
  std::unordered_map<std::string, uint32_t> vmap;   // "vi/vni" -> vertex id
  std::vector<Vertex>& verts = sc.vertices;
  bool mtl_loaded = false;
  if (mtl_override && *mtl_override) {
    if (!parse_mtl(mtl_override, mtls, sc.error)) return false;
    mtl_loaded = true;
  }
  std::string line;
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ss(line);
    std::string key; ss >> key;
    if (key == "v") {
      std::string a, b, c; ss >> a >> b >> c;
      pos.push_back({std::strtof(a.c_str(), nullptr), std::strtof(b.c_str(), nullptr), std::strtof(c.c_str(), nullptr)});
    } else if (key == "vn") {
      std::string a, b, c; ss >> a >> b >> c;
      nrm.push_back({std::strtof(a.c_str(), nullptr), std::strtof(b.c_str(), nullptr), std::strtof(c.c_str(), nullptr)});
    } else if (key == "mtllib") {
      std::string name; ss >> name;
      if (!mtl_loaded) { if (!parse_mtl(dir + name, mtls, sc.error)) return false; mtl_loaded = true; }
    } else if (key == "usemtl") {
      std::string name; ss >> name;
      elems.push_back({name, {}});
    } else if (key == "f") {
      if (elems.empty()) elems.push_back({"", {}});
      std::vector<uint32_t> corners;
      std::string tok;
      while (ss >> tok) {
        int vi = 0, ti = 0, ni = 0;
        // forms: v, v/t, v//n, v/t/n
        const char* p = tok.c_str();
        vi = std::atoi(p);
        const char* s1 = std::strchr(p, '/');
        if (s1) {
          if (s1[1] != '/') ti = std::atoi(s1 + 1);
          const char* s2 = std::strchr(s1 + 1, '/');
          if (s2) ni = std::atoi(s2 + 1);
        }
        (void)ti;
        if (vi < 0) vi = (int)pos.size() + 1 + vi;
        if (ni < 0) ni = (int)nrm.size() + 1 + ni;
        std::string key2 = std::to_string(vi) + "/" + std::to_string(ni);
        auto it = vmap.find(key2);
        uint32_t id;
        if (it == vmap.end()) {
          Vertex vx{};
          F3 P = pos.at(vi - 1); vx.v[0] = P.x; vx.v[1] = P.y; vx.v[2] = P.z;
          if (ni > 0) { F3 N = nrm.at(ni - 1); vx.n[0] = N.x; vx.n[1] = N.y; vx.n[2] = N.z; }
          id = (uint32_t)verts.size(); verts.push_back(vx); vmap.emplace(key2, id);
        } else id = it->second;
        corners.push_back(id);
      }
      for (size_t k = 1; k + 1 < corners.size(); ++k) {   // fan (all shipped faces are triangles)
        elems.back().idx.push_back(corners[0]);
        elems.back().idx.push_back(corners[k]);
        elems.back().idx.push_back(corners[k + 1]);
      }
    }
  }
  // drop empty elements (a usemtl without faces produces no SceneKit element)
  std::vector<Elem> el2;
  for (auto& e : elems) if (!e.idx.empty()) el2.push_back(std::move(e));
  // one SCNMaterial per element (geometry.materials), renderer/Renderer.mm:278
  for (auto& e : el2) {
    auto it = mtls.find(e.mtl);
    sc.materials.push_back(classify(it == mtls.end() ? MtlEntry{} : it->second));
  }
  // triangle references and light triangles — renderer/Renderer.mm:372-432
  float totalArea = 0.0f;
  const size_t M = sc.materials.size();
  for (size_t k = 0; k < el2.size(); ++k) {
    size_t materialIndex = k % M;                                            // :377
    const Material& mat = sc.materials[materialIndex];
    bool isEmitter = (mat.emissive[0] > 0.0f) || (mat.emissive[1] > 0.0f) || (mat.emissive[2] > 0.0f);  // :378-381
    const std::vector<uint32_t>& raw = el2[k].idx;
    for (size_t i = 0; i + 2 < raw.size(); i += 3) {
      uint32_t lightTriangleIndex = 0xFFFFFFFFu;
      if (isEmitter) {                                                         // :394-413
        const Vertex& v1 = sc.vertices[raw[i]];
        const Vertex& v2 = sc.vertices[raw[i + 1]];
        const Vertex& v3 = sc.vertices[raw[i + 2]];
        F3 p1 = f3(v1.v), p2 = f3(v2.v), p3 = f3(v3.v);
        lightTriangleIndex = (uint32_t)sc.lightTriangles.size();
        LightTriangle lt{};
        lt.index = (uint32_t)sc.references.size();
        lt.v1 = v1; lt.v2 = v2; lt.v3 = v3;
        lt.area = 0.5f * length(cross(sub(p2, p1), sub(p3, p1)));
        lt.emissive[0] = mat.emissive[0]; lt.emissive[1] = mat.emissive[1]; lt.emissive[2] = mat.emissive[2];
        totalArea += lt.area;
        sc.lightTriangles.push_back(lt);
      }
      TriangleReference r{};
      r.materialIndex = (uint32_t)materialIndex;
      r.lightTriangleIndex = lightTriangleIndex;
      r.tri[0] = raw[i]; r.tri[1] = raw[i + 1]; r.tri[2] = raw[i + 2];
      sc.references.push_back(r);
      sc.indices.push_back(raw[i]); sc.indices.push_back(raw[i + 1]); sc.indices.push_back(raw[i + 2]);
    }
  }
  // light pdf / cdf + sentinel — renderer/Renderer.mm:435-448
  float cdf = 0.0f;
  for (LightTriangle& lt : sc.lightTriangles) { lt.pdf = lt.area / totalArea; lt.cdf = cdf; cdf += lt.pdf; }
  sc.lightTrianglesCount = (uint32_t)sc.lightTriangles.size();
  LightTriangle sentinel{};
  sentinel.cdf = cdf; sentinel.pdf = 1.0f; sentinel.area = 0.0f;
  sc.lightTriangles.push_back(sentinel);
  return true;
}

// ============================================================================
// Noise — renderer/Renderer.mm:109-129 (initial table) and :486-496 (per
// frame), with the clock replaced by a fixed 64-bit seed.
// ============================================================================
static void noise_table(uint64_t seed, int64_t frame, float* out) {
  uint32_t lo = (uint32_t)(seed & 0xffffffffu), hi = (uint32_t)(seed >> 32);
  if (frame >= 0) { lo ^= (uint32_t)(frame + 1); hi ^= (uint32_t)(frame + 3); }
  std::seed_seq ss{lo, hi};
  std::mt19937_64 rng;
  rng.seed(ss);
  std::uniform_real_distribution<float> distribution(0.0f, 1.0f);
  for (unsigned i = 0; i < kNoiseDim * kNoiseDim * 4; ++i) out[i] = distribution(rng);
}

// ============================================================================
// MPS nearest-hit, restated as brute force (see header).
// ============================================================================
static inline bool tri_hit(F3 o, F3 d, F3 v0, F3 v1, F3 v2, float tmin, float tmax,
                           float& t, float& u, float& v) {
  F3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  F3 p = cross(d, e2);
  float det = dot(e1, p);
  if (det == 0.0f) return false;
  float inv = 1.0f / det;
  F3 s = sub(o, v0);
  float b1 = dot(s, p) * inv;
  if (!(b1 >= 0.0f && b1 <= 1.0f)) return false;
  F3 q = cross(s, e1);
  float b2 = dot(d, q) * inv;
  if (!(b2 >= 0.0f && b1 + b2 <= 1.0f)) return false;
  float tt = dot(e2, q) * inv;
  if (!(tt >= tmin && tt <= tmax)) return false;
  t = tt; u = (1.0f - b1) - b2; v = b1;
  return true;
}

static Intersection intersect_one(const Scene& sc, const float* o3, float tmin, const float* d3, float tmax) {
  Intersection r{-1.0f, 0xFFFFFFFFu, {0.0f, 0.0f}};
  if (tmax < 0.0f) return r;   // disabled ray (renderer/Shaders.metal:119,124,173)
  F3 o = f3(o3), d = f3(d3);
  const size_t T = sc.references.size();
  bool found = false;
  float bt = 0, bu = 0, bv = 0; uint32_t bk = 0;
  for (size_t k = 0; k < T; ++k) {
    const uint32_t* tri = sc.references[k].tri;
    float t, u, v;
    if (!tri_hit(o, d, f3(sc.vertices[tri[0]].v), f3(sc.vertices[tri[1]].v), f3(sc.vertices[tri[2]].v),
                 tmin, tmax, t, u, v)) continue;
    if (!found || t < bt) { found = true; bt = t; bu = u; bv = v; bk = (uint32_t)k; }
  }
  if (found) { r.distance = bt; r.triangleIndex = bk; r.coordinates[0] = bu; r.coordinates[1] = bv; }
  return r;
}

// ---- CPU baseline traversal: binned-SAH BVH2 (own build, scalar) ----------
// Conservative boxes (padded outward as the GPU builder pads, bvh.cpp) and
// the same per-triangle test (tri_hit) with the brute force's tie rule
// (nearest t, then lowest primitive index), so intersect_bvh returns exactly
// intersect_one's answer; it is what the cpu_baseline leg times.
struct BuildRef { float lo[3], hi[3], c[3]; uint32_t prim; };

static void grow(float* lo, float* hi, const float* l2, const float* h2) {
  for (int a = 0; a < 3; ++a) { lo[a] = std::fmin(lo[a], l2[a]); hi[a] = std::fmax(hi[a], h2[a]); }
}
static float half_area(const float* lo, const float* hi) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}

// Depth bound: below kSahDepth every split is a median split of the range,
// so a tree is at most kSahDepth + 32 levels deep (< 2^32 primitives) and
// intersect_bvh's fixed stack of kCpuStack entries (one push per level) never
// overflows, whatever the SAH would do on a degenerate procedural scene.
constexpr uint32_t kSahDepth = 90, kCpuStack = 128;
static_assert(kSahDepth + 32 <= kCpuStack, "oracle BVH stack");

static uint32_t build_node(const Scene& sc, std::vector<BuildRef>& refs, uint32_t b, uint32_t e, uint32_t depth) {
  const uint32_t node = (uint32_t)sc.bvh.size();
  sc.bvh.push_back(CpuBvhNode{});
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (uint32_t i = b; i < e; ++i) { grow(lo, hi, refs[i].lo, refs[i].hi); grow(clo, chi, refs[i].c, refs[i].c); }
  for (int a = 0; a < 3; ++a) {   // outward padding: the slab test stays conservative under rounding
    const float m = std::fmax(std::fabs(lo[a]), std::fabs(hi[a])), pad = 1e-5f * m + 1e-6f;
    sc.bvh[node].lo[a] = lo[a] - pad;
    sc.bvh[node].hi[a] = hi[a] + pad;
  }
  const uint32_t n = e - b;
  auto make_leaf = [&]() {
    sc.bvh[node].right_or_first = (uint32_t)sc.bvh_prims.size();
    sc.bvh[node].count = n;
    for (uint32_t i = b; i < e; ++i) sc.bvh_prims.push_back(refs[i].prim);
    return node;
  };
  if (n <= 4) return make_leaf();
  if (depth >= kSahDepth) {   // median split (depth bound above)
    const uint32_t mid = b + n / 2;
    build_node(sc, refs, b, mid, depth + 1);
    const uint32_t right = build_node(sc, refs, mid, e, depth + 1);
    sc.bvh[node].right_or_first = right;
    sc.bvh[node].count = 0;
    return node;
  }
  // 16-bin SAH on the centroid bounds' longest axis
  int axis = 0;
  for (int a = 1; a < 3; ++a) if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
  const float ext = chi[axis] - clo[axis];
  if (!(ext > 0.0f)) return make_leaf();
  constexpr int kBins = 16;
  float blo[kBins][3], bhi[kBins][3];
  uint32_t bcnt[kBins] = {};
  for (int k = 0; k < kBins; ++k) for (int a = 0; a < 3; ++a) { blo[k][a] = INFINITY; bhi[k][a] = -INFINITY; }
  auto bin_of = [&](const BuildRef& r) { return std::min(kBins - 1, (int)((r.c[axis] - clo[axis]) / ext * kBins)); };
  for (uint32_t i = b; i < e; ++i) { const int k = bin_of(refs[i]); ++bcnt[k]; grow(blo[k], bhi[k], refs[i].lo, refs[i].hi); }
  float best = INFINITY;
  int split = -1;
  for (int s = 1; s < kBins; ++s) {
    float l0[3] = {INFINITY, INFINITY, INFINITY}, l1[3] = {-INFINITY, -INFINITY, -INFINITY};
    float r0[3] = {INFINITY, INFINITY, INFINITY}, r1[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nl = 0, nr = 0;
    for (int k = 0; k < s; ++k) if (bcnt[k]) { grow(l0, l1, blo[k], bhi[k]); nl += bcnt[k]; }
    for (int k = s; k < kBins; ++k) if (bcnt[k]) { grow(r0, r1, blo[k], bhi[k]); nr += bcnt[k]; }
    if (!nl || !nr) continue;
    const float cost = half_area(l0, l1) * nl + half_area(r0, r1) * nr;
    if (cost < best) { best = cost; split = s; }
  }
  uint32_t mid;
  if (split < 0) {
    mid = b + n / 2;
  } else {
    mid = (uint32_t)(std::partition(refs.begin() + b, refs.begin() + e,
                                    [&](const BuildRef& r) { return bin_of(r) < split; }) - refs.begin());
    if (mid == b || mid == e) mid = b + n / 2;
  }
  build_node(sc, refs, b, mid, depth + 1);   // left child = node + 1
  const uint32_t right = build_node(sc, refs, mid, e, depth + 1);
  sc.bvh[node].right_or_first = right;
  sc.bvh[node].count = 0;
  return node;
}

static void build_cpu_bvh(const Scene& sc) {
  const size_t T = sc.references.size();
  std::vector<BuildRef> refs(T);
  for (size_t k = 0; k < T; ++k) {
    BuildRef& r = refs[k];
    r.prim = (uint32_t)k;
    for (int a = 0; a < 3; ++a) { r.lo[a] = INFINITY; r.hi[a] = -INFINITY; }
    for (int j = 0; j < 3; ++j) {
      const float* v = sc.vertices[sc.references[k].tri[j]].v;
      grow(r.lo, r.hi, v, v);
    }
    for (int a = 0; a < 3; ++a) r.c[a] = 0.5f * (r.lo[a] + r.hi[a]);
  }
  sc.bvh.reserve(T);
  sc.bvh_prims.reserve(T);
  if (T) build_node(sc, refs, 0, (uint32_t)T, 0);
}

static inline float safe_inv(float d) { return 1.0f / (std::fabs(d) > 1e-20f ? d : std::copysign(1e-20f, d)); }

// Culling rule of the CPU BVH's traversal.  It must not share the kernels'
// error mode (their children are culled beyond h.t * (1 + 2^-11), kernels.hip
// kCullScale), or a triangle the kernels miss by the same
// rounding would be missed here too and the comparison would pass:
//   kCullWide — boxes culled only beyond bt * (1 + 2^-6): strictly more
//               conservative than the kernels' slack, so a kernel answer equal
//               to this one shows the kernels' slack sufficed for that ray;
//   kCullNone — no culling by the current hit at all: every box whose slab
//               interval meets [tmin, tmax] is visited, which is the brute
//               force over every triangle whose padded box the ray enters.
enum CullMode : int { kCullWide = 0, kCullNone = 1 };

static Intersection intersect_bvh(const Scene& sc, const float* o3, float tmin, const float* d3, float tmax,
                                  int cull = kCullWide) {
  Intersection r{-1.0f, 0xFFFFFFFFu, {0.0f, 0.0f}};
  if (tmax < 0.0f) return r;   // disabled ray (renderer/Shaders.metal:119,124,173)
  std::call_once(sc.bvh_once, build_cpu_bvh, std::cref(sc));
  if (sc.bvh.empty()) return r;
  const F3 o = f3(o3), d = f3(d3);
  const float inv[3] = {safe_inv(d.x), safe_inv(d.y), safe_inv(d.z)};
  const float oo[3] = {o.x, o.y, o.z};
  bool found = false;
  float bt = tmax, bu = 0, bv = 0;
  uint32_t bk = 0;
  const float ray_tmax = tmax;
  auto box = [&](uint32_t n, float& tn) {
    const CpuBvhNode& b = sc.bvh[n];
    float t0 = tmin, t1 = cull == kCullNone ? ray_tmax : bt * (1.0f + 0x1p-6f);
    for (int a = 0; a < 3; ++a) {
      const float x0 = (b.lo[a] - oo[a]) * inv[a], x1 = (b.hi[a] - oo[a]) * inv[a];
      t0 = std::fmax(t0, std::fmin(x0, x1));
      t1 = std::fmin(t1, std::fmax(x0, x1));
    }
    tn = t0;
    return t0 <= t1;
  };
  uint32_t stack[kCpuStack];   // <= depth entries (build_node's bound)
  int sp = 0;
  uint32_t node = 0;
  float tn0;
  if (!box(0, tn0)) return r;
  for (;;) {
    const CpuBvhNode& nd = sc.bvh[node];
    if (nd.count) {
      for (uint32_t i = 0; i < nd.count; ++i) {
        const uint32_t k = sc.bvh_prims[nd.right_or_first + i];
        const uint32_t* tri = sc.references[k].tri;
        float t, u, v;
        if (!tri_hit(o, d, f3(sc.vertices[tri[0]].v), f3(sc.vertices[tri[1]].v), f3(sc.vertices[tri[2]].v),
                     tmin, bt, t, u, v)) continue;
        if (!found || t < bt || k < bk) { found = true; bt = t; bu = u; bv = v; bk = k; }
      }
    } else {
      const uint32_t l = node + 1, rr = nd.right_or_first;
      float tl, tr;
      const bool hl = box(l, tl), hr = box(rr, tr);
      if (hl && hr) {
        const bool lf = tl <= tr;
        stack[sp++] = lf ? rr : l;
        node = lf ? l : rr;
        continue;
      }
      if (hl || hr) { node = hl ? l : rr; continue; }
    }
    // pop (re-testing the box against the current nearest hit)
    bool next = false;
    while (sp > 0) {
      node = stack[--sp];
      float tn;
      if (box(node, tn)) { next = true; break; }
    }
    if (!next) break;
  }
  if (found) { r.distance = bt; r.triangleIndex = bk; r.coordinates[0] = bu; r.coordinates[1] = bv; }
  return r;
}

// The same brute force for a packet of rays over a large scene: triangles in
// blocks of kPacketBlock (SoA planes, resident in L2) with every ray of the
// packet tested against a block before the next block streams in.  Each test
// is tri_hit's arithmetic in a branch-free (vectorisable) form, and triangles
// are visited in increasing index order per ray with the strict `t < best`
// rule, so the result is exactly intersect_one's (ties -> lowest index).
constexpr size_t kPacketBlock = 2048;

static void build_soa(const Scene& sc) {
  const size_t T = sc.references.size();
  sc.soa.assign(9 * T, 0.0f);
  for (size_t k = 0; k < T; ++k) {
    const uint32_t* tri = sc.references[k].tri;
    const F3 v0 = f3(sc.vertices[tri[0]].v), v1 = f3(sc.vertices[tri[1]].v), v2 = f3(sc.vertices[tri[2]].v);
    const F3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const float c[9] = {v0.x, v0.y, v0.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z};
    for (int j = 0; j < 9; ++j) sc.soa[(size_t)j * T + k] = c[j];
  }
}

// hit flags and distances of one ray against triangles [b, e) (branch free)
__attribute__((target_clones("avx512f", "avx2", "default")))
static uint32_t block_tests(const float* __restrict__ soa, size_t T, size_t b, size_t e, F3 o, F3 d, float tmin,
                        float tmax, float* __restrict__ t_out, uint8_t* __restrict__ hit_out) {
  const float* __restrict__ v0x = soa + b; const float* __restrict__ v0y = soa + T + b;
  const float* __restrict__ v0z = soa + 2 * T + b; const float* __restrict__ e1x = soa + 3 * T + b;
  const float* __restrict__ e1y = soa + 4 * T + b; const float* __restrict__ e1z = soa + 5 * T + b;
  const float* __restrict__ e2x = soa + 6 * T + b; const float* __restrict__ e2y = soa + 7 * T + b;
  const float* __restrict__ e2z = soa + 8 * T + b;
  const size_t n = e - b;
  uint32_t hits = 0;
  for (size_t k = 0; k < n; ++k) {
    // p = cross(d, e2); det = dot(e1, p)
    const float px = d.y * e2z[k] - d.z * e2y[k], py = d.z * e2x[k] - d.x * e2z[k], pz = d.x * e2y[k] - d.y * e2x[k];
    const float det = (e1x[k] * px + e1y[k] * py) + e1z[k] * pz;
    const float inv = 1.0f / det;
    const float sx = o.x - v0x[k], sy = o.y - v0y[k], sz = o.z - v0z[k];
    const float b1 = ((sx * px + sy * py) + sz * pz) * inv;
    // q = cross(s, e1)
    const float qx = sy * e1z[k] - sz * e1y[k], qy = sz * e1x[k] - sx * e1z[k], qz = sx * e1y[k] - sy * e1x[k];
    const float b2 = ((d.x * qx + d.y * qy) + d.z * qz) * inv;
    const float tt = ((e2x[k] * qx + e2y[k] * qy) + e2z[k] * qz) * inv;
    const bool hit = (det != 0.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f) &
                     (tt >= tmin) & (tt <= tmax);
    t_out[k] = tt;
    hit_out[k] = hit;
    hits += hit;
  }
  return hits;
}

static void intersect_packet(const Scene& sc, const float* const* o3, const float* tmin, const float* const* d3,
                             const float* tmax, size_t n, Intersection* out) {
  std::call_once(sc.soa_once, build_soa, std::cref(sc));
  const size_t T = sc.references.size();
  std::vector<uint8_t> found(n, 0);
  std::vector<float> bt(n, 0.0f);
  std::vector<uint32_t> bk(n, 0);
  float t_blk[kPacketBlock];
  uint8_t hit_blk[kPacketBlock];
  for (size_t b = 0; b < T; b += kPacketBlock) {
    const size_t e = std::min(T, b + kPacketBlock);
    for (size_t r = 0; r < n; ++r) {
      if (tmax[r] < 0.0f) continue;
      if (!block_tests(sc.soa.data(), T, b, e, f3(o3[r]), f3(d3[r]), tmin[r], tmax[r], t_blk, hit_blk)) continue;
      for (size_t k = 0; k < e - b; ++k)
        if (hit_blk[k] && (!found[r] || t_blk[k] < bt[r])) { found[r] = 1; bt[r] = t_blk[k]; bk[r] = (uint32_t)(b + k); }
    }
  }
  for (size_t r = 0; r < n; ++r) {
    if (!found[r]) { out[r] = Intersection{-1.0f, 0xFFFFFFFFu, {0.0f, 0.0f}}; continue; }
    // (u, v) of the winning triangle: tri_hit's own expressions
    const uint32_t* tri = sc.references[bk[r]].tri;
    float t, u, v;
    const bool ok = tri_hit(f3(o3[r]), f3(d3[r]), f3(sc.vertices[tri[0]].v), f3(sc.vertices[tri[1]].v),
                            f3(sc.vertices[tri[2]].v), tmin[r], tmax[r], t, u, v);
    (void)ok;
    out[r] = Intersection{bt[r], bk[r], {u, v}};
  }
}

// ============================================================================
// Device helpers — renderer/KernelHelpers.h and renderer/Raytracing.h
// ============================================================================
// fresnel — KernelHelpers.h:7-21
static float fresnel(F3 n, F3 i, float etaOut, float etaIn) {
  float result = 1.0f;
  float etaScale = etaOut / etaIn;
  float cosThetaI = clampf(dot(n, i), -1.0f, 1.0f);
  float sinThetaTSquared = (etaScale * etaScale) * (1.0f - cosThetaI * cosThetaI);
  if (sinThetaTSquared < 1.0f) {
    float cosThetaT = std::sqrt(1.0f - sinThetaTSquared);
    float rS = (etaIn * cosThetaI - etaOut * cosThetaT) / (etaIn * cosThetaI + etaOut * cosThetaT);
    float rP = (etaIn * cosThetaT - etaOut * cosThetaI) / (etaIn * cosThetaT + etaOut * cosThetaI);
    result = 0.5f * (rS * rS + rP * rP);
  }
  return result;
}
// interpolate (float3 weights) — KernelHelpers.h:23-35
static Vertex interpolate3(const Vertex& t0, const Vertex& t1, const Vertex& t2, F3 w) {
  Vertex r;
  F3 p = add(add(mul(f3(t0.v), w.x), mul(f3(t1.v), w.y)), mul(f3(t2.v), w.z));
  F3 n = normalize(add(add(mul(f3(t0.n), w.x), mul(f3(t1.n), w.y)), mul(f3(t2.n), w.z)));
  st3(r.v, p); st3(r.n, n);
  return r;
}
// interpolate (float2 coordinates) — KernelHelpers.h:37-47
static Vertex interpolate2(const Vertex& t0, const Vertex& t1, const Vertex& t2, const float* uv) {
  return interpolate3(t0, t1, t2, {uv[0], uv[1], (1.0f - uv[0]) - uv[1]});
}
// selectLightTriangle — KernelHelpers.h:49-54
static const LightTriangle& selectLightTriangle(float xi, const LightTriangle* lt, int count) {
  int index = 0;
  for (; (index < count) && (lt[index + 1].cdf <= xi); ++index) {}
  return lt[index];
}
// triangleSamplePDF — Raytracing.h:168-171
static float triangleSamplePDF(float area, float cosTheta, float dist) {
  return (dist * dist) / (area * cosTheta);
}
// balanceHeuristic (a power heuristic) — Raytracing.h:173-178
static float balanceHeuristic(float f, float g) { float f2 = f * f, g2 = g * g; return f2 / (f2 + g2); }
// barycentric — Raytracing.h:182-187
static F3 barycentric(float sx, float sy) {
  float r1 = std::sqrt(sx), r2 = sy;
  return {1.0f - r1, r1 * (1.0f - r2), r1 * r2};
}
// buildOrthonormalBasis — Raytracing.h:189-205
static void buildOrthonormalBasis(F3 n, F3& u, F3& v) {
  if (n.z < 0.0f) {
    float a = 1.0f / (1.0f - n.z);
    float b = n.x * n.y * a;
    u = {1.0f - n.x * n.x * a, -b, n.x};
    v = {b, n.y * n.y * a - 1.0f, -n.y};
  } else {
    float a = 1.0f / (1.0f + n.z);
    float b = -n.x * n.y * a;
    u = {1.0f - n.x * n.x * a, b, -n.x};
    v = {b, 1.0f - n.y * n.y * a, -n.y};
  }
}
// alignWithNormal — Raytracing.h:207-216
static F3 alignWithNormal(F3 n, float cosTheta, float phi) {
  float sinTheta = std::sqrt(1.0f - cosTheta * cosTheta);
  F3 u, v; buildOrthonormalBasis(n, u, v);
  float cp = cos_cr(phi), sp = sin_cr(phi);
  return add(mul(add(mul(u, cp), mul(v, sp)), sinTheta), mul(n, cosTheta));
}
// generateDiffuseBounce — Raytracing.h:218-223 (smp = noise.zw)
static F3 generateDiffuseBounce(float sx, float sy, F3 n) {
  float cosTheta = std::sqrt(sy);
  float phi = sx * kPi * 2.0f;
  return alignWithNormal(n, cosTheta, phi);
}
static bool isMirrorDir(F3 wI, F3 n, F3 wO) {
  return std::fabs(dot(reflect(wI, n), wO) - 1.0f) < kAngleEpsilon;
}
// sampleMaterial — KernelHelpers.h:56-114; returns (bsdf, pdf)
static void sampleMaterial(const Material& m, F3 wI, F3 wO, F3 n, const float* noise, float& bsdf, float& pdf) {
  float cosTheta = dot(wO, n);
  constexpr float invPi = 1.0f / kPi;
  switch (m.materialType) {
    case MAT_MIRROR: {
      bool mir = isMirrorDir(wI, n, wO);
      bsdf = mir ? cosTheta : 0.0f; pdf = 1.0f; break;
    }
    case MAT_PLASTIC: {
      float fI = fresnel(n, neg(wI), 1.0f, m.ior);
      if (fI < noise[1]) { bsdf = pdf = invPi * cosTheta; }
      else { bool mir = isMirrorDir(wI, n, wO); bsdf = mir ? cosTheta : 0.0f; pdf = 1.0f; }
      break;
    }
    case MAT_DIELECTRIC: {
      float fI = fresnel(n, neg(wI), 1.0f, m.ior);
      if (fI < noise[1]) { bsdf = pdf = 0.0f; }
      else { bool mir = isMirrorDir(wI, n, wO); bsdf = mir ? cosTheta : 0.0f; pdf = 1.0f; }
      break;
    }
    default: bsdf = pdf = invPi * cosTheta; break;
  }
}
// generateNextBounce — KernelHelpers.h:116-179
static F3 generateNextBounce(const Material& m, F3 wI, float currentIoR, F3 n, const float* noise,
                             float& bsdf, float& pdf, float& ior) {
  constexpr float invPi = 1.0f / kPi;
  F3 wO; float px, py;
  ior = currentIoR;
  switch (m.materialType) {
    case MAT_MIRROR: wO = reflect(wI, n); px = dot(wO, n); py = 1.0f; break;
    case MAT_PLASTIC: {
      float fI = fresnel(n, neg(wI), currentIoR, m.ior);
      if (fI < noise[1]) { wO = generateDiffuseBounce(noise[2], noise[3], n); px = py = invPi * dot(wO, n); }
      else { wO = reflect(wI, n); px = dot(wO, n); py = 1.0f; }
      break;
    }
    case MAT_DIELECTRIC: {
      float fI = fresnel(n, neg(wI), currentIoR, m.ior);
      if (fI < noise[1]) { ior = m.ior; wO = wI; px = py = 1.0f; }
      else { wO = reflect(wI, n); px = dot(wO, n); py = 1.0f; }
      break;
    }
    default: wO = generateDiffuseBounce(noise[2], noise[3], n); px = py = invPi * dot(wO, n); break;
  }
  bsdf = px; pdf = py;
  return wO;
}
// lightTriangleSamplePDF — KernelHelpers.h:181-190
static float lightTriangleSamplePDF(float pdf, float area, F3 source, const Vertex& smp, F3& dirOut) {
  F3 d = sub(f3(smp.v), source);
  float dist = length(d);
  dirOut = normalize(d);
  float LdotD = -dot(dirOut, f3(smp.n));
  float valid = float(dist >= kDistanceEpsilon) * float(LdotD >= kAngleEpsilon);
  return valid * pdf * triangleSamplePDF(area, LdotD, dist);
}

// ============================================================================
// Kernels (per pixel) — renderer/Shaders.metal
// ============================================================================
// rayGenerator — Shaders.metal:75-103
static void rayGenerator(Ray& ray, unsigned x, unsigned y, unsigned W, unsigned H, const float* noise) {
  float aspect = float(H) / float(W);
  const float* ns = noise + 4 * ((x % kNoiseDim) + (y % kNoiseDim) * kNoiseDim);
  float wm1 = float(W - 1), hm1 = float(H - 1);
  float dudvx = (ns[0] * 2.0f - 1.0f) / wm1;
  float dudvy = (ns[1] * 2.0f - 1.0f) / hm1;
  float ncx = float(2 * x) / wm1 - 1.0f;
  float ncy = float(2 * y) / hm1 - 1.0f;
  // side=(1,0,0), up=(0,1,0), view=(0,0,-1) at t=0
  F3 dir = {dudvx + ncx, dudvy + ncy * aspect, -1.0f};
  F3 d = normalize(dir);
  ray.origin[0] = 0.0f; ray.origin[1] = 1.0f; ray.origin[2] = 2.35f;   // up - view*2.35
  st3(ray.direction, d);
  ray.maxDistance = INFINITY;
  ray.params[0] = 1.0f; ray.params[1] = 0.0f; ray.params[2] = 0.0f; ray.params[3] = 1.00029f;
  for (int i = 0; i < 3; ++i) { ray.throughput[i] = 1.0f; ray.radiance[i] = 0.0f; }
}

// intersectionHandler — Shaders.metal:105-212
static void intersectionHandler(const Scene& sc, const Intersection& isect, Ray& ray, LightSamplingRay& sray,
                                unsigned x, unsigned y, uint32_t frameIndex, uint32_t maxPathLength,
                                const float* noiseTable, bool debugMaterial = false) {
  sray.maxDistance = -1.0f;                                                   // :119
  if (isect.distance < kDistanceEpsilon) { ray.maxDistance = -1.0f; return; } // :122-126
  const TriangleReference& ref = sc.references[isect.triangleIndex];          // :129
  const Material& material = sc.materials[ref.materialIndex];                 // :130
  uint32_t bounce = (uint32_t)ray.params[2];                                  // :132
  F3 wI = f3(ray.direction);
  uint32_t noiseIndex = ((x + bounce + frameIndex / 3) % kNoiseDim) +
                        ((y + bounce + frameIndex / 5) % kNoiseDim) * kNoiseDim;   // :135-136
  const float* noise = noiseTable + 4 * noiseIndex;                           // :138
  Vertex hit = interpolate2(sc.vertices[ref.tri[0]], sc.vertices[ref.tri[1]], sc.vertices[ref.tri[2]],
                            isect.coordinates);                               // :140
  F3 hv = f3(hit.v), hn = f3(hit.n);
  if (debugMaterial) {   // DEBUG_MATERIAL (Shaders.metal:7,142-147): radiance := Fresnel(n, -wI, 1, 1.5)
    const float f = fresnel(hn, neg(wI), 1.0f, 1.5f);
    for (int i = 0; i < 3; ++i) ray.radiance[i] = f;
  }
  const LightTriangle* lts = sc.lightTriangles.data();
  if (bounce + 1 < maxPathLength) {                                           // :150-176
    const LightTriangle& lt = selectLightTriangle(noise[2], lts, (int)sc.lightTrianglesCount);
    Vertex lightVertex = interpolate3(lt.v1, lt.v2, lt.v3, barycentric(noise[3], noise[0]));
    F3 dirToLight;
    float lightPdf = lightTriangleSamplePDF(lt.pdf, lt.area, hv, lightVertex, dirToLight);
    float materialBsdf, materialPdf;
    sampleMaterial(material, wI, dirToLight, hn, noise, materialBsdf, materialPdf);
    float weight = balanceHeuristic(lightPdf, materialPdf);
    bool valid = (lightPdf > 0.0f) && (lt.index != isect.triangleIndex);
    float s = weight * materialBsdf / lightPdf;
    float e[3];
    for (int i = 0; i < 3; ++i) e[i] = ((lt.emissive[i] * material.diffuse[i]) * ray.throughput[i]) * s;
    st3(sray.origin, add(hv, mul(hn, kDistanceEpsilon)));
    st3(sray.direction, dirToLight);
    sray.maxDistance = valid ? INFINITY : -1.0f;
    sray.targetIndex = lt.index;
    for (int i = 0; i < 3; ++i) sray.throughput[i] = e[i];
  }
  if (ref.lightTriangleIndex != 0xFFFFFFFFu) {                                // :180-197
    const LightTriangle& lt = lts[ref.lightTriangleIndex];
    const TriangleReference& ref2 = sc.references[lt.index];
    Vertex lightVertex = interpolate2(sc.vertices[ref2.tri[0]], sc.vertices[ref2.tri[1]],
                                      sc.vertices[ref2.tri[2]], isect.coordinates);
    F3 dirToLight;
    float mPdf = ray.params[0];
    float lPdf = ray.params[1] * lightTriangleSamplePDF(lt.pdf, lt.area, f3(ray.origin), lightVertex, dirToLight);
    float weight = balanceHeuristic(mPdf, lPdf);
    float s = weight * mPdf;
    for (int i = 0; i < 3; ++i) ray.radiance[i] += (material.emissive[i] * ray.throughput[i]) * s;
  }
  {                                                                           // :199-211
    float bsdf = 0, pdf = 0, ior = 0;
    F3 wO = generateNextBounce(material, wI, ray.params[3], hn, noise, bsdf, pdf, ior);
    st3(ray.direction, wO);
    st3(ray.origin, add(hv, mul(hn, kDistanceEpsilon)));
    ray.maxDistance = INFINITY;
    ray.params[0] = pdf;
    ray.params[1] = float(material.materialType == MAT_DIFFUSE);
    ray.params[2] = float(bounce + 1);
    ray.params[3] = ior;
    float sc2 = bsdf / pdf;
    for (int i = 0; i < 3; ++i) ray.throughput[i] *= material.diffuse[i] * sc2;
  }
}

// lightSamplingHandler — Shaders.metal:214-231
static void lightSamplingHandler(const Intersection& isect, Ray& ray, const LightSamplingRay& sray) {
  if ((isect.distance >= kDistanceEpsilon) && (isect.triangleIndex == sray.targetIndex))
    for (int i = 0; i < 3; ++i) ray.radiance[i] += sray.throughput[i];
}

// accumulateImage — Shaders.metal:233-249 (accumulate = ACCUMULATE_IMAGE,
// Raytracing.h:14: false writes the frame's radiance alone)
static void accumulateImage(const Ray& ray, float* px, uint32_t frameIndex, bool accumulate = true) {
  float c[3] = {ray.radiance[0], ray.radiance[1], ray.radiance[2]};
  if (accumulate && frameIndex > 0) {
    float factor = float(frameIndex) / float(frameIndex + 1);
    for (int i = 0; i < 3; ++i) c[i] = mixf(c[i], px[i], factor);
  }
  px[0] = c[0]; px[1] = c[1]; px[2] = c[2]; px[3] = 1.0f;
}

// Noise schedule — SURVEY.md Appendix A.3: iteration i of frame f reads
// slot (f+i)%3 (renderer/Renderer.mm:538) which holds T_f, T_{f-2}, T_{f-1}.
static int64_t noise_frame_for(int64_t f, unsigned i) {
  switch (i % 3) {
    case 0: return f;
    case 1: return f >= 2 ? f - 2 : -1;
    default: return f >= 1 ? f - 1 : -1;
  }
}

struct NoiseCache {
  uint64_t seed;
  std::vector<std::vector<float>> tables;   // index frame+1 (0 = initial table)
  bool animate = true;                      // ANIMATE_NOISE (Raytracing.h:20); 0: the initial table for every frame
  const float* get(int64_t frame) {
    if (!animate) frame = -1;   // Renderer.mm:485-497 skipped: the slots keep the table of :109-129
    size_t k = (size_t)(frame + 1);
    if (k >= tables.size()) tables.resize(k + 1);
    if (tables[k].empty()) { tables[k].resize(kNoiseDim * kNoiseDim * 4); noise_table(seed, frame, tables[k].data()); }
    return tables[k].data();
  }
};

}  // namespace

// ============================================================================
// C ABI for ctypes (tests / bench cpu_baseline only)
// ============================================================================
extern "C" {

struct orc_scene { Scene s; };

// Scenes with at least this many triangles are rendered by orc_render in row
// packets (intersect_packet); tests lower it to check both forms agree.
static size_t g_packet_threshold = 4096;
void orc_set_packet_threshold(uint64_t triangles) { g_packet_threshold = (size_t)triangles; }

int orc_scene_load(const char* obj_path, const char* mtl_override, orc_scene** out) {
  auto* sc = new orc_scene();
  if (!load_scene(obj_path, mtl_override, sc->s)) {
    std::fprintf(stderr, "orc_scene_load: %s\n", sc->s.error.c_str());
    delete sc; *out = nullptr; return -1;
  }
  *out = sc; return 0;
}

// Build a scene from raw buffers (for procedural scenes generated by tests).
int orc_scene_from_arrays(const float* verts24, uint32_t nverts, const uint32_t* tri_refs20, uint32_t ntris,
                          const float* mats32, uint32_t nmats, orc_scene** out) {
  auto* sc = new orc_scene();
  Scene& s = sc->s;
  s.vertices.resize(nverts); std::memcpy(s.vertices.data(), verts24, nverts * sizeof(Vertex));
  s.materials.resize(nmats); std::memcpy(s.materials.data(), mats32, nmats * sizeof(Material));
  s.references.resize(ntris); std::memcpy(s.references.data(), tri_refs20, ntris * sizeof(TriangleReference));
  float totalArea = 0.0f;
  for (uint32_t k = 0; k < ntris; ++k) {
    TriangleReference& r = s.references[k];
    s.indices.push_back(r.tri[0]); s.indices.push_back(r.tri[1]); s.indices.push_back(r.tri[2]);
    const Material& mat = s.materials[r.materialIndex];
    bool isEmitter = (mat.emissive[0] > 0.0f) || (mat.emissive[1] > 0.0f) || (mat.emissive[2] > 0.0f);
    r.lightTriangleIndex = 0xFFFFFFFFu;
    if (isEmitter) {
      const Vertex &v1 = s.vertices[r.tri[0]], &v2 = s.vertices[r.tri[1]], &v3 = s.vertices[r.tri[2]];
      LightTriangle lt{};
      lt.index = k; lt.v1 = v1; lt.v2 = v2; lt.v3 = v3;
      lt.area = 0.5f * length(cross(sub(f3(v2.v), f3(v1.v)), sub(f3(v3.v), f3(v1.v))));
      for (int i = 0; i < 3; ++i) lt.emissive[i] = mat.emissive[i];
      totalArea += lt.area;
      r.lightTriangleIndex = (uint32_t)s.lightTriangles.size();
      s.lightTriangles.push_back(lt);
    }
  }
  float cdf = 0.0f;
  for (LightTriangle& lt : s.lightTriangles) { lt.pdf = lt.area / totalArea; lt.cdf = cdf; cdf += lt.pdf; }
  s.lightTrianglesCount = (uint32_t)s.lightTriangles.size();
  LightTriangle sentinel{}; sentinel.cdf = cdf; sentinel.pdf = 1.0f; sentinel.area = 0.0f;
  s.lightTriangles.push_back(sentinel);
  *out = sc; return 0;
}

void orc_scene_free(orc_scene* sc) { delete sc; }

// counts[5] = {vertices, triangles, materials, light triangles (no sentinel), light entries (with sentinel)}
void orc_scene_counts(const orc_scene* sc, uint32_t* counts) {
  counts[0] = (uint32_t)sc->s.vertices.size();
  counts[1] = (uint32_t)sc->s.references.size();
  counts[2] = (uint32_t)sc->s.materials.size();
  counts[3] = sc->s.lightTrianglesCount;
  counts[4] = (uint32_t)sc->s.lightTriangles.size();
}
const void* orc_scene_vertices(const orc_scene* sc) { return sc->s.vertices.data(); }
const void* orc_scene_indices(const orc_scene* sc) { return sc->s.indices.data(); }
const void* orc_scene_materials(const orc_scene* sc) { return sc->s.materials.data(); }
const void* orc_scene_references(const orc_scene* sc) { return sc->s.references.data(); }
const void* orc_scene_lights(const orc_scene* sc) { return sc->s.lightTriangles.data(); }

void orc_noise_table(uint64_t seed, int64_t frame, float* out16384) { noise_table(seed, frame, out16384); }
int64_t orc_noise_frame_for(int64_t frame, uint32_t iteration) { return noise_frame_for(frame, iteration); }

// ---- stage-level entry points over reference AoS buffers (host memory) ------
void orc_raygen(uint32_t W, uint32_t H, const float* noise, void* rays) {
  Ray* r = (Ray*)rays;
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) rayGenerator(r[y * W + x], x, y, W, H, noise);
}

// rays: records of `stride` bytes whose first 32 bytes are origin,min,dir,max
void orc_intersect(const orc_scene* sc, const void* rays, uint32_t stride, uint32_t count, void* isect_out) {
  const uint8_t* p = (const uint8_t*)rays;
  Intersection* out = (Intersection*)isect_out;
  if (sc->s.references.size() >= g_packet_threshold) {   // large scene: packets of 256 rays
    std::vector<const float*> op(256), dp(256);
    std::vector<float> tmn(256), tmx(256);
    for (uint32_t i0 = 0; i0 < count; i0 += 256) {
      const uint32_t n = std::min<uint32_t>(256, count - i0);
      for (uint32_t j = 0; j < n; ++j) {
        const float* f = (const float*)(p + (size_t)(i0 + j) * stride);
        op[j] = f; tmn[j] = f[3]; dp[j] = f + 4; tmx[j] = f[7];
      }
      intersect_packet(sc->s, op.data(), tmn.data(), dp.data(), tmx.data(), n, out + i0);
    }
    return;
  }
  for (uint32_t i = 0; i < count; ++i) {
    const float* f = (const float*)(p + (size_t)i * stride);
    out[i] = intersect_one(sc->s, f, f[3], f + 4, f[7]);
  }
}

// flags: ORC_DEBUG_MATERIAL (see orc_render)
void orc_shade(const orc_scene* sc, uint32_t W, uint32_t H, uint32_t frameIndex, uint32_t maxPathLength,
               const float* noise, const void* isect, void* rays, void* srays, uint32_t flags) {
  const Intersection* is = (const Intersection*)isect;
  Ray* r = (Ray*)rays; LightSamplingRay* s = (LightSamplingRay*)srays;
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) {
      uint32_t i = y * W + x;
      intersectionHandler(sc->s, is[i], r[i], s[i], x, y, frameIndex, maxPathLength, noise, (flags & 4u) != 0);
    }
}

void orc_resolve(uint32_t count, const void* isect, void* rays, const void* srays) {
  const Intersection* is = (const Intersection*)isect;
  Ray* r = (Ray*)rays; const LightSamplingRay* s = (const LightSamplingRay*)srays;
  for (uint32_t i = 0; i < count; ++i) lightSamplingHandler(is[i], r[i], s[i]);
}

// flags: ORC_NO_ACCUMULATE (see orc_render)
void orc_accumulate(uint32_t count, uint32_t frameIndex, const void* rays, float* image_rgba, uint32_t flags) {
  const Ray* r = (const Ray*)rays;
  for (uint32_t i = 0; i < count; ++i) accumulateImage(r[i], image_rgba + 4 * (size_t)i, frameIndex, !(flags & 2u));
}

// intersect through the CPU baseline's BVH (same answers as orc_intersect)
void orc_intersect_bvh(const orc_scene* sc, const void* rays, uint32_t stride, uint32_t count, void* isect_out) {
  const uint8_t* p = (const uint8_t*)rays;
  Intersection* out = (Intersection*)isect_out;
  for (uint32_t i = 0; i < count; ++i) {
    const float* f = (const float*)(p + (size_t)i * stride);
    out[i] = intersect_bvh(sc->s, f, f[3], f + 4, f[7]);
  }
}

// the same on `threads` threads with an explicit culling rule (0 = kCullWide,
// 1 = kCullNone; see intersect_bvh)
void orc_intersect_bvh_mt(const orc_scene* sc, const void* rays, uint32_t stride, uint32_t count, void* isect_out,
                          uint32_t threads, uint32_t cull) {
  const uint8_t* p = (const uint8_t*)rays;
  Intersection* out = (Intersection*)isect_out;
  std::call_once(sc->s.bvh_once, build_cpu_bvh, std::cref(sc->s));
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (uint32_t i0 = next.fetch_add(1024); i0 < count; i0 = next.fetch_add(1024))
      for (uint32_t i = i0; i < std::min(count, i0 + 1024u); ++i) {
        const float* f = (const float*)(p + (size_t)i * stride);
        out[i] = intersect_bvh(sc->s, f, f[3], f + 4, f[7], cull ? kCullNone : kCullWide);
      }
  };
  if (threads <= 1) { work(); return; }
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < threads; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
}

// ---- whole-frame driver: performRaytracing: (renderer/Renderer.mm:500-585) --
// Renders frames [frame_begin, frame_end) into image_rgba (W*H*4, row 0 =
// bottom), accumulating as accumulateImage does.  Rows are handed out one at
// a time to `threads` std::threads (pixels are independent within a frame;
// a shared row counter keeps masked bands and uneven rows balanced).
// active_out (optional) receives A = sum over iterations of rays alive at
// the start of the iteration.  pixel_mask (optional, W*H bytes) restricts the
// render to pixels with mask != 0 (others untouched) for bounded samples.
// flags: the reference's compile-time switches (renderer/Raytracing.h:11-33,
// renderer/Shaders.metal:7) and the traversal used —
//   1 ORC_STATIC_NOISE     ANIMATE_NOISE 0: every frame reads the initial table
//   2 ORC_NO_ACCUMULATE    ACCUMULATE_IMAGE false: the image is the last frame
//   4 ORC_DEBUG_MATERIAL   DEBUG_MATERIAL 1: radiance := Fresnel at each hit
//   8 ORC_BVH              nearest hits through the CPU BVH (the cpu_baseline
//                          leg) instead of brute force — the same answers;
//                          boxes culled beyond bt * (1 + 2^-6) (kCullWide)
//  16 ORC_BVH_NOCULL       with ORC_BVH: no culling by the current hit (kCullNone)
int orc_render(const orc_scene* sc, uint32_t W, uint32_t H, uint32_t maxPathLength, uint64_t seed,
               uint32_t frame_begin, uint32_t frame_end, uint32_t threads, const uint8_t* pixel_mask,
               float* image_rgba, uint64_t* active_out, uint32_t flags) {
  if (W < 2 || H < 2 || maxPathLength == 0) return -1;
  const bool use_bvh = (flags & 8u) != 0;
  const int cull = (flags & 16u) ? kCullNone : kCullWide;
  const bool use_packets = !use_bvh && sc->s.references.size() >= g_packet_threshold;
  const bool debug_material = (flags & 4u) != 0, accumulate = (flags & 2u) == 0;
  if (use_bvh) std::call_once(sc->s.bvh_once, build_cpu_bvh, std::cref(sc->s));
  NoiseCache nc{seed, {}};
  nc.animate = (flags & 1u) == 0;
  std::atomic<uint64_t> active{0};
  if (threads == 0) threads = 1;
  for (uint32_t f = frame_begin; f < frame_end; ++f) {
    const float* raygenNoise = nc.get(f);
    std::vector<const float*> iterNoise(maxPathLength);
    for (uint32_t i = 0; i < maxPathLength; ++i) iterNoise[i] = nc.get(noise_frame_for(f, i));
    std::atomic<uint32_t> next_row{0};
    // large scenes: each row is one packet through the stages (the per-pixel
    // operations and their order are the same; only pixels interleave)
    auto work_packets = [&]() {
      uint64_t local = 0;
      std::vector<Ray> rays;
      std::vector<LightSamplingRay> srays;
      std::vector<uint32_t> xs;
      std::vector<Intersection> is;
      std::vector<const float*> op, dp;
      std::vector<float> tmn, tmx;
      auto trace = [&](bool shadow) {
        const size_t n = xs.size();
        for (size_t j = 0; j < n; ++j) {
          if (shadow) { op[j] = srays[j].origin; dp[j] = srays[j].direction; tmn[j] = srays[j].minDistance; tmx[j] = srays[j].maxDistance; }
          else { op[j] = rays[j].origin; dp[j] = rays[j].direction; tmn[j] = rays[j].minDistance; tmx[j] = rays[j].maxDistance; }
        }
        intersect_packet(sc->s, op.data(), tmn.data(), dp.data(), tmx.data(), n, is.data());
      };
      for (uint32_t y = next_row++; y < H; y = next_row++) {
        xs.clear();
        for (uint32_t x = 0; x < W; ++x)
          if (!pixel_mask || pixel_mask[(size_t)y * W + x]) xs.push_back(x);
        const size_t n = xs.size();
        if (!n) continue;
        rays.assign(n, Ray{}); srays.assign(n, LightSamplingRay{}); is.resize(n);
        op.resize(n); dp.resize(n); tmn.resize(n); tmx.resize(n);
        for (size_t j = 0; j < n; ++j) rayGenerator(rays[j], xs[j], y, W, H, raygenNoise);
        for (uint32_t i = 0; i < maxPathLength; ++i) {
          for (size_t j = 0; j < n; ++j) local += rays[j].maxDistance >= 0.0f;
          trace(false);
          for (size_t j = 0; j < n; ++j)
            intersectionHandler(sc->s, is[j], rays[j], srays[j], xs[j], y, f, maxPathLength, iterNoise[i], debug_material);
          trace(true);
          for (size_t j = 0; j < n; ++j) lightSamplingHandler(is[j], rays[j], srays[j]);
        }
        for (size_t j = 0; j < n; ++j) accumulateImage(rays[j], image_rgba + 4 * ((size_t)y * W + xs[j]), f, accumulate);
      }
      active += local;
    };
    auto work = [&]() {
      if (use_packets) { work_packets(); return; }
      uint64_t local = 0;
      for (uint32_t y = next_row++; y < H; y = next_row++)
        for (uint32_t x = 0; x < W; ++x) {
          size_t pix = (size_t)y * W + x;
          if (pixel_mask && !pixel_mask[pix]) continue;
          Ray ray{}; LightSamplingRay sray{};
          rayGenerator(ray, x, y, W, H, raygenNoise);
          for (uint32_t i = 0; i < maxPathLength; ++i) {
            if (ray.maxDistance >= 0.0f) ++local;
            auto isect = [&](const float* o, float t0, const float* d, float t1) {
              return use_bvh ? intersect_bvh(sc->s, o, t0, d, t1, cull) : intersect_one(sc->s, o, t0, d, t1);
            };
            Intersection is = isect(ray.origin, ray.minDistance, ray.direction, ray.maxDistance);
            intersectionHandler(sc->s, is, ray, sray, x, y, f, maxPathLength, iterNoise[i], debug_material);
            Intersection is2 = isect(sray.origin, sray.minDistance, sray.direction, sray.maxDistance);
            lightSamplingHandler(is2, ray, sray);
          }
          accumulateImage(ray, image_rgba + 4 * pix, f, accumulate);
        }
      active += local;
    };
    if (threads == 1) work();
    else {
      std::vector<std::thread> th;
      for (uint32_t t = 0; t < threads; ++t) th.emplace_back(work);
      for (auto& t : th) t.join();
    }
  }
  if (active_out) *active_out = active.load();
  return 0;
}

}  // extern "C"
