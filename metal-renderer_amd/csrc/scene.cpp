// scene.cpp — OBJ/MTL import + flattening.  See scene.h.
#include "scene.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <unordered_map>

namespace mrt {
namespace {

struct Color { float c[3] = {0.0f, 0.0f, 0.0f}; };
struct MtlDef { Color kd, ka, ks; };

// Tokenizer over one line: whitespace = space, tab, CR.
struct Line {
  const char* p;
  const char* end;
  explicit Line(const std::string& s) : p(s.data()), end(s.data() + s.size()) {}
  bool next(std::string& tok) {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p;
    if (p >= end) return false;
    const char* b = p;
    while (p < end && !(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p;
    tok.assign(b, p - b);
    return true;
  }
};

bool read_mtl(const std::string& path, std::unordered_map<std::string, MtlDef>& out, std::string& err) {
  std::ifstream f(path);
  if (!f) { err = "cannot open material library " + path; return false; }
  std::string line, tok, current;
  while (std::getline(f, line)) {
    Line L(line);
    if (!L.next(tok) || tok[0] == '#') continue;
    if (tok == "newmtl") { L.next(current); out[current]; continue; }
    if (current.empty()) continue;
    Color* dst = nullptr;
    if (tok == "Kd") dst = &out[current].kd;
    else if (tok == "Ka") dst = &out[current].ka;    // SceneKit: Ka -> emission
    else if (tok == "Ks") dst = &out[current].ks;
    if (!dst) continue;                               // Kx, illum, Ns, ... ignored
    for (int i = 0; i < 3; ++i) {
      std::string v;
      if (!L.next(v)) break;
      dst->c[i] = std::strtof(v.c_str(), nullptr);
    }
  }
  return true;
}

inline void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

}  // namespace

RefMaterial classify_material(const float kd[3], const float ka[3], const float ks[3]) {
  RefMaterial m{};
  for (int i = 0; i < 3; ++i) { m.diffuse[i] = kd[i]; m.emissive[i] = ka[i]; }
  m.ior = ks[2];
  const float roughness = ks[0], metallness = ks[1];
  m.materialType = kDiffuse;                      // rough conductor stays value-initialised
  if (metallness > 0.0f) {
    if (roughness == 0.0f) m.materialType = kMirror;
  } else if (roughness == 1.0f) {
    m.materialType = kDiffuse;
  } else if (m.ior <= 0.0f) {
    m.ior = std::fabs(m.ior);
    m.materialType = (roughness == 0.0f) ? kPlastic : kDiffuse;
  } else {
    m.materialType = (roughness == 0.0f) ? kDielectric : kDiffuse;
  }
  return m;
}

bool import_obj(const std::string& obj_path, const std::string& mtl_override, HostScene& scene,
                std::string& error) {
  std::ifstream f(obj_path);
  if (!f) { error = "cannot open scene " + obj_path; return false; }
  const size_t slash = obj_path.find_last_of('/');
  const std::string dir = slash == std::string::npos ? std::string() : obj_path.substr(0, slash + 1);

  std::unordered_map<std::string, MtlDef> mtl;
  bool have_mtl = false;
  if (!mtl_override.empty()) {
    if (!read_mtl(mtl_override, mtl, error)) return false;
    have_mtl = true;
  }
  std::vector<float> pos, nrm;                 // 3 floats each
  std::vector<std::string> element_mtl;
  std::vector<std::vector<uint32_t>> element_idx;
  std::unordered_map<uint64_t, uint32_t> corner_to_vertex;   // (v, vn) -> vertex id
  std::string line, tok;
  std::vector<uint32_t> corners;
  while (std::getline(f, line)) {
    Line L(line);
    if (!L.next(tok) || tok[0] == '#') continue;
    if (tok == "v" || tok == "vn") {
      std::vector<float>& dst = (tok == "v") ? pos : nrm;
      for (int i = 0; i < 3; ++i) {
        std::string v;
        L.next(v);
        dst.push_back(std::strtof(v.c_str(), nullptr));
      }
    } else if (tok == "mtllib") {
      std::string name;
      L.next(name);
      if (!have_mtl) {
        if (!read_mtl(dir + name, mtl, error)) return false;
        have_mtl = true;
      }
    } else if (tok == "usemtl") {
      std::string name;
      L.next(name);
      element_mtl.push_back(name);
      element_idx.emplace_back();
    } else if (tok == "f") {
      if (element_idx.empty()) { element_mtl.emplace_back(); element_idx.emplace_back(); }
      corners.clear();
      std::string c;
      while (L.next(c)) {
        long vi = std::strtol(c.c_str(), nullptr, 10), ni = 0;
        const char* s1 = std::strchr(c.c_str(), '/');
        if (s1) {
          const char* s2 = std::strchr(s1 + 1, '/');
          if (s2) ni = std::strtol(s2 + 1, nullptr, 10);
        }
        if (vi < 0) vi += (long)(pos.size() / 3) + 1;
        if (ni < 0) ni += (long)(nrm.size() / 3) + 1;
        if (vi <= 0 || (size_t)vi > pos.size() / 3 || ni < 0 || (size_t)ni > nrm.size() / 3) {
          error = "bad face index in " + obj_path;
          return false;
        }
        const uint64_t key = ((uint64_t)vi << 32) | (uint64_t)ni;
        auto it = corner_to_vertex.find(key);
        uint32_t id;
        if (it == corner_to_vertex.end()) {
          RefVertex v{};
          for (int k = 0; k < 3; ++k) v.v[k] = pos[3 * (vi - 1) + k];
          if (ni > 0) for (int k = 0; k < 3; ++k) v.n[k] = nrm[3 * (ni - 1) + k];
          id = (uint32_t)scene.vertices.size();
          scene.vertices.push_back(v);
          corner_to_vertex.emplace(key, id);
        } else {
          id = it->second;
        }
        corners.push_back(id);
      }
      std::vector<uint32_t>& idx = element_idx.back();
      for (size_t k = 1; k + 1 < corners.size(); ++k) {
        idx.push_back(corners[0]);
        idx.push_back(corners[k]);
        idx.push_back(corners[k + 1]);
      }
    }
  }
  // one element (+ one SCNMaterial) per non-empty usemtl group, file order
  for (size_t e = 0; e < element_idx.size(); ++e) {
    if (element_idx[e].empty()) continue;
    MtlDef def{};
    auto it = mtl.find(element_mtl[e]);
    if (it != mtl.end()) def = it->second;
    SceneElement el;
    el.material = (uint32_t)scene.materials.size();
    el.indices = std::move(element_idx[e]);
    scene.materials.push_back(classify_material(def.kd.c, def.ka.c, def.ks.c));
    scene.elements.push_back(std::move(el));
  }
  if (scene.elements.empty()) { error = "scene has no triangles: " + obj_path; return false; }
  return true;
}

void append_procedural_mesh(HostScene& scene, uint32_t triangles, uint64_t seed) {
  // Lat-long grid of rings x segs quads (2 triangles each) on a sphere with a
  // seeded sum-of-sines radial displacement.  rings * segs * 2 == triangles
  // when triangles = 2 * r * 2r (e.g. 1,048,576 = 2 * 512 * 1024).
  uint32_t quads = triangles / 2;
  uint32_t rings = 1;
  while ((uint64_t)(rings * 2) * (rings * 2) * 2 <= quads) rings *= 2;
  rings = std::max<uint32_t>(rings, 2);
  uint32_t segs = std::max<uint32_t>(quads / rings, 3);
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  float amp[6], fu[6], fv[6], ph[6];
  for (int k = 0; k < 6; ++k) {
    amp[k] = 0.012f + 0.02f * U(rng);
    fu[k] = (float)(2 + (int)(U(rng) * 14.0f));
    fv[k] = (float)(2 + (int)(U(rng) * 14.0f));
    ph[k] = 6.2831853f * U(rng);
  }
  const float cx = 0.0f, cy = 0.9f, cz = 0.0f, R = 0.55f;
  auto radius = [&](float th, float phi) {
    float r = R;
    for (int k = 0; k < 6; ++k) r += amp[k] * std::sin(fu[k] * phi + ph[k]) * std::sin(fv[k] * th);
    return r;
  };
  auto point = [&](uint32_t i, uint32_t j, float out[3]) {
    const float th = 3.14159265f * (float)i / (float)rings;
    const float phi = 6.2831853f * (float)(j % segs) / (float)segs;
    const float r = radius(th, phi);
    out[0] = cx + r * std::sin(th) * std::cos(phi);
    out[1] = cy + r * std::cos(th);
    out[2] = cz + r * std::sin(th) * std::sin(phi);
  };
  const uint32_t base = (uint32_t)scene.vertices.size();
  // vertices (rings+1) x segs, normals from central differences
  for (uint32_t i = 0; i <= rings; ++i)
    for (uint32_t j = 0; j < segs; ++j) {
      RefVertex v{};
      point(i, j, v.v);
      float a[3], b[3], c[3], d[3];
      point(i == 0 ? 0 : i - 1, j, a);
      point(i == rings ? rings : i + 1, j, b);
      point(i, j + segs - 1, c);
      point(i, j + 1, d);
      float du[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
      float dv[3] = {d[0] - c[0], d[1] - c[1], d[2] - c[2]};
      float n[3];
      cross3(du, dv, n);
      float l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      if (!(l > 0.0f)) {  // poles: radial direction
        n[0] = v.v[0] - cx; n[1] = v.v[1] - cy; n[2] = v.v[2] - cz;
        l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      }
      // orient outward
      const float out = n[0] * (v.v[0] - cx) + n[1] * (v.v[1] - cy) + n[2] * (v.v[2] - cz);
      const float s = (out < 0.0f ? -1.0f : 1.0f) / l;
      for (int k = 0; k < 3; ++k) v.n[k] = n[k] * s;
      scene.vertices.push_back(v);
    }
  SceneElement el;
  el.material = (uint32_t)scene.materials.size();
  const float kd[3] = {0.8f, 0.8f, 0.8f}, ka[3] = {0.0f, 0.0f, 0.0f}, ks[3] = {1.0f, 0.0f, 0.0f};
  scene.materials.push_back(classify_material(kd, ka, ks));
  el.indices.reserve((size_t)rings * segs * 6);
  for (uint32_t i = 0; i < rings; ++i)
    for (uint32_t j = 0; j < segs; ++j) {
      const uint32_t a = base + i * segs + j, b = base + i * segs + (j + 1) % segs;
      const uint32_t c = base + (i + 1) * segs + j, d = base + (i + 1) * segs + (j + 1) % segs;
      el.indices.insert(el.indices.end(), {a, c, b, b, c, d});
    }
  scene.elements.push_back(std::move(el));
}

void flatten(HostScene& scene) {
  scene.indices.clear();
  scene.references.clear();
  scene.lights.clear();
  float total_area = 0.0f;
  const size_t M = scene.materials.size();
  size_t element_index = 0;
  for (const SceneElement& el : scene.elements) {
    // renderer/Renderer.mm:377 — material = elementIndex % materialCount
    const uint32_t mi = (uint32_t)(element_index % M);
    const RefMaterial& mat = scene.materials[mi];
    const bool emitter = mat.emissive[0] > 0.0f || mat.emissive[1] > 0.0f || mat.emissive[2] > 0.0f;
    for (size_t i = 0; i + 2 < el.indices.size(); i += 3) {
      uint32_t light_index = 0xFFFFFFFFu;
      if (emitter) {   // renderer/Renderer.mm:394-413
        const RefVertex& a = scene.vertices[el.indices[i]];
        const RefVertex& b = scene.vertices[el.indices[i + 1]];
        const RefVertex& c = scene.vertices[el.indices[i + 2]];
        RefLightTriangle lt{};
        lt.index = (uint32_t)scene.references.size();
        lt.v1 = a; lt.v2 = b; lt.v3 = c;
        float e1[3], e2[3], x[3];
        for (int k = 0; k < 3; ++k) { e1[k] = b.v[k] - a.v[k]; e2[k] = c.v[k] - a.v[k]; }
        cross3(e1, e2, x);
        lt.area = 0.5f * std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
        for (int k = 0; k < 3; ++k) lt.emissive[k] = mat.emissive[k];
        total_area += lt.area;
        light_index = (uint32_t)scene.lights.size();
        scene.lights.push_back(lt);
      }
      RefTriangleReference r{};
      r.tri[0] = el.indices[i]; r.tri[1] = el.indices[i + 1]; r.tri[2] = el.indices[i + 2];
      r.materialIndex = mi;
      r.lightTriangleIndex = light_index;
      scene.references.push_back(r);
      scene.indices.insert(scene.indices.end(), {r.tri[0], r.tri[1], r.tri[2]});
    }
    ++element_index;
  }
  // renderer/Renderer.mm:435-448 — pdf, exclusive-prefix cdf, sentinel
  float cdf = 0.0f;
  for (RefLightTriangle& lt : scene.lights) {
    lt.pdf = lt.area / total_area;
    lt.cdf = cdf;
    cdf += lt.pdf;
  }
  scene.light_count = (uint32_t)scene.lights.size();
  RefLightTriangle sentinel{};
  sentinel.cdf = cdf;
  sentinel.pdf = 1.0f;
  sentinel.area = 0.0f;
  scene.lights.push_back(sentinel);
}

}  // namespace mrt
