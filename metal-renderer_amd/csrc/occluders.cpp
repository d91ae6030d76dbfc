// occluders.cpp — supporting planes whose triangles cannot occlude a shadow
// ray from an origin on the lights' side of them (occluders.h).
//
// Float-error margin.  Let T be a culled triangle, P its plane, and let the
// shadow origin p and every light vertex (hence the light point q, a convex
// combination) lie inside P by at least d.  The segment [p, q] does not meet
// P; the leaf test (kernels.hip tri_bary) could still report t in [0, t_q]
// only through rounding.  Its t = (s . (e1 x e2)) / (d . (e2 x e1)) with
// s = p - v0: the numerator is off by about 5u |s||e1||e2| (u = 2^-24) against
// a true value d_p * |e1 x e2|, the denominator by 5u |e1||e2| against
// |n.d| |e1 x e2|.  With c = |e1||e2| / |e1 x e2| (1 / sin of T's angle at v0),
// S >= |s|, t_q and the scene diagonal, a margin d >= 128 u c S keeps the
// numerator's sign and keeps a crossing beyond q (relative distance
// d_q / d_p from q) beyond the true t_q for every direction; a grazing
// direction gives |t| > 6 S > t_q.  Triangles with c > 16 (slivers) are kept.
//
// The light's own t_q (the target test, kernels.hip tri_test) is computed
// too: by the same analysis its error is about 10 u S c_L / |cos_L| (c_L the
// light triangle's c, cos_L the ray's cosine to the light's plane), which
// grows without bound for rays grazing the light plane (the reference only
// asks cos_L >= ANGLE_EPSILON, 3.8e-5).  A computed t_q above the true one
// could then reach a culled crossing.  The distance from q to a culled plane
// along the ray is at least D_L (the light vertices' least distance inside the
// culled planes), so the crossing stays beyond the computed t_q whenever the
// culled triangles' error (covered by margin, D_L >= 4 margin is required)
// plus the light's error stays below D_L: the kernels use the occluder tree
// only for shadow rays with cos_L >= cos_min = 20 u S c_L / D_L (light error
// <= D_L / 2), taken against the interpolated light normal the kernels
// already compute, so cos_min also adds twice the largest deviation of a
// light vertex normal from its triangle's geometric normal (ANGLE below).
// Rays under cos_min (a negligible share) traverse the main tree.
#include "occluders.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <utility>

namespace mrt {

namespace {

struct D3 { double x, y, z; };
D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double len(D3 a) { return std::sqrt(dot(a, a)); }

struct Plane {
  D3 n;            // unit normal, pointing out of the scene
  double w;        // n . x = w on the plane
  std::vector<uint32_t> tris;
  double c_max = 0.0;
  double dev = 0.0;   // largest gap between a member's own plane and this one over the scene box
};

constexpr uint32_t kMaxClassifiedTriangles = 16384;
constexpr double kSliver = 16.0;
constexpr size_t kMinCulledFraction = 8;   // cull at least 1/8 of the triangles
constexpr double kUnit = 5.9604644775390625e-08;   // 2^-24

}  // namespace

bool find_occluders(const float* positions, size_t stride_bytes, uint32_t num_vertices, const uint32_t* indices,
                    uint32_t num_triangles, const float* light_vertices, const float* light_normals,
                    uint32_t num_lights, OccluderSet& out) {
  out = OccluderSet{};
  if (num_triangles == 0 || num_triangles > kMaxClassifiedTriangles || num_vertices == 0) return false;
  const size_t stride = stride_bytes / sizeof(float);
  auto V = [&](uint32_t i) {
    const float* p = positions + stride * i;
    return D3{p[0], p[1], p[2]};
  };
  // scene box and scale S (bounds |s| = |p - v0|, t_q and the diagonal)
  D3 lo = V(0), hi = V(0);
  double amax = 0.0;
  for (uint32_t i = 0; i < num_vertices; ++i) {
    const D3 v = V(i);
    lo = {std::min(lo.x, v.x), std::min(lo.y, v.y), std::min(lo.z, v.z)};
    hi = {std::max(hi.x, v.x), std::max(hi.y, v.y), std::max(hi.z, v.z)};
    amax = std::max({amax, std::fabs(v.x), std::fabs(v.y), std::fabs(v.z)});
  }
  const double S = std::max(len(sub(hi, lo)), 2.0 * amax);
  if (!(S > 0.0)) return false;
  const double tol = 4.0 * kUnit * S;   // a vertex this close to a plane is on it
  const D3 corners[8] = {{lo.x, lo.y, lo.z}, {hi.x, lo.y, lo.z}, {lo.x, hi.y, lo.z}, {hi.x, hi.y, lo.z},
                         {lo.x, lo.y, hi.z}, {hi.x, lo.y, hi.z}, {lo.x, hi.y, hi.z}, {hi.x, hi.y, hi.z}};

  std::vector<Plane> planes;
  for (uint32_t t = 0; t < num_triangles; ++t) {
    const D3 v0 = V(indices[3 * t]), v1 = V(indices[3 * t + 1]), v2 = V(indices[3 * t + 2]);
    const D3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const D3 nr = cross(e1, e2);
    const double area2 = len(nr);
    if (!(area2 > 1e-12 * S * S)) continue;
    const double c = len(e1) * len(e2) / area2;
    if (c > kSliver) continue;
    D3 n = {nr.x / area2, nr.y / area2, nr.z / area2};
    double w = dot(n, v0);
    // an already found plane holding this triangle
    Plane* on = nullptr;
    for (Plane& P : planes) {
      if (std::fabs(dot(P.n, n)) < 1.0 - 1e-9) continue;
      if (std::fabs(dot(P.n, v0) - P.w) <= tol && std::fabs(dot(P.n, v1) - P.w) <= tol &&
          std::fabs(dot(P.n, v2) - P.w) <= tol) { on = &P; break; }
    }
    if (!on) {
      // a supporting plane: every scene vertex on one side (early out)
      bool below = true, above = true;
      for (uint32_t i = 0; i < num_vertices && (below || above); ++i) {
        const double s = dot(n, V(i)) - w;
        if (s > tol) below = false;
        if (s < -tol) above = false;
      }
      if (!below && !above) continue;
      if (!below) { n = {-n.x, -n.y, -n.z}; w = -w; }
      planes.push_back(Plane{n, w, {}, 0.0, 0.0});
      on = &planes.back();
    }
    // the member's own plane against the group's over the scene box
    const double wt = dot(n, v0);
    const D3 nt = dot(n, on->n) < 0 ? D3{-n.x, -n.y, -n.z} : n;
    const double wts = dot(n, on->n) < 0 ? -wt : wt;
    double dev = 0.0;
    for (const D3& k : corners) dev = std::max(dev, std::fabs((dot(nt, k) - wts) - (dot(on->n, k) - on->w)));
    on->tris.push_back(t);
    on->c_max = std::max(on->c_max, c);
    on->dev = std::max(on->dev, dev);
  }
  if (planes.empty()) return false;
  // the margin: the float-error bound of the worst culled triangle, plus the
  // gap between member planes and group planes, plus the runtime check's own
  // rounding (a float dot product against |x| <= S)
  double c_all = 1.0, dev_all = 0.0;
  for (const Plane& P : planes) { c_all = std::max(c_all, P.c_max); dev_all = std::max(dev_all, P.dev); }
  const double margin = 128.0 * kUnit * c_all * S + dev_all + 8.0 * kUnit * S;
  // every light vertex strictly inside (by four margins: two for the culled
  // triangles' error, two left for the light's, see cos_min); planes holding
  // a light triangle (or too close to one) keep their triangles
  std::vector<Plane> used;
  for (Plane& P : planes) {
    bool ok = true;
    for (uint32_t l = 0; l < num_lights * 3 && ok; ++l) {
      const float* q = light_vertices + 3 * l;
      if (!(dot(P.n, D3{q[0], q[1], q[2]}) - P.w <= -4.0 * margin)) ok = false;
    }
    if (ok) used.push_back(std::move(P));
  }
  // the planes that cull the most triangles, at most kMaxOccPlanes
  std::stable_sort(used.begin(), used.end(), [](const Plane& a, const Plane& b) { return a.tris.size() > b.tris.size(); });
  if (used.size() > kMaxOccPlanes) used.resize(kMaxOccPlanes);
  std::vector<uint8_t> culled(num_triangles, 0);
  for (const Plane& P : used) {
    for (uint32_t t : P.tris) culled[t] = 1;
    out.planes.push_back({(float)P.n.x, (float)P.n.y, (float)P.n.z, (float)P.w});
  }
  for (uint32_t t = 0; t < num_triangles; ++t) {
    if (culled[t]) ++out.culled;
    else out.keep.push_back(t);
  }
  // the float plane differs from the double one by rounding: covered by the
  // runtime check's 8 u S term
  out.margin = (float)margin;
  // the grazing guard (header comment): D_L over the planes used, c_L and the
  // normal deviation over the light triangles
  double D_L = 1e300, c_L = 1.0, ndev = 0.0;
  for (const Plane& P : used)
    for (uint32_t l = 0; l < num_lights * 3; ++l) {
      const float* q = light_vertices + 3 * l;
      D_L = std::min(D_L, P.w - dot(P.n, D3{q[0], q[1], q[2]}));
    }
  for (uint32_t l = 0; l < num_lights; ++l) {
    const float* q = light_vertices + 9 * (size_t)l;
    const D3 a{q[0], q[1], q[2]}, b{q[3], q[4], q[5]}, c{q[6], q[7], q[8]};
    const D3 ng0 = cross(sub(b, a), sub(c, a));
    const double A = len(ng0);
    if (!(A > 0.0)) { out = OccluderSet{}; return false; }   // degenerate light: no culling
    const D3 ng = {ng0.x / A, ng0.y / A, ng0.z / A};
    const D3 v[3] = {a, b, c};
    for (int k = 0; k < 3; ++k)   // c at each vertex (tri_test takes the triangle's first vertex as v0)
      c_L = std::max(c_L, len(sub(v[(k + 1) % 3], v[k])) * len(sub(v[(k + 2) % 3], v[k])) / A);
    for (int k = 0; k < 3; ++k) {
      const float* nv = light_normals + 9 * (size_t)l + 3 * k;
      const D3 n{nv[0], nv[1], nv[2]};
      const double nl = len(n);
      if (!(nl > 0.0)) { out = OccluderSet{}; return false; }
      // either orientation of the geometric normal (the kernels use |cos|)
      const D3 u{n.x / nl, n.y / nl, n.z / nl};
      ndev = std::max(ndev, std::min(len(sub(u, ng)), len(sub(u, D3{-ng.x, -ng.y, -ng.z}))));
    }
  }
  if (!(D_L > 0.0) || D_L > 1e299) { out = OccluderSet{}; return false; }
  // + 1e-5: the kernels' float cosine (a normalised interpolated normal and
  // direction, a few u) with room to spare
  out.cos_min = (float)(20.0 * kUnit * S * c_L / D_L + 2.0 * ndev + 1e-5);
  if (!(out.cos_min < 0.5f)) { out = OccluderSet{}; return false; }   // too few rays would qualify
  // a second tree pays only when it is markedly smaller than the main one:
  // it costs a plane test per shadow ray and its own nodes in LDS / L2
  if ((size_t)out.culled * kMinCulledFraction < num_triangles) {
    out = OccluderSet{};
    return false;
  }
  return true;
}

bool find_convex_occluders(const float* vertices, size_t stride_bytes, uint32_t num_vertices, const uint32_t* indices,
                           uint32_t num_triangles, const std::vector<uint32_t>& keep, const OccluderSet& occ,
                           ConvexSet& out) {
  out = ConvexSet{};
  if (keep.empty() || occ.planes.empty() || num_vertices == 0) return false;
  const size_t stride = stride_bytes / sizeof(float);
  auto V = [&](uint32_t i) { const float* p = vertices + stride * i; return D3{p[0], p[1], p[2]}; };
  auto N = [&](uint32_t i) { const float* p = vertices + stride * i + 3; return D3{p[0], p[1], p[2]}; };
  double amax = 0.0;
  for (uint32_t i = 0; i < num_vertices; ++i) {
    const D3 v = V(i);
    amax = std::max({amax, std::fabs(v.x), std::fabs(v.y), std::fabs(v.z)});
  }
  const double S = std::max(amax, 1e-6);
  const double tol = 1e-6 * S;
  // corners are matched by position (vertex records are per position and normal)
  auto key = [&](uint32_t vi) {
    const float* p = vertices + stride * vi;
    uint32_t b[3];
    std::memcpy(b, p, 12);
    return std::array<uint32_t, 3>{b[0], b[1], b[2]};
  };
  std::map<std::array<uint32_t, 3>, uint32_t> pos_id;
  std::vector<uint32_t> tri_pos(3 * keep.size());
  for (size_t i = 0; i < keep.size(); ++i)
    for (int c = 0; c < 3; ++c) {
      const auto k = key(indices[3 * keep[i] + c]);
      auto it = pos_id.emplace(k, (uint32_t)pos_id.size()).first;
      tri_pos[3 * i + c] = it->second;
    }
  // connected components over shared positions (union-find)
  std::vector<uint32_t> parent(pos_id.size());
  for (size_t i = 0; i < parent.size(); ++i) parent[i] = (uint32_t)i;
  auto find = [&](uint32_t a) { while (parent[a] != a) a = parent[a] = parent[parent[a]]; return a; };
  for (size_t i = 0; i < keep.size(); ++i) {
    const uint32_t a = find(tri_pos[3 * i]);
    parent[find(tri_pos[3 * i + 1])] = a;
    parent[find(tri_pos[3 * i + 2])] = find(tri_pos[3 * i]);
  }
  std::map<uint32_t, std::vector<size_t>> comps;   // root -> kept-triangle slots
  for (size_t i = 0; i < keep.size(); ++i) comps[find(tri_pos[3 * i])].push_back(i);
  if (comps.size() > kMaxConvex) return false;
  const double delta = 16.0 * (1e-5 * S + 1e-6);   // 16x the BVH boxes' padding (bvh.cpp)
  out.prim_face.assign(num_triangles, 0u);
  for (auto& [root, slots] : comps) {
    (void)root;
    // the solid's corner positions and centroid
    std::vector<D3> pts;
    std::vector<uint8_t> seen(pos_id.size(), 0);
    D3 cen{0, 0, 0};
    for (size_t i : slots)
      for (int c = 0; c < 3; ++c)
        if (!seen[tri_pos[3 * i + c]]) {
          seen[tri_pos[3 * i + c]] = 1;
          const D3 v = V(indices[3 * keep[i] + c]);
          pts.push_back(v);
          cen = {cen.x + v.x, cen.y + v.y, cen.z + v.z};
        }
    cen = {cen.x / pts.size(), cen.y / pts.size(), cen.z / pts.size()};
    struct Face { D3 n; double w; std::vector<uint32_t> tris; };
    std::vector<Face> faces;
    for (size_t i : slots) {
      const uint32_t t = keep[i];
      const D3 v0 = V(indices[3 * t]), v1 = V(indices[3 * t + 1]), v2 = V(indices[3 * t + 2]);
      const D3 nr = cross(sub(v1, v0), sub(v2, v0));
      const double a = len(nr);
      if (!(a > 1e-12 * S * S)) return false;
      D3 n{nr.x / a, nr.y / a, nr.z / a};
      double w = dot(n, v0);
      if (dot(n, cen) - w > 0.0) { n = {-n.x, -n.y, -n.z}; w = -w; }   // outward
      // flat shading normals: the shadow origin's offset (hit + n_interp * 1e-4)
      // is then along the face normal
      for (int c = 0; c < 3; ++c) {
        const D3 vn = N(indices[3 * t + c]);
        const double l = len(vn);
        if (!(l > 0.0) || dot(vn, n) / l < 0.999) return false;
      }
      Face* on = nullptr;
      for (Face& F : faces)
        if (dot(F.n, n) > 1.0 - 1e-9 && std::fabs(F.w - w) <= tol) { on = &F; break; }
      if (!on) { faces.push_back(Face{n, w, {}}); on = &faces.back(); }
      on->tris.push_back(t);
      if (on->tris.size() > 2) return false;
    }
    // the culled planes the solid stands on (its missing faces, e.g. a box's bottom)
    for (const auto& cp : occ.planes) {
      const D3 n{cp[0], cp[1], cp[2]};
      const double w = cp[3];
      bool touches = false;
      for (const D3& v : pts) touches |= std::fabs(dot(n, v) - w) <= tol;
      bool dup = false;
      for (const Face& F : faces) dup |= dot(F.n, n) > 1.0 - 1e-9 && std::fabs(F.w - w) <= tol;
      if (touches && !dup) faces.push_back(Face{n, w, {}});
    }
    // convex: every corner inside every face plane
    for (const Face& F : faces)
      for (const D3& v : pts)
        if (dot(F.n, v) - F.w > tol) return false;
    // three pairs of parallel faces (a parallelepiped); axis a's normal is the
    // first face's of the pair (its "hi" face), the other is the "lo" face
    if (faces.size() != 6) return false;
    std::array<float, 16> obb{};
    std::array<uint32_t, 8> ft;
    ft.fill(0xFFFFFFFFu);
    std::array<float, 18> fn{};
    std::vector<uint8_t> used(6, 0);
    uint32_t axis = 0;
    auto pack = [&](const Face& F) -> uint32_t {
      const uint32_t t0 = F.tris.size() > 0 ? F.tris[0] : 0xFFFFu, t1 = F.tris.size() > 1 ? F.tris[1] : 0xFFFFu;
      return (t0 & 0xFFFFu) | (t1 << 16);
    };
    for (size_t i = 0; i < 6 && axis < 3; ++i) {
      if (used[i]) continue;
      size_t j = 6;
      for (size_t k = i + 1; k < 6; ++k)   // the face most nearly opposite (within ~8 degrees)
        if (!used[k] && dot(faces[i].n, faces[k].n) < -0.99 && (j == 6 || dot(faces[i].n, faces[k].n) <
                                                                           dot(faces[i].n, faces[j].n)))
          j = k;
      if (j == 6) return false;
      used[i] = used[j] = 1;
      const Face& H = faces[i];   // n . x <= w_H
      const Face& L = faces[j];   // -n . x <= w_L  ->  n . x >= -w_L
      obb[3 * axis] = (float)H.n.x;
      obb[3 * axis + 1] = (float)H.n.y;
      obb[3 * axis + 2] = (float)H.n.z;
      // the slab the solid's corners span along n (the solid's faces need not
      // be exactly parallel: the Cornell box's blocks are slightly skewed),
      // [lo - delta, hi + delta] rounded outward: it holds every triangle
      const D3 na{(double)(float)H.n.x, (double)(float)H.n.y, (double)(float)H.n.z};
      double lo = 1e300, hi = -1e300;
      for (const D3& v : pts) { lo = std::min(lo, dot(na, v)); hi = std::max(hi, dot(na, v)); }
      obb[9 + 2 * axis] = std::nextafter((float)(lo - delta), -INFINITY);
      obb[9 + 2 * axis + 1] = std::nextafter((float)(hi + delta), INFINITY);
      for (uint32_t t : L.tris) { if (t >= 0xFFFFu) return false; out.prim_face[t] = out.count * 8 + 2 * axis + 1; }
      for (uint32_t t : H.tris) { if (t >= 0xFFFFu) return false; out.prim_face[t] = out.count * 8 + 2 * axis + 2; }
      ft[2 * axis] = pack(L);
      ft[2 * axis + 1] = pack(H);
      const double ln[3] = {L.n.x, L.n.y, L.n.z}, hn[3] = {H.n.x, H.n.y, H.n.z};
      for (int c = 0; c < 3; ++c) {
        fn[3 * (2 * axis) + c] = (float)ln[c];
        fn[3 * (2 * axis + 1) + c] = (float)hn[c];
      }
      ++axis;
    }
    if (axis != 3) return false;
    out.obb.push_back(obb);
    out.face_tris.push_back(ft);
    out.face_normal.push_back(fn);
    out.count += 1;
  }
  out.delta = (float)delta;
  return true;
}

}  // namespace mrt
