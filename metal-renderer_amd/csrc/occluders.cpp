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
// d_q / d_p from q) beyond the computed t_q for every direction; a grazing
// direction gives |t| > 6 S > t_q.  Triangles with c > 16 (slivers) are kept.
#include "occluders.h"

#include <algorithm>
#include <cmath>

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
                    uint32_t num_triangles, const float* light_vertices, uint32_t num_lights, OccluderSet& out) {
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
  // every light vertex strictly inside (by twice the margin); planes holding a
  // light triangle (or too close to one) keep their triangles
  std::vector<Plane> used;
  for (Plane& P : planes) {
    bool ok = true;
    for (uint32_t l = 0; l < num_lights * 3 && ok; ++l) {
      const float* q = light_vertices + 3 * l;
      if (!(dot(P.n, D3{q[0], q[1], q[2]}) - P.w <= -2.0 * margin)) ok = false;
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
  // a second tree pays only when it is markedly smaller than the main one:
  // it costs a plane test per shadow ray and its own nodes in LDS / L2
  if ((size_t)out.culled * kMinCulledFraction < num_triangles) {
    out = OccluderSet{};
    return false;
  }
  return true;
}

}  // namespace mrt
