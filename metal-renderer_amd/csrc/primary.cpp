// primary.cpp — camera-ray candidate lists per 8x8 pixel block (see primary.h).
//
// Conservative by construction, in double precision:
//   * the block's rectangle on the image plane covers every direction
//     camera_ray (kernels.hip, = rayGenerator, renderer/Shaders.metal:75-103)
//     can produce for its pixels: pixel centre +- the noise jitter
//     (ns * 2 - 1) / (W - 1) in x and (ns * 2 - 1) / (H - 1) in y, ns in [0, 1);
//   * a triangle is listed when its perspective projection, grown by a margin
//     that bounds the float Moller-Trumbore test's error for that triangle,
//     overlaps the rectangle (separating-axis test: the two rectangle axes and
//     the three projected edge normals);
//   * triangles that reach the camera plane, are (nearly) edge-on to the
//     camera, or are degenerate go into every list.
#include "primary.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace mrt {
namespace {

struct D3 { double x, y, z; };
D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double len(D3 a) { return std::sqrt(dot(a, a)); }

// image-plane rectangle [x0, x1] x [y0, y1] of the camera directions (X, Y, -1)
struct Rect { double x0, x1, y0, y1; };

// 2-D separating-axis test of triangle p[3] against rectangle r grown by m
bool overlaps(const double (*p)[2], const Rect& r, double m) {
  const double x0 = r.x0 - m, x1 = r.x1 + m, y0 = r.y0 - m, y1 = r.y1 + m;
  const double tx0 = std::min({p[0][0], p[1][0], p[2][0]}), tx1 = std::max({p[0][0], p[1][0], p[2][0]});
  const double ty0 = std::min({p[0][1], p[1][1], p[2][1]}), ty1 = std::max({p[0][1], p[1][1], p[2][1]});
  if (tx1 < x0 || tx0 > x1 || ty1 < y0 || ty0 > y1) return false;
  const double cx = 0.5 * (x0 + x1), cy = 0.5 * (y0 + y1), hx = 0.5 * (x1 - x0), hy = 0.5 * (y1 - y0);
  for (int e = 0; e < 3; ++e) {
    const double* a = p[e];
    const double* b = p[(e + 1) % 3];
    const double nx = -(b[1] - a[1]), ny = b[0] - a[0];
    if (nx * nx + ny * ny < 1e-30) continue;   // zero-length projected edge: no axis
    double lo = INFINITY, hi = -INFINITY;
    for (int k = 0; k < 3; ++k) {
      const double v = p[k][0] * nx + p[k][1] * ny;
      lo = std::min(lo, v);
      hi = std::max(hi, v);
    }
    const double c = cx * nx + cy * ny, h = hx * std::fabs(nx) + hy * std::fabs(ny);
    if (hi < c - h || lo > c + h) return false;
  }
  return true;
}

}  // namespace

bool build_primary_lists(const float* tris, uint32_t num_tris, uint32_t W, uint32_t H, uint32_t cap,
                         PrimaryLists& out) {
  out = PrimaryLists{};
  if (W < 2 || H < 2 || num_tris == 0 || cap == 0 || cap >= kPrimaryFallback) return false;
  const uint32_t BX = (W + kPrimaryBlock - 1) / kPrimaryBlock, BY = (H + kPrimaryBlock - 1) / kPrimaryBlock;
  const uint64_t nblocks = (uint64_t)BX * BY;
  const double W1 = W - 1.0, H1 = H - 1.0, aspect = (double)H / (double)W;
  const D3 O = {(double)kCameraX, (double)kCameraY, (double)kCameraZ};   // camera_ray's origin (mrt_layout.h)
  // rectangle of block (bx, by): pixel centres x0..x1, y0..y1 plus the jitter
  auto rect = [&](uint32_t bx, uint32_t by) {
    const double px0 = bx * kPrimaryBlock, px1 = std::min<double>(px0 + kPrimaryBlock - 1, W - 1.0);
    const double py0 = by * kPrimaryBlock, py1 = std::min<double>(py0 + kPrimaryBlock - 1, H - 1.0);
    return Rect{2.0 * px0 / W1 - 1.0 - 1.0 / W1, 2.0 * px1 / W1 - 1.0 + 1.0 / W1,
                (2.0 * py0 / H1 - 1.0) * aspect - 1.0 / H1, (2.0 * py1 / H1 - 1.0) * aspect + 1.0 / H1};
  };
  constexpr double kMargin = 1e-4;   // image-plane units (a 1080p pixel is ~1e-3)
  constexpr double kEps = 6e-8;      // float unit roundoff
  std::vector<std::vector<uint32_t>> lists(nblocks);
  std::vector<uint32_t> everywhere;
  uint64_t entries = 0;
  const uint64_t budget = nblocks * (uint64_t)cap * 2;   // candidate entries worth building at all
  for (uint32_t k = 0; k < num_tris; ++k) {
    const float* t = tris + 12 * (size_t)k;
    const D3 v0 = {t[0], t[1], t[2]}, e1 = {t[4], t[5], t[6]}, e2 = {t[8], t[9], t[10]};
    const D3 v[3] = {v0, add(v0, e1), add(v0, e2)};
    D3 rel[3];
    double smin = INFINITY, smax = -INFINITY, R = 0.0;
    for (int i = 0; i < 3; ++i) {
      rel[i] = sub(v[i], O);
      const double s = -rel[i].z;   // depth in front of the camera
      smin = std::min(smin, s);
      smax = std::max(smax, s);
      R = std::max(R, len(rel[i]));
    }
    if (smax < -1e-3) continue;   // wholly behind the camera: no camera ray reaches it
    const D3 n = cross(e1, e2);
    const double nl = len(n), l1 = len(e1), l2 = len(e2);
    const double hgt = nl > 0.0 ? std::fabs(dot(n, sub(v0, O))) / nl : 0.0;   // camera's distance to the plane
    bool all = smin < 1e-3 || !(nl > 1e-9 * l1 * l2) || !(hgt > 1e-7 * R);
    double m = kMargin;
    double p[3][2];
    if (!all) {
      double pmax = 0.0;
      for (int i = 0; i < 3; ++i) {
        p[i][0] = rel[i].x / -rel[i].z;
        p[i][1] = rel[i].y / -rel[i].z;
        pmax = std::max(pmax, std::fabs(p[i][0]) + std::fabs(p[i][1]));
      }
      // Float error of the test (tri_bary: det = e1.(d x e2), b1 = (s.p)/det,
      // b2 = (d.q)/det, s = o - v0 with |s| <= R): a camera ray meeting the
      // plane at distance r <= R has |det| = |n| hgt / r >= |n| hgt / R, the
      // numerators' rounding is ~eps R |e| and det's ~eps |e1||e2|, so a
      // barycentric is off by at most db (generous constant).  That moves the
      // hit point by db * |e|max in 3-D, at depth >= smin: at most
      // db |e|max (1 + |p|) / smin on the image plane.
      const double emax = std::max(l1, l2);
      const double db = 16.0 * kEps * R * (R * emax + l1 * l2) / (nl * hgt);
      m += 2.0 * db * emax * (1.0 + pmax) / smin;
      if (!(m < 0.25)) all = true;
    }
    if (all) {
      everywhere.push_back(k);
      if (everywhere.size() > cap) return false;
      continue;
    }
    // blocks whose pixel range can meet the projection's bounding box
    const double X0 = std::min({p[0][0], p[1][0], p[2][0]}) - m, X1 = std::max({p[0][0], p[1][0], p[2][0]}) + m;
    const double Y0 = std::min({p[0][1], p[1][1], p[2][1]}) - m, Y1 = std::max({p[0][1], p[1][1], p[2][1]}) + m;
    const double px0 = (X0 + 1.0) * W1 * 0.5, px1 = (X1 + 1.0) * W1 * 0.5;
    const double py0 = (Y0 / aspect + 1.0) * H1 * 0.5, py1 = (Y1 / aspect + 1.0) * H1 * 0.5;
    const double slack_y = 1.0 / aspect + 1.0;
    const int64_t bx0 = std::max<int64_t>(0, (int64_t)std::floor((px0 - kPrimaryBlock - 1.0) / kPrimaryBlock));
    const int64_t bx1 = std::min<int64_t>(BX - 1, (int64_t)std::floor((px1 + 1.0) / kPrimaryBlock));
    const int64_t by0 = std::max<int64_t>(0, (int64_t)std::floor((py0 - kPrimaryBlock - slack_y) / kPrimaryBlock));
    const int64_t by1 = std::min<int64_t>(BY - 1, (int64_t)std::floor((py1 + slack_y) / kPrimaryBlock));
    if (bx0 > bx1 || by0 > by1) continue;
    if (entries + (uint64_t)(bx1 - bx0 + 1) * (by1 - by0 + 1) > 4 * budget) return false;   // too dense to pay off
    for (int64_t by = by0; by <= by1; ++by)
      for (int64_t bx = bx0; bx <= bx1; ++bx) {
        std::vector<uint32_t>& l = lists[(size_t)by * BX + bx];
        if (l.size() > cap) continue;   // already over: stays a fallback block
        if (!overlaps(p, rect((uint32_t)bx, (uint32_t)by), m)) continue;
        l.push_back(k);
        ++entries;
      }
  }
  out.blocks_x = BX;
  out.blocks_y = BY;
  out.words.assign(nblocks, 0u);
  uint64_t listed = 0, total = 0;
  for (uint64_t b = 0; b < nblocks; ++b) {
    std::vector<uint32_t>& l = lists[b];
    const size_t n = l.size() + everywhere.size();
    if (n > cap) {
      out.words[b] = kPrimaryFallback;
      continue;
    }
    const uint64_t off = out.words.size();
    if (off >= (1ull << 24)) { out = PrimaryLists{}; return false; }
    l.insert(l.end(), everywhere.begin(), everywhere.end());
    std::sort(l.begin(), l.end());
    out.words[b] = (uint32_t)(off << 8) | (uint32_t)n;
    out.words.insert(out.words.end(), l.begin(), l.end());
    ++listed;
    total += n;
  }
  out.listed_blocks = (uint32_t)listed;
  out.mean_count = listed ? (double)total / (double)listed : 0.0;
  if (listed * 2 < nblocks) {   // most blocks would traverse anyway
    out = PrimaryLists{};
    return false;
  }
  return true;
}

}  // namespace mrt
