// primary_check — CPU check that the camera-ray candidate lists (csrc/primary.cpp)
// are conservative: for every pixel of a W x H frame and `jitters` noise
// samples per pixel (plus the jitter extremes), the camera ray is formed with
// camera_ray's float arithmetic (kernels.hip, = rayGenerator,
// renderer/Shaders.metal:75-103) and its nearest hit found by brute force over
// every triangle with the kernels' Moller-Trumbore arithmetic (tri_bary, IEEE
// float, no contraction); a listed block must contain the winning triangle.
// Prints "violations N blocks B listed L mean M" and exits non-zero on a
// violation.
// Argument 7 = 1: the FAST build's arithmetic instead (kernels.hip
// MRT_PRECISE=0): dot products and crosses contracted into FMAs, reciprocals
// and the normalisation's reciprocal square root approximate — each result
// perturbed by a random -1 / 0 / +1 ulp per use, the documented accuracy of
// v_rcp_f32 / v_rsq_f32 — so the lists are checked against the answers the
// benchmarked build can give, not only the IEEE ones.
// build: g++ -O2 -std=c++17 -ffp-contract=off -I../metal-renderer_amd/csrc primary_check.cpp
//        ../metal-renderer_amd/csrc/{scene,bvh,primary}.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "bvh.h"
#include "primary.h"
#include "scene.h"

using namespace mrt;

namespace {

struct V { float x, y, z; };
bool g_fast = false;
uint32_t g_ulp = 0x9E3779B9u;   // xorshift32 state of the ulp choice
// an approximate unit's result: the IEEE value moved by -1, 0 or +1 ulp,
// chosen by a hash of the value and a per-ray salt (no serial state)
float approx(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  const uint32_t k = ((u ^ g_ulp) * 0x9E3779B1u) >> 30;   // 0..3: 0 and 3 keep the value
  if (k == 0 || k == 3 || (u & 0x7F800000u) == 0x7F800000u || (u & 0x7FFFFFFFu) == 0) return x;
  u = k == 1 ? u + 1 : u - 1;   // one ulp away from / toward zero
  std::memcpy(&x, &u, 4);
  return x;
}
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <bool F>
float dot(V a, V b) {
  if (F) return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x));
  return (a.x * b.x + a.y * b.y) + a.z * b.z;
}
template <bool F>
V cross(V a, V b) {
  if (F)
    return {std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)), std::fma(a.x, b.y, -(a.y * b.x))};
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

template <bool F>
bool tri_bary(V o, V d, V v0, V e1, V e2, float& t) {
  const V p = cross<F>(d, e2);
  const float det = dot<F>(e1, p);
  const float inv = F ? approx(1.0f / det) : 1.0f / det;
  const V s = sub(o, v0);
  const float b1 = dot<F>(s, p) * inv;
  const V q = cross<F>(s, e1);
  const float b2 = dot<F>(d, q) * inv;
  t = dot<F>(e2, q) * inv;
  return (det != 0.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f);
}

template <bool F>
void camera_ray(uint32_t x, uint32_t y, uint32_t W, uint32_t H, float nsx, float nsy, V& o, V& d) {
  const float wm1 = float(W - 1), hm1 = float(H - 1);
  o = {kCameraX, kCameraY, kCameraZ};   // mrt_layout.h, shared with kernels.hip camera_ray
  if (F) {   // m_div(a, b) = a * rcp(b), contracted where the compiler can
    const float rw = approx(1.0f / float(W)), rw1 = approx(1.0f / wm1), rh1 = approx(1.0f / hm1);
    const float aspect = float(H) * rw;
    const float dudvx = (nsx * 2.0f - 1.0f) * rw1, dudvy = (nsy * 2.0f - 1.0f) * rh1;
    const float ncx = std::fma(float(2 * x), rw1, -1.0f), ncy = std::fma(float(2 * y), rh1, -1.0f);
    V v = {dudvx + ncx, std::fma(ncy, aspect, dudvy), -1.0f};
    const float r = approx(1.0f / std::sqrt(dot<F>(v, v)));
    d = {v.x * r, v.y * r, v.z * r};
    return;
  }
  const float aspect = float(H) / float(W);
  const float dudvx = (nsx * 2.0f - 1.0f) / wm1, dudvy = (nsy * 2.0f - 1.0f) / hm1;
  const float ncx = float(2 * x) / wm1 - 1.0f, ncy = float(2 * y) / hm1 - 1.0f;
  V v = {dudvx + ncx, dudvy + ncy * aspect, -1.0f};
  const float l = std::sqrt(dot<F>(v, v));
  d = {v.x * (1.0f / l), v.y * (1.0f / l), v.z * (1.0f / l)};
}

// every pixel's jittered camera rays: brute-force nearest triangle vs the
// block's list; returns violations << 40 | rays
template <bool F>
uint64_t check(const BvhResult& b, const PrimaryLists& pl, uint32_t T, uint32_t W, uint32_t H, int jitters) {
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  const float extremes[3] = {0.0f, 0.99999994f, 0.5f};   // ns in [0, 1)
  uint64_t violations = 0, rays = 0;
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) {
      const uint32_t blk = x / kPrimaryBlock + (y / kPrimaryBlock) * pl.blocks_x;
      const uint32_t hd = pl.words[blk];
      if ((hd & 0xFFu) == kPrimaryFallback) continue;
      const uint32_t* list = pl.words.data() + (hd >> 8);
      const uint32_t cnt = hd & 0xFFu;
      for (int j = 0; j < jitters + 9; ++j) {
        const float nx = j < 9 ? extremes[j % 3] : U(rng), ny = j < 9 ? extremes[j / 3] : U(rng);
        V o, d;
        g_ulp = (uint32_t)rays * 0x85EBCA6Bu;   // per-ray salt of the ulp choices
        camera_ray<F>(x, y, W, H, nx, ny, o, d);
        ++rays;
        float best = INFINITY;
        uint32_t bp = 0xFFFFFFFFu, bk = 0;
        bool found = false;
        for (uint32_t k = 0; k < T; ++k) {
          const float* t = b.tris.data() + 12 * (size_t)k;
          float tt;
          if (!tri_bary<F>(o, d, {t[0], t[1], t[2]}, {t[4], t[5], t[6]}, {t[8], t[9], t[10]}, tt)) continue;
          uint32_t prim;
          std::memcpy(&prim, &t[3], 4);
          if (tt >= 0.0f && tt <= best && (!found || tt < best || prim < bp)) {
            found = true;
            best = tt;
            bp = prim;
            bk = k;
          }
        }
        if (!found) continue;
        bool in = false;
        for (uint32_t i = 0; i < cnt; ++i) in |= list[i] == bk;
        if (!in) {
          if (violations < 10)
            std::printf("miss: pixel (%u, %u) ns (%.7g, %.7g) hit leaf triangle %u (prim %u, t %.7g) not in block %u's list\n",
                        x, y, nx, ny, bk, bp, best, blk);
          ++violations;
        }
      }
    }
  return (violations << 40) | rays;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: primary_check scene.obj W H [jitters] [procedural_tris] [cap] [fast]\n");
    return 2;
  }
  const uint32_t W = (uint32_t)std::atoi(argv[2]), H = (uint32_t)std::atoi(argv[3]);
  const int jitters = argc > 4 ? std::atoi(argv[4]) : 4;
  const uint32_t proc = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 0;
  const uint32_t cap = argc > 6 ? (uint32_t)std::atoi(argv[6]) : 12;
  g_fast = argc > 7 && std::atoi(argv[7]) != 0;
  HostScene sc;
  std::string err;
  if (!import_obj(argv[1], "", sc, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 2; }
  if (proc) append_procedural_mesh(sc, proc, 1);
  flatten(sc);
  BvhBuildOptions opt;
  opt.width = 4;
  BvhResult b;
  if (!build_bvh(sc.vertices.data()->v, sizeof(RefVertex), sc.indices.data(), (uint32_t)sc.references.size(), opt, b,
                 err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 2; }
  const uint32_t T = (uint32_t)(b.tris.size() / 12);
  PrimaryLists pl;
  const bool built = build_primary_lists(b.tris.data(), T, W, H, cap, pl);
  if (!built) {
    std::printf("violations 0 blocks %u listed 0 mean 0 (lists not built)\n", (W + 7) / 8 * ((H + 7) / 8));
    return 0;
  }
  const uint64_t rays_violations = g_fast ? check<true>(b, pl, T, W, H, jitters) : check<false>(b, pl, T, W, H, jitters);
  const uint64_t violations = rays_violations >> 40, rays = rays_violations & ((1ull << 40) - 1);
  std::printf("violations %llu rays %llu blocks %zu listed %u mean %.2f\n", (unsigned long long)violations,
              (unsigned long long)rays, (size_t)pl.blocks_x * pl.blocks_y, pl.listed_blocks, pl.mean_count);
  return violations ? 1 : 0;
}
