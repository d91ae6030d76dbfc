// bvh_stats — CPU model of the GPU traversal loop (diagnostic tool).
// Builds the product BVH for a scene, traces camera rays (8x8 pixel blocks
// per 64-lane wave, as bounce 0 does) and cosine-distributed secondary rays
// from camera-ray hit points, and reports per-ray node steps / leaf visits /
// triangle tests plus the wave-level loop trip counts of the "if-if" loop
// (max over lanes of per-lane iterations) — the SIMD efficiency model.
// build: g++ -O2 -std=c++17 -I../metal-renderer_amd/csrc bvh_stats.cpp ../metal-renderer_amd/csrc/{scene,bvh}.cpp
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "bvh.h"
#include "scene.h"

using namespace mrt;

struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

static bool g_cull = true;
struct Counts { int steps = 0, inner = 0, leaves = 0, tris = 0; float t = INFINITY; };

static Counts trace(const BvhResult& b, V o, V d) {
  Counts c;
  V inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
  int32_t node = b.root;
  std::vector<int32_t> st;
  std::vector<float> st_t;
  while (true) {
    c.steps++;
    if (node >= 0 && b.width == 4) {
      // BVH4: test 4 children, descend into the nearest hit, push the others
      // far-to-near with their entry distance (culled on pop)
      c.inner++;
      const float* n = &b.nodes[32 * (size_t)node];
      float tn[4];
      int32_t ref[4];
      int hits = 0;
      for (int k = 0; k < 4; ++k) {
        ref[k] = (int32_t)fb(n[24 + k]);
        float a0 = (n[k] - o.x) * inv.x, a1 = (n[4 + k] - o.x) * inv.x;
        float b0 = (n[8 + k] - o.y) * inv.y, b1 = (n[12 + k] - o.y) * inv.y;
        float c0 = (n[16 + k] - o.z) * inv.z, c1 = (n[20 + k] - o.z) * inv.z;
        float t0 = std::max(std::max(std::min(a0, a1), std::min(b0, b1)), std::max(std::min(c0, c1), 0.0f));
        float t1 = std::min(std::min(std::max(a0, a1), std::max(b0, b1)), std::min(std::max(c0, c1), c.t));
        tn[k] = (ref[k] != 0x7FFFFFFF && t0 <= t1) ? t0 : INFINITY;
        hits += tn[k] < INFINITY;
      }
      if (hits) {
        int idx[4] = {0, 1, 2, 3};
        std::sort(idx, idx + 4, [&](int a, int bb) { return tn[a] < tn[bb]; });
        for (int k = hits - 1; k >= 1; --k) { st.push_back(ref[idx[k]]); st_t.push_back(tn[idx[k]]); }
        node = ref[idx[0]];
        continue;
      }
    } else if (node >= 0) {
      c.inner++;
      const float* n = &b.nodes[16 * (size_t)node];
      auto box = [&](float x0, float x1, float y0, float y1, float z0, float z1, float& tn) {
        float a0 = (x0 - o.x) * inv.x, a1 = (x1 - o.x) * inv.x;
        float b0 = (y0 - o.y) * inv.y, b1 = (y1 - o.y) * inv.y;
        float c0 = (z0 - o.z) * inv.z, c1 = (z1 - o.z) * inv.z;
        tn = std::max(std::max(std::min(a0, a1), std::min(b0, b1)), std::max(std::min(c0, c1), 0.0f));
        float tf = std::min(std::min(std::max(a0, a1), std::max(b0, b1)), std::min(std::max(c0, c1), c.t));
        return tn <= tf;
      };
      float tl, tr;
      bool hl = box(n[0], n[1], n[2], n[3], n[8], n[9], tl), hr = box(n[4], n[5], n[6], n[7], n[10], n[11], tr);
      int32_t rl = (int32_t)fb(n[12]), rr = (int32_t)fb(n[13]);
      if (hl && hr) { bool sw = tr < tl; st.push_back(sw ? rl : rr); node = sw ? rr : rl; continue; }
      if (hl) { node = rl; continue; }
      if (hr) { node = rr; continue; }
    } else {
      c.leaves++;
      uint32_t lr = ~(uint32_t)node, first = lr >> 4, cnt = (lr & 15) + 1;
      for (uint32_t k = 0; k < cnt; ++k) {
        c.tris++;
        const float* t = &b.tris[12 * (size_t)(first + k)];
        V v0 = {t[0], t[1], t[2]}, e1 = {t[4], t[5], t[6]}, e2 = {t[8], t[9], t[10]};
        V p = cross(d, e2);
        float det = dot(e1, p);
        if (det == 0) continue;
        float iv = 1.0f / det;
        V s = sub(o, v0);
        float b1 = dot(s, p) * iv;
        if (b1 < 0 || b1 > 1) continue;
        V q = cross(s, e1);
        float b2 = dot(d, q) * iv;
        if (b2 < 0 || b1 + b2 > 1) continue;
        float tt = dot(e2, q) * iv;
        if (tt >= 0 && tt <= c.t) c.t = tt;
      }
    }
    if (b.width == 4) {
      bool found = false;
      while (!st.empty()) {
        node = st.back();
        float t = st_t.back();
        st.pop_back();
        st_t.pop_back();
        if (t <= c.t || !g_cull) { found = true; break; }
      }
      if (!found) break;
      continue;
    }
    if (st.empty()) break;
    node = st.back();
    st.pop_back();
  }
  return c;
}

int main(int argc, char** argv) {
  const std::string obj = argc > 1 ? argv[1] : "../metal-renderer_amd/scenes/cornellbox.obj";
  const uint32_t proc = argc > 2 ? (uint32_t)atoi(argv[2]) : 0;
  const uint32_t leaf = argc > 3 ? (uint32_t)atoi(argv[3]) : 4;
  const uint32_t width = argc > 4 ? (uint32_t)atoi(argv[4]) : 2;
  g_cull = argc > 5 ? atoi(argv[5]) != 0 : true;
  HostScene sc;
  std::string err;
  if (!import_obj(obj, "", sc, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
  if (proc) append_procedural_mesh(sc, proc, 1);
  flatten(sc);
  BvhBuildOptions opt;
  opt.max_leaf_size = leaf;
  opt.width = width;
  BvhResult b;
  if (!build_bvh(sc.vertices.data()->v, sizeof(RefVertex), sc.indices.data(), (uint32_t)sc.references.size(), opt, b,
                 err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
  std::printf("%s: %zu tris, BVH%u %u nodes, %u leaves, depth %u (wide %u), stack %u, SAH %.2f\n", obj.c_str(),
              sc.references.size(), b.width, b.num_nodes, b.num_leaves, b.max_depth, b.wide_depth, b.max_stack,
              b.sah_cost);
  const uint32_t W = 256, H = 144;
  std::mt19937 rng(5);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  for (int pass = 0; pass < 2; ++pass) {
    double steps = 0, inner = 0, leaves = 0, tris = 0, wave_iters = 0, lane_iters = 0;
    uint64_t rays = 0;
    for (uint32_t by = 0; by + 8 <= H; by += 8)
      for (uint32_t bx = 0; bx + 8 <= W; bx += 8) {
        int wave_max = 0;
        for (uint32_t q = 0; q < 64; ++q) {
          uint32_t x = bx + (q & 7), y = by + (q >> 3);
          float ncx = 2.0f * x / (W - 1) - 1.0f, ncy = (2.0f * y / (H - 1) - 1.0f) * H / W;
          V d = {ncx, ncy, -1.0f};
          float l = std::sqrt(dot(d, d));
          d = {d.x / l, d.y / l, d.z / l};
          V o = {0.0f, 1.0f, 2.35f};
          Counts c = trace(b, o, d);
          if (pass == 1) {   // a diffuse bounce from the primary hit (random hemisphere-ish)
            if (!std::isfinite(c.t)) continue;
            V h = {o.x + d.x * c.t * 0.999f, o.y + d.y * c.t * 0.999f, o.z + d.z * c.t * 0.999f};
            V r;
            do { r = {2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1}; } while (dot(r, r) > 1 || dot(r, r) < 1e-4f);
            float rl = std::sqrt(dot(r, r));
            r = {r.x / rl, r.y / rl, r.z / rl};
            if (dot(r, d) > 0) r = {-r.x, -r.y, -r.z};
            c = trace(b, h, r);
          }
          steps += c.steps; inner += c.inner; leaves += c.leaves; tris += c.tris; ++rays;
          wave_max = std::max(wave_max, c.steps);
          lane_iters += c.steps;
        }
        wave_iters += 64.0 * wave_max;
      }
    std::printf("%s rays: per ray steps %.1f (interior %.1f, leaves %.1f, tri tests %.1f); if-if SIMD efficiency %.2f\n",
                pass ? "secondary" : "camera", steps / rays, inner / rays, leaves / rays, tris / rays,
                lane_iters / wave_iters);
  }
  // ray-sorting model: secondary rays in pixel-block order, then stably
  // sorted by a direction key inside windows of S rays; efficiency of waves
  {
    struct R { V o, d; int key; int steps; };
    std::vector<R> rs;
    std::mt19937 rng2(7);
    for (uint32_t by = 0; by + 8 <= H; by += 8)
      for (uint32_t bx = 0; bx + 8 <= W; bx += 8)
        for (uint32_t q = 0; q < 64; ++q) {
          uint32_t x = bx + (q & 7), y = by + (q >> 3);
          float ncx = 2.0f * x / (W - 1) - 1.0f, ncy = (2.0f * y / (H - 1) - 1.0f) * H / W;
          V d = {ncx, ncy, -1.0f};
          float l = std::sqrt(dot(d, d));
          d = {d.x / l, d.y / l, d.z / l};
          V o = {0.0f, 1.0f, 2.35f};
          Counts c = trace(b, o, d);
          if (!std::isfinite(c.t)) continue;
          V h = {o.x + d.x * c.t * 0.999f, o.y + d.y * c.t * 0.999f, o.z + d.z * c.t * 0.999f};
          V r;
          do { r = {2 * U(rng2) - 1, 2 * U(rng2) - 1, 2 * U(rng2) - 1}; } while (dot(r, r) > 1 || dot(r, r) < 1e-4f);
          float rl = std::sqrt(dot(r, r));
          r = {r.x / rl, r.y / rl, r.z / rl};
          if (dot(r, d) > 0) r = {-r.x, -r.y, -r.z};
          R rr{h, r, 0, trace(b, h, r).steps};
          rs.push_back(rr);
        }
    for (int axis = 0; axis < 3; ++axis) {   // 1-bit keys: sign of one direction component, global 2-way partition
      std::vector<R> v = rs;
      std::stable_sort(v.begin(), v.end(), [&](const R& a, const R& c) {
        const float da = axis == 0 ? a.d.x : axis == 1 ? a.d.y : a.d.z, dc = axis == 0 ? c.d.x : axis == 1 ? c.d.y : c.d.z;
        return (da > 0) < (dc > 0); });
      double li = 0, wi = 0;
      for (size_t w0 = 0; w0 < v.size(); w0 += 64) {
        int mx = 0;
        for (size_t i = w0; i < std::min(v.size(), w0 + 64); ++i) { li += v[i].steps; mx = std::max(mx, v[i].steps); }
        wi += 64.0 * mx;
      }
      std::printf("sorted secondaries: sign of d[%d] (global 2-way): SIMD efficiency %.3f\n", axis, li / wi);
    }
    for (int keybits : {0, 3, 6}) {
      for (size_t S : {size_t(128), size_t(1024), size_t(8192), rs.size()}) {
        std::vector<R> v = rs;
        for (R& x : v) {
          int k = (x.d.x > 0) | ((x.d.y > 0) << 1) | ((x.d.z > 0) << 2);
          if (keybits == 6) {   // octant + dominant axis + half
            float ax = std::fabs(x.d.x), ay = std::fabs(x.d.y), az = std::fabs(x.d.z);
            int dom = ax >= ay && ax >= az ? 0 : (ay >= az ? 1 : 2);
            k = k * 8 + dom * 2 + (std::max(ax, std::max(ay, az)) > 0.8f);
          }
          x.key = keybits ? k : 0;
        }
        for (size_t w0 = 0; w0 < v.size(); w0 += S)
          std::stable_sort(v.begin() + w0, v.begin() + std::min(v.size(), w0 + S), [](const R& a, const R& c) { return a.key < c.key; });
        double li = 0, wi = 0;
        for (size_t w0 = 0; w0 < v.size(); w0 += 64) {
          int mx = 0;
          for (size_t i = w0; i < std::min(v.size(), w0 + 64); ++i) { li += v[i].steps; mx = std::max(mx, v[i].steps); }
          wi += 64.0 * mx;
        }
        std::printf("sorted secondaries: key bits %d window %zu: SIMD efficiency %.3f\n", keybits, S, li / wi);
        if (!keybits) break;
      }
    }
  }
  return 0;
}
