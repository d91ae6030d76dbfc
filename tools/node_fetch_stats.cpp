// node_fetch_stats — CPU model of the path kernel's BVH4 node fetches (C4 /
// C5 scene), to see where a larger LDS-resident top of the tree would pay.
// Builds the product tree (bvh.cpp, the options mrt_scene_create uses for a
// >= 64 K-triangle scene; the first 256 interior nodes in BFS order), reads
// query records written by tools/node_fetch_rays.py (origin, tmin, direction,
// tmax, kind: 0 nearest, 1 any-hit below tmax) and traverses each as the
// kernels do (children entered near to far, culled beyond h.t * (1 + 2^-11);
// any-hit queries stop at their first hit).  Reports interior-node visits per
// query: total, by depth, and how many would be global-memory fetches for an
// LDS top of B nodes (BFS prefix).
// build: g++ -O2 -std=c++17 -I../metal-renderer_amd/csrc node_fetch_stats.cpp \
//        ../metal-renderer_amd/csrc/{scene,bvh}.cpp -o node_fetch_stats -lpthread
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "bvh.h"
#include "scene.h"

using namespace mrt;

static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: node_fetch_stats <obj> <rays.bin> [procedural]\n"); return 1; }
  const uint32_t proc = argc > 3 ? (uint32_t)atoi(argv[3]) : 1u << 20;
  HostScene sc;
  std::string err;
  if (!import_obj(argv[1], "", sc, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
  if (proc) append_procedural_mesh(sc, proc, 1);
  flatten(sc);
  BvhBuildOptions opt;   // mrt_scene_create for T >= 65536
  opt.width = 4;
  opt.lds_node_budget = 256;
  if (sc.references.size() >= 65536) { opt.bins = 64; opt.exact_sah_below = 65536; }
  BvhResult b;
  if (!build_bvh(sc.vertices.data()->v, sizeof(RefVertex), sc.indices.data(), (uint32_t)sc.references.size(), opt, b,
                 err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
  std::vector<uint8_t> depth(b.num_nodes, 0);
  for (uint32_t n = 0; n < b.num_nodes; ++n)
    for (int c = 0; c < 4; ++c) {
      const int32_t r = (int32_t)fb(b.nodes[32 * (size_t)n + 24 + c]);
      if (r >= 0 && r != kEmptyChild) depth[r] = depth[n] + 1;
    }
  FILE* f = std::fopen(argv[2], "rb");
  if (!f) return 1;
  std::vector<float> rec;
  float buf[9];
  while (std::fread(buf, 4, 9, f) == 9) rec.insert(rec.end(), buf, buf + 9);
  std::fclose(f);
  const size_t n = rec.size() / 9;
  const uint32_t budgets[] = {45, 64, 90, 128, 180, 256};
  constexpr int kB = 6;
  double visits[2] = {0, 0}, global[2][kB] = {}, by_depth[2][32] = {}, leaf_visits[2] = {0, 0};
  size_t count[2] = {0, 0};
  std::vector<std::pair<float, int32_t>> st;
  for (size_t i = 0; i < n; ++i) {
    const float* r = &rec[9 * i];
    const float o[3] = {r[0], r[1], r[2]}, d[3] = {r[4], r[5], r[6]};
    const float tmin = r[3];
    float tmax = r[7];
    const int kind = (int)r[8];
    float inv[3];
    for (int a = 0; a < 3; ++a) inv[a] = 1.0f / (std::fabs(d[a]) > 1e-20f ? d[a] : std::copysign(1e-20f, d[a]));
    st.clear();
    int32_t node = b.root;
    bool done = false;
    count[kind]++;
    while (!done) {
      if (node >= 0) {
        visits[kind] += 1;
        by_depth[kind][std::min<int>(31, depth[node])] += 1;
        for (int k = 0; k < kB; ++k) global[kind][k] += (uint32_t)node >= budgets[k];
        const float* nd = &b.nodes[32 * (size_t)node];
        std::pair<float, int32_t> ch[4];
        int nc = 0;
        for (int c = 0; c < 4; ++c) {
          const int32_t ref = (int32_t)fb(nd[24 + c]);
          if (ref == kEmptyChild) continue;
          float t0 = tmin, t1 = tmax * (1.0f + 0x1p-11f);
          for (int a = 0; a < 3; ++a) {
            const float x0 = (nd[8 * a + c] - o[a]) * inv[a], x1 = (nd[8 * a + 4 + c] - o[a]) * inv[a];
            t0 = std::max(t0, std::min(x0, x1));
            t1 = std::min(t1, std::max(x0, x1));
          }
          if (t0 <= t1) ch[nc++] = {t0, ref};
        }
        std::sort(ch, ch + nc, [](auto& x, auto& y) { return x.first < y.first; });
        for (int c = nc - 1; c >= 1; --c) st.push_back(ch[c]);
        if (nc) { node = ch[0].second; continue; }
      } else {
        leaf_visits[kind] += 1;
        const uint32_t lr = ~(uint32_t)node, first = lr >> kLeafCountBits, cnt = (lr & (kMaxLeafSize - 1)) + 1;
        for (uint32_t k = first; k < first + cnt; ++k) {
          const float* t = &b.tris[12 * (size_t)k];
          const float v0[3] = {t[0], t[1], t[2]}, e1[3] = {t[4], t[5], t[6]}, e2[3] = {t[8], t[9], t[10]};
          const float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
          const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
          if (det == 0.0f) continue;
          const float iv = 1.0f / det;
          const float s[3] = {o[0] - v0[0], o[1] - v0[1], o[2] - v0[2]};
          const float b1 = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * iv;
          if (b1 < 0.0f || b1 > 1.0f) continue;
          const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
          const float b2 = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * iv;
          if (b2 < 0.0f || b1 + b2 > 1.0f) continue;
          const float tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * iv;
          if (tt >= tmin && tt <= tmax) {
            tmax = tt;
            if (kind == 1) { done = true; break; }
          }
        }
        if (done) break;
      }
      node = 0x7FFFFFFF;
      while (!st.empty()) {
        auto e = st.back();
        st.pop_back();
        if (e.first <= tmax * (1.0f + 0x1p-11f)) { node = e.second; break; }
      }
      if (node == 0x7FFFFFFF) done = true;
    }
  }
  std::printf("tree: %u nodes, %u leaves, depth %u\n", b.num_nodes, b.num_leaves, b.max_depth);
  for (int k = 0; k < 2; ++k) {
    const double c = (double)std::max<size_t>(1, count[k]);
    std::printf("%s queries %zu: interior visits %.2f, leaf visits %.2f per query\n", k ? "any-hit" : "nearest", count[k],
                visits[k] / c, leaf_visits[k] / c);
    std::printf("  global interior fetches per query by LDS top:");
    for (int j = 0; j < kB; ++j) std::printf("  B=%u %.2f", budgets[j], global[k][j] / c);
    std::printf("\n  visits by depth:");
    for (int j = 0; j < 16; ++j) std::printf(" %d:%.2f", j, by_depth[k][j] / c);
    std::printf("\n");
  }
  return 0;
}
