// bvh.cpp — binned-SAH BVH2 builder.  See bvh.h.
#include "bvh.h"
#include "diag_env.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <array>
#include <deque>
#include <functional>

namespace mrt {
namespace {

struct Box {
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
  float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  void grow(const float p[3]) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
  }
  bool valid() const { return lo[0] <= hi[0]; }
  float area() const {
    if (!valid()) return 0.0f;
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
  }
};

struct BuildNode {
  Box box;
  int32_t child[2] = {-1, -1};   // build-node ids, -1 for leaves
  uint32_t first = 0, count = 0; // leaf range in `order`
  uint32_t depth = 0;
};

struct Builder {
  const BvhBuildOptions& opt;
  std::vector<Box> prim_box;
  std::vector<float> centroid;      // 3 per prim
  std::vector<uint32_t> order;
  std::vector<BuildNode> nodes;
  uint32_t max_depth = 0;
  std::string err;

  explicit Builder(const BvhBuildOptions& o) : opt(o) {}

  // returns build-node id
  int32_t build(uint32_t first, uint32_t count, uint32_t depth) {
    const int32_t id = (int32_t)nodes.size();
    nodes.emplace_back();
    Box box, cbox;
    for (uint32_t i = first; i < first + count; ++i) {
      box.grow(prim_box[order[i]]);
      cbox.grow(&centroid[3 * order[i]]);
    }
    nodes[id].box = box;
    nodes[id].depth = depth;
    const float leaf_cost = (float)count;
    const bool depth_limited = depth + 1 >= (uint32_t)kMaxBvhDepth;
    if (count <= 1 || (depth_limited && count <= (uint32_t)kMaxLeafSize)) {
      make_leaf(id, first, count, depth);
      return id;
    }
    if (depth_limited) { err = "BVH depth limit reached with an oversize leaf"; make_leaf(id, first, count, depth); return id; }

    // binned SAH over the centroid bounds
    const uint32_t B = std::max<uint32_t>(4, opt.bins);
    int best_axis = -1;
    uint32_t best_split = 0;
    float best_cost = FLT_MAX;
    std::vector<Box> bin_box(B);
    std::vector<uint32_t> bin_cnt(B);
    std::vector<float> right_area(B);
    std::vector<uint32_t> right_cnt(B);
    for (int axis = 0; axis < 3; ++axis) {
      const float ext = cbox.hi[axis] - cbox.lo[axis];
      if (!(ext > 0.0f)) continue;
      const float scale = (float)B / ext;
      std::fill(bin_box.begin(), bin_box.end(), Box());
      std::fill(bin_cnt.begin(), bin_cnt.end(), 0u);
      for (uint32_t i = first; i < first + count; ++i) {
        const uint32_t p = order[i];
        uint32_t b = (uint32_t)((centroid[3 * p + axis] - cbox.lo[axis]) * scale);
        b = std::min(b, B - 1);
        bin_box[b].grow(prim_box[p]);
        bin_cnt[b]++;
      }
      Box acc;
      uint32_t cnt = 0;
      for (uint32_t b = B - 1; b > 0; --b) {
        acc.grow(bin_box[b]);
        cnt += bin_cnt[b];
        right_area[b] = acc.area();
        right_cnt[b] = cnt;
      }
      acc = Box();
      cnt = 0;
      for (uint32_t b = 0; b + 1 < B; ++b) {
        acc.grow(bin_box[b]);
        cnt += bin_cnt[b];
        const uint32_t rc = right_cnt[b + 1];
        if (cnt == 0 || rc == 0) continue;
        const float cost = acc.area() * (float)cnt + right_area[b + 1] * (float)rc;
        if (cost < best_cost) { best_cost = cost; best_axis = axis; best_split = b + 1; }
      }
    }
    // small ranges: exact SAH over every centroid-sorted split (the binned
    // estimate is coarse when a node holds a few dozen triangles)
    bool exact = false;
    std::vector<uint32_t> exact_order;
    if (count <= opt.exact_sah_below) {
      std::vector<uint32_t> idx(order.begin() + first, order.begin() + first + count);
      std::vector<float> racc(count);
      for (int axis = 0; axis < 3; ++axis) {
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
          return centroid[3 * a + axis] < centroid[3 * b + axis];
        });
        Box acc;
        for (uint32_t k = count; k-- > 1;) { acc.grow(prim_box[idx[k]]); racc[k] = acc.area(); }
        acc = Box();
        for (uint32_t k = 0; k + 1 < count; ++k) {
          acc.grow(prim_box[idx[k]]);
          const float cost = acc.area() * (float)(k + 1) + racc[k + 1] * (float)(count - k - 1);
          if (cost < best_cost) {
            best_cost = cost;
            best_axis = axis;
            best_split = k + 1;
            exact = true;
            exact_order = idx;
          }
        }
      }
    }
    const float parent_area = box.area();
    const float split_cost = parent_area > 0.0f ? opt.traversal_cost + best_cost / parent_area : FLT_MAX;
    uint32_t mid;
    if (exact) {
      if (count <= opt.max_leaf_size && leaf_cost <= split_cost) { make_leaf(id, first, count, depth); return id; }
      std::copy(exact_order.begin(), exact_order.end(), order.begin() + first);
      mid = first + best_split;
    } else if (best_axis < 0) {
      // all centroids coincide: leaf if it fits, else split the range in half
      if (count <= opt.max_leaf_size) { make_leaf(id, first, count, depth); return id; }
      mid = first + count / 2;
    } else {
      if (count <= opt.max_leaf_size && leaf_cost <= split_cost) { make_leaf(id, first, count, depth); return id; }
      const float scale = (float)B / (cbox.hi[best_axis] - cbox.lo[best_axis]);
      const float lo = cbox.lo[best_axis];
      auto it = std::partition(order.begin() + first, order.begin() + first + count, [&](uint32_t p) {
        uint32_t b = (uint32_t)((centroid[3 * p + best_axis] - lo) * scale);
        return std::min(b, B - 1) < best_split;
      });
      mid = (uint32_t)(it - order.begin());
      if (mid == first || mid == first + count) mid = first + count / 2;
    }
    const int32_t l = build(first, mid - first, depth + 1);
    const int32_t r = build(mid, first + count - mid, depth + 1);
    nodes[id].child[0] = l;
    nodes[id].child[1] = r;
    return id;
  }

  // ---- full sweep SAH (opt.full_sweep): every node takes the exact best
  // split over its centroid-sorted triangles on all three axes.  The node's
  // triangles are kept sorted per axis in srt[0..2] over the same range
  // [first, first + count) (one initial sort, ties by index); a split on axis
  // a at k keeps srt[a] as is and stably partitions the other two by side, so
  // the whole build is O(n log n) after the sort.  Leaves read srt[0]
  // (copied to `order` at the end).
  std::vector<uint32_t> srt[3], tmp;
  std::vector<uint8_t> side;
  std::vector<float> racc;

  void init_full(uint32_t n) {
    for (int a = 0; a < 3; ++a) {
      srt[a].resize(n);
      for (uint32_t i = 0; i < n; ++i) srt[a][i] = i;
      std::sort(srt[a].begin(), srt[a].end(), [&](uint32_t x, uint32_t y) {
        const float cx = centroid[3 * x + a], cy = centroid[3 * y + a];
        return cx < cy || (cx == cy && x < y);
      });
    }
    tmp.resize(n);
    side.resize(n);
    racc.resize(n);
  }

  void split_full(uint32_t first, uint32_t count, int axis, uint32_t k) {
    for (uint32_t i = 0; i < count; ++i) side[srt[axis][first + i]] = i < k ? 0 : 1;
    for (int a = 0; a < 3; ++a) {
      if (a == axis) continue;
      uint32_t* s = &srt[a][first];
      uint32_t nl = 0, nr = 0;
      for (uint32_t i = 0; i < count; ++i) {
        if (side[s[i]] == 0) s[nl++] = s[i];
        else tmp[nr++] = s[i];
      }
      std::copy(tmp.begin(), tmp.begin() + nr, s + nl);
    }
  }

  int32_t build_full(uint32_t first, uint32_t count, uint32_t depth) {
    const int32_t id = (int32_t)nodes.size();
    nodes.emplace_back();
    Box box;
    for (uint32_t i = first; i < first + count; ++i) box.grow(prim_box[srt[0][i]]);
    nodes[id].box = box;
    nodes[id].depth = depth;
    const bool depth_limited = depth + 1 >= (uint32_t)kMaxBvhDepth;
    if (count <= 1 || (depth_limited && count <= (uint32_t)kMaxLeafSize)) return leaf_full(id, first, count, depth);
    int best_axis = -1;
    uint32_t best_k = 0;
    float best_cost = FLT_MAX;
    for (int axis = 0; axis < 3; ++axis) {
      const uint32_t* s = &srt[axis][first];
      Box acc;
      for (uint32_t k = count; k-- > 1;) { acc.grow(prim_box[s[k]]); racc[k] = acc.area(); }
      acc = Box();
      for (uint32_t k = 0; k + 1 < count; ++k) {
        acc.grow(prim_box[s[k]]);
        const float cost = acc.area() * (float)(k + 1) + racc[k + 1] * (float)(count - k - 1);
        if (cost < best_cost) { best_cost = cost; best_axis = axis; best_k = k + 1; }
      }
    }
    const float parent_area = box.area();
    const float split_cost = parent_area > 0.0f ? opt.traversal_cost + best_cost / parent_area : FLT_MAX;
    if (count <= opt.max_leaf_size && (float)count <= split_cost) return leaf_full(id, first, count, depth);
    if (depth_limited) err = "BVH depth limit reached with an oversize leaf";
    if (best_axis < 0 || depth_limited) { best_axis = 0; best_k = count / 2; }
    split_full(first, count, best_axis, best_k);
    const int32_t l = build_full(first, best_k, depth + 1);
    const int32_t r = build_full(first + best_k, count - best_k, depth + 1);
    nodes[id].child[0] = l;
    nodes[id].child[1] = r;
    return id;
  }

  int32_t leaf_full(int32_t id, uint32_t first, uint32_t count, uint32_t depth) {
    nodes[id].first = first;
    nodes[id].count = count;
    max_depth = std::max(max_depth, depth);
    return id;
  }

  void make_leaf(int32_t id, uint32_t first, uint32_t count, uint32_t depth) {
    // leaves hold at most kMaxLeafSize triangles; larger ranges become a
    // small subtree of full leaves (only reachable when centroids coincide)
    if (count > (uint32_t)kMaxLeafSize) {
      const uint32_t mid = first + count / 2;
      const int32_t l = build(first, mid - first, depth + 1);
      const int32_t r = build(mid, first + count - mid, depth + 1);
      nodes[id].child[0] = l;
      nodes[id].child[1] = r;
      return;
    }
    nodes[id].first = first;
    nodes[id].count = count;
    max_depth = std::max(max_depth, depth);
  }
};

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float bitsf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// the slab-test box of a node: padded outward so the test is conservative
// under rounding (both kernel builds), see bvh.h
inline void padded_box(const Box& bx, float lo[3], float hi[3]) {
  for (int k = 0; k < 3; ++k) {
    const float m = std::max(std::fabs(bx.lo[k]), std::fabs(bx.hi[k]));
    const float pad = 1e-5f * m + 1e-6f;
    lo[k] = bx.lo[k] - pad;
    hi[k] = bx.hi[k] + pad;
  }
}

}  // namespace

bool build_bvh(const float* positions, size_t stride_bytes, const uint32_t* indices, uint32_t num_triangles,
               const BvhBuildOptions& opt, BvhResult& out, std::string& error) {
  if (num_triangles == 0) { error = "empty scene"; return false; }
  if (opt.width != 2 && opt.width != 4) { error = "BVH width must be 2 or 4"; return false; }
  if (opt.max_leaf_size == 0 || opt.max_leaf_size > (uint32_t)kMaxLeafSize) { error = "bad leaf size"; return false; }
  if (num_triangles >= (1u << (31 - kLeafCountBits))) { error = "too many triangles"; return false; }
  Builder b(opt);
  const size_t stride = stride_bytes / sizeof(float);
  auto P = [&](uint32_t vi) { return positions + (size_t)vi * stride; };
  b.prim_box.resize(num_triangles);
  b.centroid.resize(3 * (size_t)num_triangles);
  b.order.resize(num_triangles);
  for (uint32_t t = 0; t < num_triangles; ++t) {
    Box bx;
    for (int k = 0; k < 3; ++k) bx.grow(P(indices[3 * t + k]));
    b.prim_box[t] = bx;
    for (int k = 0; k < 3; ++k) b.centroid[3 * t + k] = 0.5f * (bx.lo[k] + bx.hi[k]);
    b.order[t] = t;
  }
  b.nodes.reserve(2 * (size_t)num_triangles / std::max<uint32_t>(1, opt.max_leaf_size) + 16);
  if (opt.full_sweep) {
    b.init_full(num_triangles);
    b.build_full(0, num_triangles, 0);
    b.order = b.srt[0];
  } else {
    b.build(0, num_triangles, 0);
  }
  if (!b.err.empty()) { error = b.err; return false; }
  // ---- collapse to the output width ----------------------------------------
  // Greedy: a wide node's children are found by repeatedly opening the
  // largest-area interior child of the binary node (width 2 is the identity).
  // DP (opt.collapse_dp, width 4): the binary leaves stay leaves, so the
  // collapse only chooses which binary interior nodes become wide nodes; the
  // SAH's expected node visits are the summed area of those.  best[m][k] =
  // least summed area covering m's subtree with at most k + 1 child slots
  // (m itself as one slot: area(m) + its own best 4-slot split), computed
  // bottom-up (children have larger build ids than their parent).
  const std::vector<BuildNode>& bn = b.nodes;
  const uint32_t W = opt.width;
  auto is_leaf = [&](int32_t id) { return bn[id].child[0] < 0; };
  bool dp = opt.collapse_dp > 0 || (opt.collapse_dp < 0 && num_triangles < kGreedyCollapseTriangles);
  if (opt.collapse_dp < 0)
    if (const char* v = mrt::diag_env("MRT_COLLAPSE")) dp = std::atoi(v) != 0;   // 0: greedy, 1: DP
  dp = dp && W == 4;
  std::vector<std::array<float, 4>> best;
  std::vector<std::array<uint8_t, 4>> pick;   // k1 of the split (0: m is one slot)
  std::vector<uint8_t> inner;                 // m as a wide node: k1 of its children's slots (k2 = 4 - k1 at most)
  std::vector<uint8_t> inner2;
  if (dp) {
    best.assign(bn.size(), {0.0f, 0.0f, 0.0f, 0.0f});
    pick.assign(bn.size(), {0, 0, 0, 0});
    inner.assign(bn.size(), 1);
    inner2.assign(bn.size(), 1);
    for (size_t i = bn.size(); i-- > 0;) {
      if (is_leaf((int32_t)i)) continue;   // a leaf costs nothing here, in any number of slots
      const int32_t l = bn[i].child[0], r = bn[i].child[1];
      float in = FLT_MAX;
      for (uint32_t k1 = 1; k1 <= 3; ++k1)
        for (uint32_t k2 = 1; k1 + k2 <= 4; ++k2) {
          const float c = best[l][k1 - 1] + best[r][k2 - 1];
          if (c < in) { in = c; inner[i] = (uint8_t)k1; inner2[i] = (uint8_t)k2; }
        }
      best[i][0] = bn[i].box.area() + in;
      pick[i][0] = 0;
      for (uint32_t k = 1; k < 4; ++k) {   // at most k + 1 slots
        best[i][k] = best[i][k - 1];
        pick[i][k] = pick[i][k - 1];
        for (uint32_t k1 = 1; k1 <= k; ++k1) {
          const uint32_t k2 = k + 1 - k1;
          const float c = best[l][k1 - 1] + best[r][k2 - 1];
          if (c < best[i][k]) { best[i][k] = c; pick[i][k] = (uint8_t)k1; }
        }
      }
    }
  }
  // the children of wide node `id` under the DP choice
  std::function<void(int32_t, uint32_t, int32_t*, uint32_t&)> expand = [&](int32_t m, uint32_t k, int32_t* ch,
                                                                             uint32_t& n) {
    if (is_leaf(m) || pick[m][k - 1] == 0) { ch[n++] = m; return; }
    const uint32_t k1 = pick[m][k - 1];
    expand(bn[m].child[0], k1, ch, n);
    expand(bn[m].child[1], k - k1, ch, n);
  };
  auto collapse = [&](int32_t id, int32_t ch[4]) {
    uint32_t n = 2;
    if (dp) {
      n = 0;
      expand(bn[id].child[0], inner[id], ch, n);
      expand(bn[id].child[1], inner2[id], ch, n);
      return n;
    }
    ch[0] = bn[id].child[0];
    ch[1] = bn[id].child[1];
    while (n < W) {
      int best = -1;
      float best_area = -1.0f;
      for (uint32_t i = 0; i < n; ++i)
        if (!is_leaf(ch[i]) && bn[ch[i]].box.area() > best_area) { best = (int)i; best_area = bn[ch[i]].box.area(); }
      if (best < 0) break;
      const int32_t c = ch[best];
      ch[best] = bn[c].child[0];
      ch[n++] = bn[c].child[1];
    }
    return n;
  };

  // ---- layout: BFS for the top interior nodes, DFS below -----------------
  std::vector<int32_t> out_index(bn.size(), -1);
  std::vector<int32_t> emit_order;   // build ids of (wide) interior nodes in output order
  std::vector<std::array<int32_t, 4>> wide_children;
  std::vector<uint32_t> wide_count;
  std::vector<uint32_t> stack_need;  // traversal stack entries pending when the node is entered
  auto visit = [&](int32_t id) {
    out_index[id] = (int32_t)emit_order.size();
    emit_order.push_back(id);
    std::array<int32_t, 4> ch{-1, -1, -1, -1};
    wide_count.push_back(collapse(id, ch.data()));
    wide_children.push_back(ch);
  };
  if (!is_leaf(0)) {
    std::deque<int32_t> q{0};
    while (!q.empty() && emit_order.size() < opt.lds_node_budget) {
      const int32_t id = q.front();
      q.pop_front();
      visit(id);
      const auto& ch = wide_children.back();
      for (uint32_t c = 0; c < wide_count.back(); ++c)
        if (!is_leaf(ch[c])) q.push_back(ch[c]);
    }
    out.lds_nodes = (uint32_t)emit_order.size();
    // remaining frontier subtrees in DFS order
    std::vector<int32_t> stack;
    for (int32_t root_id : q) {
      stack.push_back(root_id);
      while (!stack.empty()) {
        const int32_t id = stack.back();
        stack.pop_back();
        visit(id);
        const auto ch = wide_children.back();
        for (int c = (int)wide_count.back() - 1; c >= 0; --c)
          if (!is_leaf(ch[c])) stack.push_back(ch[c]);
      }
    }
    // stack bound: entries pushed at the ancestors (all children but the one
    // descended into) — parents are emitted before their children
    stack_need.assign(emit_order.size(), 0);
    uint32_t wide_depth_max = 0;
    std::vector<uint32_t> wide_depth(emit_order.size(), 0);
    for (size_t k = 0; k < emit_order.size(); ++k) {
      const uint32_t below = stack_need[k] + (wide_count[k] - 1);
      out.max_stack = std::max(out.max_stack, below);
      wide_depth_max = std::max(wide_depth_max, wide_depth[k] + 1);
      for (uint32_t c = 0; c < wide_count[k]; ++c) {
        const int32_t cid = wide_children[k][c];
        if (is_leaf(cid)) continue;
        stack_need[out_index[cid]] = below;
        wide_depth[out_index[cid]] = wide_depth[k] + 1;
      }
    }
    out.wide_depth = wide_depth_max;
  }
  // leaf triangle runs in output order of their parents (DFS-ish locality)
  std::vector<int32_t> leaf_ref_of(bn.size(), 0);
  uint32_t tri_cursor = 0;
  out.tris.assign(12 * (size_t)num_triangles, 0.0f);
  auto emit_leaf = [&](int32_t id) {
    const BuildNode& n = bn[id];
    for (uint32_t i = 0; i < n.count; ++i) {
      const uint32_t prim = b.order[n.first + i];
      const float* v0 = P(indices[3 * prim]);
      const float* v1 = P(indices[3 * prim + 1]);
      const float* v2 = P(indices[3 * prim + 2]);
      float* o = &out.tris[12 * (size_t)(tri_cursor + i)];
      o[0] = v0[0]; o[1] = v0[1]; o[2] = v0[2]; o[3] = bitsf(prim);
      o[4] = v1[0] - v0[0]; o[5] = v1[1] - v0[1]; o[6] = v1[2] - v0[2]; o[7] = 0.0f;
      o[8] = v2[0] - v0[0]; o[9] = v2[1] - v0[1]; o[10] = v2[2] - v0[2]; o[11] = 0.0f;
    }
    leaf_ref_of[id] = leaf_ref(tri_cursor, n.count);
    tri_cursor += n.count;
    out.num_leaves++;
  };
  if (is_leaf(0)) {
    emit_leaf(0);
    out.root = leaf_ref_of[0];
  } else {
    for (size_t k = 0; k < emit_order.size(); ++k)
      for (uint32_t c = 0; c < wide_count[k]; ++c)
        if (is_leaf(wide_children[k][c])) emit_leaf(wide_children[k][c]);
    out.root = 0;
  }
  out.width = W;
  out.num_nodes = (uint32_t)emit_order.size();
  const size_t node_floats = W == 4 ? 32 : 16;
  out.nodes.assign(node_floats * (size_t)std::max<uint32_t>(1, out.num_nodes), 0.0f);
  auto padded = [](const Box& bx, float lo[3], float hi[3]) {
    for (int k = 0; k < 3; ++k) {
      const float m = std::max(std::fabs(bx.lo[k]), std::fabs(bx.hi[k]));
      const float pad = 1e-5f * m + 1e-6f;
      lo[k] = bx.lo[k] - pad;
      hi[k] = bx.hi[k] + pad;
    }
  };
  auto child_ref = [&](int32_t cid) { return is_leaf(cid) ? leaf_ref_of[cid] : out_index[cid]; };
  double sah = 0.0;
  const double root_area = std::max(1e-30, (double)bn[0].box.area());
  for (size_t k = 0; k < emit_order.size(); ++k) {
    const BuildNode& n = bn[emit_order[k]];
    float* o = &out.nodes[node_floats * k];
    sah += opt.traversal_cost * n.box.area() / root_area;
    for (uint32_t c = 0; c < wide_count[k]; ++c) {
      const BuildNode& C = bn[wide_children[k][c]];
      if (is_leaf(wide_children[k][c])) sah += (double)C.count * C.box.area() / root_area;
    }
    if (W == 2) {
      float l_lo[3], l_hi[3], r_lo[3], r_hi[3];
      padded(bn[wide_children[k][0]].box, l_lo, l_hi);
      padded(bn[wide_children[k][1]].box, r_lo, r_hi);
      o[0] = l_lo[0]; o[1] = l_hi[0]; o[2] = l_lo[1]; o[3] = l_hi[1];
      o[4] = r_lo[0]; o[5] = r_hi[0]; o[6] = r_lo[1]; o[7] = r_hi[1];
      o[8] = l_lo[2]; o[9] = l_hi[2]; o[10] = r_lo[2]; o[11] = r_hi[2];
      o[12] = bitsf((uint32_t)child_ref(wide_children[k][0]));
      o[13] = bitsf((uint32_t)child_ref(wide_children[k][1]));
    } else {
      // BVH4: component-major (SoA within the node), see mrt_layout.h
      for (uint32_t c = 0; c < 4; ++c) {
        if (c < wide_count[k]) {
          float lo[3], hi[3];
          padded(bn[wide_children[k][c]].box, lo, hi);
          for (int a = 0; a < 3; ++a) { o[8 * a + c] = lo[a]; o[8 * a + 4 + c] = hi[a]; }
          o[24 + c] = bitsf((uint32_t)child_ref(wide_children[k][c]));
        } else {
          // an inverted box: no ray order's slab test hits it (kernels.hip box4)
          for (int a = 0; a < 3; ++a) { o[8 * a + c] = INFINITY; o[8 * a + 4 + c] = -INFINITY; }
          o[24 + c] = bitsf((uint32_t)kEmptyChild);
        }
      }
    }
  }
  if (is_leaf(0)) out.wide_depth = 0;
  (void)fbits;
  out.sah_cost = sah;
  out.max_depth = b.max_depth;
  if (tri_cursor != num_triangles) { error = "internal: leaf triangle count mismatch"; return false; }
  return true;
}

}  // namespace mrt
