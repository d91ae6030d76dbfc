// bvh_gpu.hip — device-side LBVH build into the BVH4 layout (see bvh_gpu.h).
// Replaces MPSTriangleAccelerationStructure.rebuild (renderer/Renderer.mm:456-462).
#include "bvh_gpu.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "bvh.h"
#include "mrt_layout.h"

namespace mrt {
namespace {

constexpr int kB = 256;

// order-preserving float <-> uint mapping for atomicMin/atomicMax on floats
__device__ __forceinline__ uint32_t f2o(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

struct Tri3 { float3 a, b, c; };
__device__ __forceinline__ Tri3 load_tri(const uint8_t* pos, uint32_t stride, const uint32_t* idx, uint32_t t) {
  Tri3 r;
  float3* v[3] = {&r.a, &r.b, &r.c};
  for (int k = 0; k < 3; ++k) {
    const float* p = reinterpret_cast<const float*>(pos + (size_t)idx[3 * (size_t)t + k] * stride);
    *v[k] = make_float3(p[0], p[1], p[2]);
  }
  return r;
}
__device__ __forceinline__ float3 centroid(const Tri3& t) {
  return make_float3((t.a.x + t.b.x + t.c.x) * (1.0f / 3.0f), (t.a.y + t.b.y + t.c.y) * (1.0f / 3.0f),
                     (t.a.z + t.b.z + t.c.z) * (1.0f / 3.0f));
}

// scene centroid bounds: bounds[0..2] = ordered min, [3..5] = ordered max
__global__ __launch_bounds__(kB) void k_centroid_bounds(const uint8_t* pos, uint32_t stride, const uint32_t* idx,
                                                        uint32_t T, uint32_t* bounds) {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (uint32_t t = blockIdx.x * kB + threadIdx.x; t < T; t += gridDim.x * kB) {
    const float3 c = centroid(load_tri(pos, stride, idx, t));
    lo[0] = fminf(lo[0], c.x); lo[1] = fminf(lo[1], c.y); lo[2] = fminf(lo[2], c.z);
    hi[0] = fmaxf(hi[0], c.x); hi[1] = fmaxf(hi[1], c.y); hi[2] = fmaxf(hi[2], c.z);
  }
  for (int k = 0; k < 3; ++k) {
    for (int off = 32; off > 0; off >>= 1) {
      lo[k] = fminf(lo[k], __shfl_xor(lo[k], off));
      hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off));
    }
  }
  if ((threadIdx.x & 63u) == 0) {
    for (int k = 0; k < 3; ++k) {
      atomicMin(&bounds[k], f2o(lo[k]));
      atomicMax(&bounds[3 + k], f2o(hi[k]));
    }
  }
}

__device__ __forceinline__ uint64_t split3(uint32_t a) {   // 21 bits -> every third bit of 63
  uint64_t x = a & 0x1FFFFFu;
  x = (x | x << 32) & 0x1F00000000FFFFull;
  x = (x | x << 16) & 0x1F0000FF0000FFull;
  x = (x | x << 8) & 0x100F00F00F00F00Full;
  x = (x | x << 4) & 0x10C30C30C30C30C3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

// 63-bit Morton code of the centroid (21 bits per axis) + triangle index
__global__ __launch_bounds__(kB) void k_morton(const uint8_t* pos, uint32_t stride, const uint32_t* idx, uint32_t T,
                                               const uint32_t* bounds, uint64_t* keys, uint32_t* vals) {
  const uint32_t t = blockIdx.x * kB + threadIdx.x;
  if (t >= T) return;
  const float3 c = centroid(load_tri(pos, stride, idx, t));
  const float cc[3] = {c.x, c.y, c.z};
  uint32_t q[3];
  for (int k = 0; k < 3; ++k) {
    const float lo = o2f(bounds[k]), hi = o2f(bounds[3 + k]);
    const float ext = hi - lo;
    const float u = ext > 0.0f ? (cc[k] - lo) / ext : 0.0f;
    q[k] = (uint32_t)fminf(fmaxf(u * 2097152.0f, 0.0f), 2097151.0f);
  }
  keys[t] = (split3(q[0]) << 2) | (split3(q[1]) << 1) | split3(q[2]);
  vals[t] = t;
}

// Binary radix tree over the sorted keys (Karras 2012): one thread per
// internal node i in [0, T-2].  child refs: >= 0 internal, < 0 leaf ~p
// (p = sorted position).  Equal codes are told apart by their sorted
// position (the augmented common prefix of Karras §4).
__device__ __forceinline__ int delta(const uint64_t* k, int n, int a, int b) {
  if (b < 0 || b >= n) return -1;
  const uint64_t x = k[a] ^ k[b];
  return x ? __clzll(x) : 64 + __clz((uint32_t)(a ^ b));
}
__global__ __launch_bounds__(kB) void k_radix_tree(const uint64_t* keys, int n, int32_t* child, int32_t* parent_int,
                                                   int32_t* parent_leaf, uint32_t* rfirst, uint32_t* rcount) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n - 1) return;
  const int d = delta(keys, n, i, i + 1) > delta(keys, n, i, i - 1) ? 1 : -1;
  const int dmin = delta(keys, n, i, i - d);
  int lmax = 2;
  while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(keys, n, i, j);
  int s = 0, t = l;
  do {
    t = (t + 1) >> 1;
    if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
  } while (t > 1);
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  if (first == gamma) { child[2 * i] = ~gamma; parent_leaf[gamma] = i; }
  else { child[2 * i] = gamma; parent_int[gamma] = i; }
  if (last == gamma + 1) { child[2 * i + 1] = ~(gamma + 1); parent_leaf[gamma + 1] = i; }
  else { child[2 * i + 1] = gamma + 1; parent_int[gamma + 1] = i; }
  rfirst[i] = (uint32_t)first;
  rcount[i] = (uint32_t)(last - first + 1);
  if (i == 0) parent_int[0] = -1;
}

// Leaf records + bottom-up boxes.  Thread p owns sorted triangle p: writes
// its leaf-ordered triangle {v0|prim, e1, e2} and box, then climbs; the
// second thread to reach an internal node (arrival counter) computes its
// box from both children.  Release/acquire at agent scope around the
// counter makes the sibling's box visible across XCDs.
__global__ __launch_bounds__(kB) void k_leaves_refit(const uint8_t* pos, uint32_t stride, const uint32_t* idx,
                                                     const uint32_t* order, uint32_t T, const int32_t* child,
                                                     const int32_t* parent_int, const int32_t* parent_leaf,
                                                     float4* tris, float4* leaf_box, float4* node_box,
                                                     uint32_t* arrivals, bool climb) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= T) return;
  const uint32_t t = order[p];
  const Tri3 v = load_tri(pos, stride, idx, t);
  tris[3 * (size_t)p + 0] = make_float4(v.a.x, v.a.y, v.a.z, __uint_as_float(t));
  tris[3 * (size_t)p + 1] = make_float4(v.b.x - v.a.x, v.b.y - v.a.y, v.b.z - v.a.z, 0.0f);
  tris[3 * (size_t)p + 2] = make_float4(v.c.x - v.a.x, v.c.y - v.a.y, v.c.z - v.a.z, 0.0f);
  float4 lo = make_float4(fminf(fminf(v.a.x, v.b.x), v.c.x), fminf(fminf(v.a.y, v.b.y), v.c.y),
                          fminf(fminf(v.a.z, v.b.z), v.c.z), 0.0f);
  float4 hi = make_float4(fmaxf(fmaxf(v.a.x, v.b.x), v.c.x), fmaxf(fmaxf(v.a.y, v.b.y), v.c.y),
                          fmaxf(fmaxf(v.a.z, v.b.z), v.c.z), 0.0f);
  leaf_box[2 * (size_t)p] = lo;
  leaf_box[2 * (size_t)p + 1] = hi;
  if (!climb) return;
  int32_t node = parent_leaf[p];
  while (node >= 0) {
    __threadfence();   // release this thread's box writes
    if (atomicAdd(&arrivals[node], 1u) == 0u) return;   // first arrival: the sibling finishes the node
    __threadfence();   // acquire the sibling's box
    for (int c = 0; c < 2; ++c) {
      const int32_t ch = child[2 * node + c];
      const float4* b = ch >= 0 ? node_box + 2 * (size_t)ch : leaf_box + 2 * (size_t)(~ch);
      const float4 blo = b[0], bhi = b[1];
      lo = make_float4(fminf(lo.x, blo.x), fminf(lo.y, blo.y), fminf(lo.z, blo.z), 0.0f);
      hi = make_float4(fmaxf(hi.x, bhi.x), fmaxf(hi.y, bhi.y), fmaxf(hi.z, bhi.z), 0.0f);
    }
    node_box[2 * (size_t)node] = lo;
    node_box[2 * (size_t)node + 1] = hi;
    node = parent_int[node];
  }
}

__device__ __forceinline__ int32_t dev_leaf_ref(uint32_t first, uint32_t count) {   // bvh.h leaf_ref
  return (int32_t)~((first << kLeafCountBits) | (count - 1));
}
__device__ __forceinline__ float box_area(float4 lo, float4 hi) {
  const float x = hi.x - lo.x, y = hi.y - lo.y, z = hi.z - lo.z;
  return 2.0f * (x * y + y * z + z * x);
}
__device__ __forceinline__ float pad_of(float a, float b) {   // same outward padding as the host builder
  const float m = fmaxf(fabsf(a), fabsf(b));
  return __fadd_rn(__fmul_rn(1e-5f, m), 1e-6f);
}

struct LevelArgs {
  const int32_t* child;
  const uint32_t* rfirst;
  const uint32_t* rcount;
  const float4* leaf_box;
  const float4* node_box;
  const int32_t* in_node;     // binary internal node of each frontier slot
  const uint32_t* in_need;    // stack entries on the way down to it
  uint32_t in_count;
  uint32_t base;              // output index of frontier slot 0
  uint32_t next_base;         // output index of next-frontier slot 0
  int32_t* out_node;
  uint32_t* out_need;
  uint32_t* out_count;
  uint32_t* stats;            // [0] leaves, [1] max stack
  uint32_t max_leaf;
  float* nodes;               // BVH4 records, 32 floats each
};

// One BVH4 node per frontier slot: open the largest-area interior child until
// four children (or none left to open), emit the node, append interior
// children to the next level.
__global__ __launch_bounds__(kB) void k_collapse_level(LevelArgs a) {
  const uint32_t slot = blockIdx.x * kB + threadIdx.x;
  if (slot >= a.in_count) return;
  const int32_t b = a.in_node[slot];
  const uint32_t need = a.in_need[slot];
  auto count_of = [&](int32_t c) -> uint32_t { return c >= 0 ? a.rcount[c] : 1u; };
  int32_t ch[4] = {a.child[2 * b], a.child[2 * b + 1], 0, 0};
  int n = 2;
  while (n < 4) {
    int best = -1;
    float best_area = -1.0f;
    for (int c = 0; c < n; ++c) {
      if (ch[c] >= 0 && count_of(ch[c]) > a.max_leaf) {
        const float ar = box_area(a.node_box[2 * (size_t)ch[c]], a.node_box[2 * (size_t)ch[c] + 1]);
        if (ar > best_area) { best_area = ar; best = c; }
      }
    }
    if (best < 0) break;
    const int32_t x = ch[best];
    ch[best] = a.child[2 * x];
    ch[n++] = a.child[2 * x + 1];
  }
  float* o = a.nodes + 32 * (size_t)(a.base + slot);
  const uint32_t child_need = need + (uint32_t)n - 1u;
  atomicMax(&a.stats[1], child_need);
  for (int c = 0; c < 4; ++c) {
    if (c >= n) {
      for (int k = 0; k < 3; ++k) { o[8 * k + c] = 0.0f; o[8 * k + 4 + c] = 0.0f; }
      o[24 + c] = __uint_as_float((uint32_t)kEmptyChild);
      continue;
    }
    const int32_t x = ch[c];
    const float4* bx = x >= 0 ? a.node_box + 2 * (size_t)x : a.leaf_box + 2 * (size_t)(~x);
    const float4 lo = bx[0], hi = bx[1];
    const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
    for (int k = 0; k < 3; ++k) {
      const float pd = pad_of(l3[k], h3[k]);
      o[8 * k + c] = __fsub_rn(l3[k], pd);
      o[8 * k + 4 + c] = __fadd_rn(h3[k], pd);
    }
    int32_t ref;
    if (x < 0) {
      ref = dev_leaf_ref((uint32_t)(~x), 1u);
      atomicAdd(&a.stats[0], 1u);
    } else if (a.rcount[x] <= a.max_leaf) {
      ref = dev_leaf_ref(a.rfirst[x], a.rcount[x]);
      atomicAdd(&a.stats[0], 1u);
    } else {
      const uint32_t s = atomicAdd(a.out_count, 1u);
      a.out_node[s] = x;
      a.out_need[s] = child_need;
      ref = (int32_t)(a.next_base + s);
    }
    o[24 + c] = __uint_as_float((uint32_t)ref);
  }
  for (int k = 28; k < 32; ++k) o[k] = 0.0f;
}

struct Tmp {
  void* p = nullptr;
  ~Tmp() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 16)); }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

#define GB_TRY(x)                                                   \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      error = std::string(#x) + ": " + hipGetErrorString(e_);       \
      return e_;                                                    \
    }                                                               \
  } while (0)

}  // namespace

hipError_t build_bvh_gpu(const float* positions, uint32_t stride_bytes, const uint32_t* indices,
                         uint32_t T, uint32_t max_leaf, hipStream_t s, GpuBvhResult& out, std::string& error) {
  out = GpuBvhResult{};
  max_leaf = std::max<uint32_t>(1, std::min<uint32_t>(max_leaf ? max_leaf : 4, (uint32_t)kMaxLeafSize));
  if (T >= (1u << (32 - kLeafCountBits - 1))) { error = "too many triangles for the leaf encoding"; return hipErrorInvalidValue; }
  hipEvent_t e0, e1;
  GB_TRY(hipEventCreate(&e0));
  GB_TRY(hipEventCreate(&e1));
  GB_TRY(hipEventRecord(e0, s));
  const uint8_t* pos = reinterpret_cast<const uint8_t*>(positions);
  const uint32_t blocks = (std::max<uint32_t>(T, 1) + kB - 1) / kB;

  // leaf-ordered triangles (kept)
  GB_TRY(hipMalloc(&out.tris, std::max<size_t>(16, (size_t)T * 48)));
  out.tris_bytes = (size_t)T * 48;
  if (T <= max_leaf) {
    // tiny scene: one node whose single child is the leaf of every triangle
    // (or no child at all for an empty scene)
    Tmp order, lbox;
    GB_TRY(order.alloc((size_t)T * 4));
    GB_TRY(lbox.alloc((size_t)T * 32));
    std::vector<uint32_t> ho(T);
    for (uint32_t t = 0; t < T; ++t) ho[t] = t;
    if (T) GB_TRY(hipMemcpyAsync(order.p, ho.data(), (size_t)T * 4, hipMemcpyHostToDevice, s));
    if (T) k_leaves_refit<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, order.as<uint32_t>(), T, nullptr, nullptr,
                                                nullptr, reinterpret_cast<float4*>(out.tris), lbox.as<float4>(),
                                                nullptr, nullptr, false);
    GB_TRY(hipGetLastError());
    std::vector<float> lb((size_t)T * 8);
    if (T) GB_TRY(hipMemcpyAsync(lb.data(), lbox.p, (size_t)T * 32, hipMemcpyDeviceToHost, s));
    GB_TRY(hipStreamSynchronize(s));
    std::vector<float> node(32, 0.0f);
    for (int c = 0; c < 4; ++c) {
      uint32_t ref = (uint32_t)kEmptyChild;
      std::memcpy(&node[24 + c], &ref, 4);
    }
    if (T) {
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (uint32_t t = 0; t < T; ++t)
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], lb[8 * t + k]); hi[k] = std::max(hi[k], lb[8 * t + 4 + k]); }
      for (int k = 0; k < 3; ++k) {
        const float m = std::max(std::fabs(lo[k]), std::fabs(hi[k]));
        const float pd = 1e-5f * m + 1e-6f;
        node[8 * k] = lo[k] - pd;
        node[8 * k + 4] = hi[k] + pd;
      }
      const uint32_t ref = (uint32_t)leaf_ref(0, T);
      std::memcpy(&node[24], &ref, 4);
      out.num_leaves = 1;
      out.max_stack = 0;
    }
    GB_TRY(hipMalloc(&out.nodes, 128));
    out.nodes_bytes = 128;
    GB_TRY(hipMemcpyAsync(out.nodes, node.data(), 128, hipMemcpyHostToDevice, s));
    out.root = 0;
    out.num_nodes = 1;
    out.levels = 1;
  } else {
    Tmp bounds, keys, keys_sorted, vals, vals_sorted, child, pint, pleaf, rfirst, rcount, lbox, nbox, arr, sort_tmp, fr_node[2],
        fr_need[2], counters;
    GB_TRY(bounds.alloc(24));
    const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    GB_TRY(hipMemcpyAsync(bounds.p, init, 24, hipMemcpyHostToDevice, s));
    GB_TRY(keys.alloc((size_t)T * 8));
    GB_TRY(keys_sorted.alloc((size_t)T * 8));
    GB_TRY(vals.alloc((size_t)T * 4));
    GB_TRY(vals_sorted.alloc((size_t)T * 4));
    const uint32_t nb = std::min<uint32_t>(blocks, 4096);
    k_centroid_bounds<<<nb, kB, 0, s>>>(pos, stride_bytes, indices, T, bounds.as<uint32_t>());
    GB_TRY(hipGetLastError());
    k_morton<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, T, bounds.as<uint32_t>(), keys.as<uint64_t>(),
                                   vals.as<uint32_t>());
    GB_TRY(hipGetLastError());
    size_t tmp_bytes = 0;
    GB_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys.as<uint64_t>(), keys_sorted.as<uint64_t>(),
                                     vals.as<uint32_t>(), vals_sorted.as<uint32_t>(), T, 0, 63, s));
    GB_TRY(sort_tmp.alloc(tmp_bytes));
    GB_TRY(rocprim::radix_sort_pairs(sort_tmp.p, tmp_bytes, keys.as<uint64_t>(), keys_sorted.as<uint64_t>(),
                                     vals.as<uint32_t>(), vals_sorted.as<uint32_t>(), T, 0, 63, s));
    GB_TRY(child.alloc((size_t)(T - 1) * 8));
    GB_TRY(pint.alloc((size_t)(T - 1) * 4));
    GB_TRY(pleaf.alloc((size_t)T * 4));
    GB_TRY(rfirst.alloc((size_t)(T - 1) * 4));
    GB_TRY(rcount.alloc((size_t)(T - 1) * 4));
    k_radix_tree<<<(T - 1 + kB - 1) / kB, kB, 0, s>>>(keys_sorted.as<uint64_t>(), (int)T, child.as<int32_t>(),
                                                      pint.as<int32_t>(), pleaf.as<int32_t>(), rfirst.as<uint32_t>(),
                                                      rcount.as<uint32_t>());
    GB_TRY(hipGetLastError());
    GB_TRY(lbox.alloc((size_t)T * 32));
    GB_TRY(nbox.alloc((size_t)(T - 1) * 32));
    GB_TRY(arr.alloc((size_t)(T - 1) * 4));
    GB_TRY(hipMemsetAsync(arr.p, 0, (size_t)(T - 1) * 4, s));
    k_leaves_refit<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, vals_sorted.as<uint32_t>(), T,
                                         child.as<int32_t>(), pint.as<int32_t>(), pleaf.as<int32_t>(),
                                         reinterpret_cast<float4*>(out.tris), lbox.as<float4>(), nbox.as<float4>(),
                                         arr.as<uint32_t>(), true);
    GB_TRY(hipGetLastError());
    // level-synchronous collapse; BVH4 nodes <= binary internal nodes
    Tmp nodes_ub;
    GB_TRY(nodes_ub.alloc((size_t)(T - 1) * 128));
    for (int k = 0; k < 2; ++k) {
      GB_TRY(fr_node[k].alloc((size_t)T * 4));
      GB_TRY(fr_need[k].alloc((size_t)T * 4));
    }
    GB_TRY(counters.alloc(16));
    GB_TRY(hipMemsetAsync(counters.p, 0, 16, s));   // [0] leaves, [1] max stack, [2] next-level count
    const int32_t root_bin = 0;
    const uint32_t zero = 0;
    GB_TRY(hipMemcpyAsync(fr_node[0].p, &root_bin, 4, hipMemcpyHostToDevice, s));
    GB_TRY(hipMemcpyAsync(fr_need[0].p, &zero, 4, hipMemcpyHostToDevice, s));
    uint32_t base = 0, count = 1, levels = 0;
    int cur = 0;
    while (count) {
      GB_TRY(hipMemsetAsync(counters.as<uint32_t>() + 2, 0, 4, s));
      LevelArgs la;
      la.child = child.as<int32_t>();
      la.rfirst = rfirst.as<uint32_t>();
      la.rcount = rcount.as<uint32_t>();
      la.leaf_box = lbox.as<float4>();
      la.node_box = nbox.as<float4>();
      la.in_node = fr_node[cur].as<int32_t>();
      la.in_need = fr_need[cur].as<uint32_t>();
      la.in_count = count;
      la.base = base;
      la.next_base = base + count;
      la.out_node = fr_node[cur ^ 1].as<int32_t>();
      la.out_need = fr_need[cur ^ 1].as<uint32_t>();
      la.out_count = counters.as<uint32_t>() + 2;
      la.stats = counters.as<uint32_t>();
      la.max_leaf = max_leaf;
      la.nodes = nodes_ub.as<float>();
      k_collapse_level<<<(count + kB - 1) / kB, kB, 0, s>>>(la);
      GB_TRY(hipGetLastError());
      uint32_t next = 0;
      GB_TRY(hipMemcpyAsync(&next, counters.as<uint32_t>() + 2, 4, hipMemcpyDeviceToHost, s));
      GB_TRY(hipStreamSynchronize(s));
      base += count;
      count = next;
      cur ^= 1;
      ++levels;
    }
    uint32_t stats[2];
    GB_TRY(hipMemcpyAsync(stats, counters.p, 8, hipMemcpyDeviceToHost, s));
    GB_TRY(hipStreamSynchronize(s));
    out.num_nodes = base;
    out.num_leaves = stats[0];
    out.max_stack = stats[1];
    out.levels = levels;
    out.root = 0;
    out.nodes_bytes = (size_t)base * 128;
    GB_TRY(hipMalloc(&out.nodes, out.nodes_bytes));
    GB_TRY(hipMemcpyAsync(out.nodes, nodes_ub.p, out.nodes_bytes, hipMemcpyDeviceToDevice, s));
    GB_TRY(hipStreamSynchronize(s));
  }
  GB_TRY(hipEventRecord(e1, s));
  GB_TRY(hipEventSynchronize(e1));
  float ms = 0.0f;
  GB_TRY(hipEventElapsedTime(&ms, e0, e1));
  out.build_ms = ms;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return hipSuccess;
}

}  // namespace mrt
