// bvh_gpu.hip — device-side LBVH build into the BVH4 layout (see bvh_gpu.h).
// Replaces MPSTriangleAccelerationStructure.rebuild (renderer/Renderer.mm:456-462).
#include "bvh_gpu.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

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

// Leaf boxes + (LBVH) bottom-up refit.  Thread p owns sorted triangle p:
// writes its box, then (climb) walks up; the second thread to reach an
// internal node (arrival counter) computes its box from both children.
// Release/acquire at agent scope around the counter makes the sibling's box
// visible across XCDs.
__global__ __launch_bounds__(kB) void k_leaves_refit(const uint8_t* pos, uint32_t stride, const uint32_t* idx,
                                                     const uint32_t* order, uint32_t T, const int32_t* child,
                                                     const int32_t* parent_int, const int32_t* parent_leaf,
                                                     float4* leaf_box, float4* node_box, uint32_t* arrivals,
                                                     bool climb) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= T) return;
  const Tri3 v = load_tri(pos, stride, idx, order[p]);
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

// leaf-ordered triangle record {v0|prim, e1, e2} of triangle t at slot q
__device__ __forceinline__ void write_tri(const uint8_t* pos, uint32_t stride, const uint32_t* idx, uint32_t t,
                                          float4* tris, uint32_t q) {
  const Tri3 v = load_tri(pos, stride, idx, t);
  tris[3 * (size_t)q + 0] = make_float4(v.a.x, v.a.y, v.a.z, __uint_as_float(t));
  tris[3 * (size_t)q + 1] = make_float4(v.b.x - v.a.x, v.b.y - v.a.y, v.b.z - v.a.z, 0.0f);
  tris[3 * (size_t)q + 2] = make_float4(v.c.x - v.a.x, v.c.y - v.a.y, v.c.z - v.a.z, 0.0f);
}
__global__ __launch_bounds__(kB) void k_tris_in_order(const uint8_t* pos, uint32_t stride, const uint32_t* idx,
                                                      uint32_t T, float4* tris) {
  const uint32_t t = blockIdx.x * kB + threadIdx.x;
  if (t < T) write_tri(pos, stride, idx, t, tris, t);
}

// ---- PLOC (Meister & Bittner 2018): clusters in Morton order, each merges
// with its nearest neighbour (smallest merged-box area) within +-kR
// positions when the choice is mutual; repeat until one cluster remains.
constexpr int kR = 16;

__device__ __forceinline__ float union_area(float4 alo, float4 ahi, float4 blo, float4 bhi) {
  const float x = fmaxf(ahi.x, bhi.x) - fminf(alo.x, blo.x);
  const float y = fmaxf(ahi.y, bhi.y) - fminf(alo.y, blo.y);
  const float z = fmaxf(ahi.z, bhi.z) - fminf(alo.z, blo.z);
  return 2.0f * (x * y + y * z + z * x);
}

// nn[i] = argmin_{0 < |j - i| <= kR} area(box_i U box_j), ties -> smallest j
// (a total order on pairs, so the globally best pair is always mutual and
// every iteration merges at least one pair)
__global__ __launch_bounds__(kB) void k_ploc_nn(uint32_t n, const float4* cb, int32_t* nn) {
  __shared__ float4 s_lo[kB + 2 * kR], s_hi[kB + 2 * kR];
  const int64_t b0 = (int64_t)blockIdx.x * kB - kR;
  for (int k = threadIdx.x; k < kB + 2 * kR; k += kB) {
    const int64_t g = b0 + k;
    if (g >= 0 && g < (int64_t)n) { s_lo[k] = cb[2 * g]; s_hi[k] = cb[2 * g + 1]; }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= (int64_t)n) return;
  const float4 lo = s_lo[threadIdx.x + kR], hi = s_hi[threadIdx.x + kR];
  int32_t best = -1;
  float best_a = INFINITY;
  for (int o = -kR; o <= kR; ++o) {
    const int64_t j = i + o;
    if (o == 0 || j < 0 || j >= (int64_t)n) continue;
    const float a = union_area(lo, hi, s_lo[threadIdx.x + kR + o], s_hi[threadIdx.x + kR + o]);
    if (a < best_a) { best_a = a; best = (int32_t)j; }
  }
  nn[i] = best;
}

// merge flag (i < j of a mutual pair) and keep flag (not the absorbed j)
__global__ __launch_bounds__(kB) void k_ploc_flags(uint32_t n, const int32_t* nn, uint32_t* merge, uint32_t* keep) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const int32_t j = nn[i];
  const bool mutual = j >= 0 && nn[j] == (int32_t)i;
  merge[i] = (mutual && (int32_t)i < j) ? 1u : 0u;
  keep[i] = (mutual && (int32_t)i > j) ? 0u : 1u;
}

__global__ __launch_bounds__(kB) void k_ploc_merge(uint32_t n, const int32_t* nn, const uint32_t* merge,
                                                   const uint32_t* mscan, const uint32_t* keep,
                                                   const uint32_t* kscan, const int32_t* cid, const float4* cb,
                                                   uint32_t node_base, int32_t* child, float4* node_box,
                                                   uint32_t* count, int32_t* out_cid, float4* out_cb) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n || !keep[i]) return;
  int32_t c = cid[i];
  float4 lo = cb[2 * (size_t)i], hi = cb[2 * (size_t)i + 1];
  if (merge[i]) {
    const int32_t j = nn[i];
    const int32_t cj = cid[j];
    const uint32_t id = node_base + mscan[i];
    const float4 blo = cb[2 * (size_t)j], bhi = cb[2 * (size_t)j + 1];
    lo = make_float4(fminf(lo.x, blo.x), fminf(lo.y, blo.y), fminf(lo.z, blo.z), 0.0f);
    hi = make_float4(fmaxf(hi.x, bhi.x), fmaxf(hi.y, bhi.y), fmaxf(hi.z, bhi.z), 0.0f);
    child[2 * (size_t)id] = c;
    child[2 * (size_t)id + 1] = cj;
    node_box[2 * (size_t)id] = lo;
    node_box[2 * (size_t)id + 1] = hi;
    count[id] = (c >= 0 ? count[c] : 1u) + (cj >= 0 ? count[cj] : 1u);
    c = (int32_t)id;
  }
  const uint32_t o = kscan[i];
  out_cid[o] = c;
  out_cb[2 * (size_t)o] = lo;
  out_cb[2 * (size_t)o + 1] = hi;
}

__global__ __launch_bounds__(kB) void k_ploc_init(uint32_t T, const float4* leaf_box, int32_t* cid, float4* cb) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= T) return;
  cid[p] = ~(int32_t)p;
  cb[2 * (size_t)p] = leaf_box[2 * (size_t)p];
  cb[2 * (size_t)p + 1] = leaf_box[2 * (size_t)p + 1];
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
  const uint32_t* rcount;     // triangles under each binary internal node
  const float4* leaf_box;
  const float4* node_box;
  const int32_t* in_node;     // binary internal node of each frontier slot
  const uint32_t* in_need;    // stack entries on the way down to it
  const uint32_t* in_first;   // first leaf-order slot of its triangles
  uint32_t in_count;
  uint32_t base;              // output index of frontier slot 0
  uint32_t next_base;         // output index of next-frontier slot 0
  int32_t* out_node;
  uint32_t* out_need;
  uint32_t* out_first;
  uint32_t* out_count;
  uint32_t* stats;            // [0] leaves, [1] max stack
  uint32_t max_leaf;
  float* nodes;               // BVH4 records, 32 floats each
  // leaf triangle records
  const uint8_t* pos;
  uint32_t stride;
  const uint32_t* idx;
  const uint32_t* order;      // sorted position -> triangle
  float4* tris;
};

// One BVH4 node per frontier slot: open the largest-area interior child until
// four children (or none left to open), emit the node, append interior
// children to the next level.  A subtree's triangles occupy the contiguous
// leaf-order range [first, first + count); children split it in child order,
// and a child small enough to be a leaf writes its triangle records there.
__global__ __launch_bounds__(kB) void k_collapse_level(LevelArgs a) {
  const uint32_t slot = blockIdx.x * kB + threadIdx.x;
  if (slot >= a.in_count) return;
  const int32_t b = a.in_node[slot];
  const uint32_t need = a.in_need[slot];
  uint32_t first = a.in_first[slot];
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
      for (int k = 0; k < 3; ++k) { o[8 * k + c] = __builtin_inff(); o[8 * k + 4 + c] = -__builtin_inff(); }   // inverted box
      o[24 + c] = __uint_as_float((uint32_t)kEmptyChild);
      continue;
    }
    const int32_t x = ch[c];
    const uint32_t cnt = count_of(x);
    const float4* bx = x >= 0 ? a.node_box + 2 * (size_t)x : a.leaf_box + 2 * (size_t)(~x);
    const float4 lo = bx[0], hi = bx[1];
    const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
    for (int k = 0; k < 3; ++k) {
      const float pd = pad_of(l3[k], h3[k]);
      o[8 * k + c] = __fsub_rn(l3[k], pd);
      o[8 * k + 4 + c] = __fadd_rn(h3[k], pd);
    }
    int32_t ref;
    if (cnt <= a.max_leaf) {
      // leaf: write the subtree's triangles in order (depth-first, <= 16 of them)
      ref = dev_leaf_ref(first, cnt);
      atomicAdd(&a.stats[0], 1u);
      int32_t st[kMaxLeafSize];
      int sp = 0;
      st[sp++] = x;
      uint32_t q = first;
      while (sp) {
        const int32_t y = st[--sp];
        if (y < 0) {
          write_tri(a.pos, a.stride, a.idx, a.order[~y], a.tris, q++);
        } else {
          st[sp++] = a.child[2 * (size_t)y + 1];
          st[sp++] = a.child[2 * (size_t)y];
        }
      }
    } else {
      const uint32_t s = atomicAdd(a.out_count, 1u);
      a.out_node[s] = x;
      a.out_need[s] = child_need;
      a.out_first[s] = first;
      ref = (int32_t)(a.next_base + s);
    }
    first += cnt;
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

hipError_t build_bvh_gpu(const float* positions, uint32_t stride_bytes, const uint32_t* indices, uint32_t T,
                         uint32_t max_leaf, GpuBvhAlgo algo, hipStream_t s, GpuBvhResult& out, std::string& error) {
  out = GpuBvhResult{};
  max_leaf = std::max<uint32_t>(1, std::min<uint32_t>(max_leaf ? max_leaf : 2, (uint32_t)kMaxLeafSize));
  if (T >= (1u << (32 - kLeafCountBits - 1))) { error = "too many triangles for the leaf encoding"; return hipErrorInvalidValue; }
  hipEvent_t e0, e1;
  GB_TRY(hipEventCreate(&e0));
  GB_TRY(hipEventCreate(&e1));
  GB_TRY(hipEventRecord(e0, s));
  const uint8_t* pos = reinterpret_cast<const uint8_t*>(positions);
  const uint32_t blocks = (std::max<uint32_t>(T, 1) + kB - 1) / kB;
  auto grid = [](uint32_t n) { return (std::max<uint32_t>(n, 1) + kB - 1) / kB; };

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
    if (T) {
      GB_TRY(hipMemcpyAsync(order.p, ho.data(), (size_t)T * 4, hipMemcpyHostToDevice, s));
      k_tris_in_order<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, T, reinterpret_cast<float4*>(out.tris));
      GB_TRY(hipGetLastError());
      k_leaves_refit<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, order.as<uint32_t>(), T, nullptr, nullptr,
                                           nullptr, lbox.as<float4>(), nullptr, nullptr, false);
      GB_TRY(hipGetLastError());
    }
    std::vector<float> lb((size_t)T * 8);
    if (T) GB_TRY(hipMemcpyAsync(lb.data(), lbox.p, (size_t)T * 32, hipMemcpyDeviceToHost, s));
    GB_TRY(hipStreamSynchronize(s));
    std::vector<float> node(32, 0.0f);
    for (int c = 0; c < 4; ++c) {   // empty slots: kEmptyChild with an inverted box (kernels.hip box4)
      uint32_t ref = (uint32_t)kEmptyChild;
      std::memcpy(&node[24 + c], &ref, 4);
      for (int k = 0; k < 3; ++k) { node[8 * k + c] = INFINITY; node[8 * k + 4 + c] = -INFINITY; }
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
    // 1. Morton order of the triangle centroids
    Tmp bounds, keys, keys_sorted, vals, order, child, rcount, lbox, nbox, sort_tmp;
    GB_TRY(bounds.alloc(24));
    const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    GB_TRY(hipMemcpyAsync(bounds.p, init, 24, hipMemcpyHostToDevice, s));
    GB_TRY(keys.alloc((size_t)T * 8));
    GB_TRY(keys_sorted.alloc((size_t)T * 8));
    GB_TRY(vals.alloc((size_t)T * 4));
    GB_TRY(order.alloc((size_t)T * 4));
    k_centroid_bounds<<<std::min<uint32_t>(blocks, 4096), kB, 0, s>>>(pos, stride_bytes, indices, T,
                                                                      bounds.as<uint32_t>());
    GB_TRY(hipGetLastError());
    k_morton<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, T, bounds.as<uint32_t>(), keys.as<uint64_t>(),
                                   vals.as<uint32_t>());
    GB_TRY(hipGetLastError());
    size_t tmp_bytes = 0, scan_bytes = 0;
    GB_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys.as<uint64_t>(), keys_sorted.as<uint64_t>(),
                                     vals.as<uint32_t>(), order.as<uint32_t>(), T, 0, 63, s));
    GB_TRY(rocprim::exclusive_scan(nullptr, scan_bytes, vals.as<uint32_t>(), vals.as<uint32_t>(), 0u, T,
                                   rocprim::plus<uint32_t>(), s));
    GB_TRY(sort_tmp.alloc(std::max(tmp_bytes, scan_bytes)));
    GB_TRY(rocprim::radix_sort_pairs(sort_tmp.p, tmp_bytes, keys.as<uint64_t>(), keys_sorted.as<uint64_t>(),
                                     vals.as<uint32_t>(), order.as<uint32_t>(), T, 0, 63, s));
    // 2. binary tree over the sorted triangles (internal nodes 0..T-2)
    GB_TRY(child.alloc((size_t)(T - 1) * 8));
    GB_TRY(rcount.alloc((size_t)(T - 1) * 4));
    GB_TRY(lbox.alloc((size_t)T * 32));
    GB_TRY(nbox.alloc((size_t)(T - 1) * 32));
    int32_t root_bin = 0;
    if (algo == GpuBvhAlgo::kLbvh) {
      Tmp pint, pleaf, rfirst, arr;
      GB_TRY(pint.alloc((size_t)(T - 1) * 4));
      GB_TRY(pleaf.alloc((size_t)T * 4));
      GB_TRY(rfirst.alloc((size_t)(T - 1) * 4));
      GB_TRY(arr.alloc((size_t)(T - 1) * 4));
      k_radix_tree<<<grid(T - 1), kB, 0, s>>>(keys_sorted.as<uint64_t>(), (int)T, child.as<int32_t>(),
                                              pint.as<int32_t>(), pleaf.as<int32_t>(), rfirst.as<uint32_t>(),
                                              rcount.as<uint32_t>());
      GB_TRY(hipGetLastError());
      GB_TRY(hipMemsetAsync(arr.p, 0, (size_t)(T - 1) * 4, s));
      k_leaves_refit<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, order.as<uint32_t>(), T, child.as<int32_t>(),
                                           pint.as<int32_t>(), pleaf.as<int32_t>(), lbox.as<float4>(),
                                           nbox.as<float4>(), arr.as<uint32_t>(), true);
      GB_TRY(hipGetLastError());
      GB_TRY(hipStreamSynchronize(s));
      root_bin = 0;
    } else {
      k_leaves_refit<<<blocks, kB, 0, s>>>(pos, stride_bytes, indices, order.as<uint32_t>(), T, nullptr, nullptr,
                                           nullptr, lbox.as<float4>(), nullptr, nullptr, false);
      GB_TRY(hipGetLastError());
      Tmp cid[2], cb[2], nn, mflag, mscan, keep, kscan;
      for (int k = 0; k < 2; ++k) {
        GB_TRY(cid[k].alloc((size_t)T * 4));
        GB_TRY(cb[k].alloc((size_t)T * 32));
      }
      GB_TRY(nn.alloc((size_t)T * 4));
      GB_TRY(mflag.alloc((size_t)T * 4));
      GB_TRY(mscan.alloc((size_t)T * 4));
      GB_TRY(keep.alloc((size_t)T * 4));
      GB_TRY(kscan.alloc((size_t)T * 4));
      k_ploc_init<<<blocks, kB, 0, s>>>(T, lbox.as<float4>(), cid[0].as<int32_t>(), cb[0].as<float4>());
      GB_TRY(hipGetLastError());
      uint32_t n = T, node_base = 0;
      int cur = 0;
      uint32_t iters = 0;
      while (n > 1) {
        k_ploc_nn<<<grid(n), kB, 0, s>>>(n, cb[cur].as<float4>(), nn.as<int32_t>());
        GB_TRY(hipGetLastError());
        k_ploc_flags<<<grid(n), kB, 0, s>>>(n, nn.as<int32_t>(), mflag.as<uint32_t>(), keep.as<uint32_t>());
        GB_TRY(hipGetLastError());
        size_t sb = scan_bytes;
        GB_TRY(rocprim::exclusive_scan(sort_tmp.p, sb, mflag.as<uint32_t>(), mscan.as<uint32_t>(), 0u, n,
                                       rocprim::plus<uint32_t>(), s));
        sb = scan_bytes;
        GB_TRY(rocprim::exclusive_scan(sort_tmp.p, sb, keep.as<uint32_t>(), kscan.as<uint32_t>(), 0u, n,
                                       rocprim::plus<uint32_t>(), s));
        k_ploc_merge<<<grid(n), kB, 0, s>>>(n, nn.as<int32_t>(), mflag.as<uint32_t>(), mscan.as<uint32_t>(),
                                            keep.as<uint32_t>(), kscan.as<uint32_t>(), cid[cur].as<int32_t>(),
                                            cb[cur].as<float4>(), node_base, child.as<int32_t>(), nbox.as<float4>(),
                                            rcount.as<uint32_t>(), cid[cur ^ 1].as<int32_t>(), cb[cur ^ 1].as<float4>());
        GB_TRY(hipGetLastError());
        uint32_t tail[4];
        GB_TRY(hipMemcpyAsync(&tail[0], mscan.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        GB_TRY(hipMemcpyAsync(&tail[1], mflag.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        GB_TRY(hipMemcpyAsync(&tail[2], kscan.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        GB_TRY(hipMemcpyAsync(&tail[3], keep.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        GB_TRY(hipStreamSynchronize(s));
        const uint32_t merges = tail[0] + tail[1], next = tail[2] + tail[3];
        if (merges == 0 || next + merges != n) { error = "PLOC made no progress"; return hipErrorUnknown; }
        node_base += merges;
        n = next;
        cur ^= 1;
        ++iters;
      }
      GB_TRY(hipMemcpy(&root_bin, cid[cur].p, 4, hipMemcpyDeviceToHost));
      if (node_base != T - 1 || root_bin != (int32_t)(T - 2)) { error = "PLOC tree incomplete"; return hipErrorUnknown; }
      out.build_iterations = iters;
    }
    // 3. level-synchronous collapse into BVH4 nodes (breadth-first order)
    Tmp nodes_ub, fr_node[2], fr_need[2], fr_first[2], counters;
    GB_TRY(nodes_ub.alloc((size_t)(T - 1) * 128));
    for (int k = 0; k < 2; ++k) {
      GB_TRY(fr_node[k].alloc((size_t)T * 4));
      GB_TRY(fr_need[k].alloc((size_t)T * 4));
      GB_TRY(fr_first[k].alloc((size_t)T * 4));
    }
    GB_TRY(counters.alloc(16));
    GB_TRY(hipMemsetAsync(counters.p, 0, 16, s));   // [0] leaves, [1] max stack, [2] next-level count
    const uint32_t zero = 0;
    GB_TRY(hipMemcpyAsync(fr_node[0].p, &root_bin, 4, hipMemcpyHostToDevice, s));
    GB_TRY(hipMemcpyAsync(fr_need[0].p, &zero, 4, hipMemcpyHostToDevice, s));
    GB_TRY(hipMemcpyAsync(fr_first[0].p, &zero, 4, hipMemcpyHostToDevice, s));
    uint32_t base = 0, count = 1, levels = 0;
    int cur = 0;
    while (count) {
      GB_TRY(hipMemsetAsync(counters.as<uint32_t>() + 2, 0, 4, s));
      LevelArgs la;
      la.child = child.as<int32_t>();
      la.rcount = rcount.as<uint32_t>();
      la.leaf_box = lbox.as<float4>();
      la.node_box = nbox.as<float4>();
      la.in_node = fr_node[cur].as<int32_t>();
      la.in_need = fr_need[cur].as<uint32_t>();
      la.in_first = fr_first[cur].as<uint32_t>();
      la.in_count = count;
      la.base = base;
      la.next_base = base + count;
      la.out_node = fr_node[cur ^ 1].as<int32_t>();
      la.out_need = fr_need[cur ^ 1].as<uint32_t>();
      la.out_first = fr_first[cur ^ 1].as<uint32_t>();
      la.out_count = counters.as<uint32_t>() + 2;
      la.stats = counters.as<uint32_t>();
      la.max_leaf = max_leaf;
      la.nodes = nodes_ub.as<float>();
      la.pos = pos;
      la.stride = stride_bytes;
      la.idx = indices;
      la.order = order.as<uint32_t>();
      la.tris = reinterpret_cast<float4*>(out.tris);
      k_collapse_level<<<grid(count), kB, 0, s>>>(la);
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
