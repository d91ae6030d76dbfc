// kernels.hip — gfx950 kernels of the path-tracing hot path.
//
// Compiled twice (see kernels.h): MRT_PRECISE=1 -> namespace mrt::precise,
// MRT_PRECISE=0 -> mrt::fast.  Every device function below restates one
// reference function; the citation is on the function.  Evaluation order of
// every float expression follows the reference source so the precise build is
// bit-comparable with the CPU oracle.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "diag_env.h"
#include "kernels.h"

#ifndef MRT_PRECISE
#error "compile with -DMRT_PRECISE=0 or 1"
#endif
#ifndef MRT_TU
#define MRT_TU 0
#endif
// The stream kernel's entry points: in unit 2 of the split fast build, or in
// the whole-file build (0) — and in unit 1 for lane-statistics builds, whose
// counters (g_lanes) must live in the unit that reads them (unit 2 then
// emits nothing)
#ifndef MRT_LANESTATS
#define MRT_LANESTATS 0
#endif
#define MRT_EMIT_STREAM (MRT_TU == 0 || (MRT_TU == 2 && !MRT_LANESTATS) || (MRT_TU == 1 && MRT_LANESTATS))
#define MRT_EMIT_MAIN (MRT_TU != 2)
#if MRT_PRECISE
#define MRT_NS precise
#else
#define MRT_NS fast
#endif

namespace mrt {
namespace MRT_NS {
namespace {

constexpr int kBlock = 256;   // 4 waves of 64 lanes
// Minimum waves per SIMD for the bounce kernel (launch bounds; the stream
// kernel has its own, MRT_STREAM_WAVES): 5 caps it at
// 96 VGPRs with 48 B/lane of scratch spills; 6 (80 VGPRs) spills ~140 B/lane
// and 4 (no spills) hides less latency — 5 measured best with one stream.
#ifndef MRT_BOUNCE_WAVES
#define MRT_BOUNCE_WAVES 5
#endif

// ---------------------------------------------------------------------------
// scalar math (precision policy)
// ---------------------------------------------------------------------------
#if MRT_PRECISE
__device__ __forceinline__ float m_rcp(float x) { return 1.0f / x; }
__device__ __forceinline__ float m_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ float m_rsqrt(float x) { return 1.0f / sqrtf(x); }
__device__ __forceinline__ float m_div(float a, float b) { return a / b; }
__device__ __forceinline__ float m_sin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float m_cos(float x) { return (float)cos((double)x); }
#else
__device__ __forceinline__ float m_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float m_sqrt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float m_rsqrt(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float m_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float m_sin(float x) { return __sinf(x); }
__device__ __forceinline__ float m_cos(float x) { return __cosf(x); }
#endif

// ---------------------------------------------------------------------------
// float3 helpers with explicit evaluation order (MSL semantics)
// ---------------------------------------------------------------------------
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ V3 mk(const float4& a) { return {a.x, a.y, a.z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float length(V3 a) { return m_sqrt(dot(a, a)); }
__device__ __forceinline__ V3 normalize(V3 a) { return mul(a, m_rsqrt(dot(a, a))); }
// MSL reflect(I, N) = I - 2 * dot(N, I) * N
__device__ __forceinline__ V3 reflect(V3 i, V3 n) { const float k = 2.0f * dot(n, i); return sub(i, mul(n, k)); }
// MSL mix(x, y, a) = x + (y - x) * a
__device__ __forceinline__ float mixf(float x, float y, float a) { return x + (y - x) * a; }

__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
// set bits of a wave mask in the lanes below this one (v_mbcnt: no per-lane
// 64-bit mask kept live — in the stream kernel that mask was spilled, r6)
__device__ __forceinline__ uint32_t lanes_below_in(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ---------------------------------------------------------------------------
// Geometry: MPS nearest-hit semantics (renderer/Renderer.mm:464-469)
// ---------------------------------------------------------------------------
// Moller-Trumbore, cull none; (u, v) are the weights of (V0, V1) as
// interpolate() expects (renderer/KernelHelpers.h:37-47).
// The fast build contracts the test's products and sums into FMAs (a
// no-contraction variant measured slower and was removed in r6); which
// triangle a near-tie ray reports may then differ from the IEEE answer, never
// with the visiting order (the culling slack, interior_step).
__device__ __forceinline__ float tdot(V3 a, V3 b) {
  return (a.x * b.x + a.y * b.y) + a.z * b.z;
}
__device__ __forceinline__ V3 tcross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ bool tri_test(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float tmin, float tmax, float& t,
                                         float& u, float& v) {
  // early exits: most candidate triangles fail the first barycentric test,
  // and a wave whose lanes all fail skips the rest (s_cbranch_execz)
  const V3 p = tcross(d, e2);
  const float det = tdot(e1, p);
  if (det == 0.0f) return false;
  const float inv = m_rcp(det);
  const V3 s = sub(o, v0);
  const float b1 = tdot(s, p) * inv;
  if (!(b1 >= 0.0f && b1 <= 1.0f)) return false;
  const V3 q = tcross(s, e1);
  const float b2 = tdot(d, q) * inv;
  if (!(b2 >= 0.0f && b1 + b2 <= 1.0f)) return false;
  const float tt = tdot(e2, q) * inv;
  if (!(tt >= tmin && tt <= tmax)) return false;
  t = tt;
  u = (1.0f - b1) - b2;
  v = b1;
  return true;
}

// The same arithmetic as tri_test without the early exits (so the same hits,
// bit for bit), for the leaf loops: the distance range test is left to the
// caller.  Every operand is needed before the first decision, so the loads of
// a triangle are all in flight together instead of v0's being issued only
// after the determinant test passed.
__device__ __forceinline__ bool tri_bary(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float& t, float& u, float& v) {
  const V3 p = tcross(d, e2);
  const float det = tdot(e1, p);
  const float inv = m_rcp(det);
  const V3 s = sub(o, v0);
  const float b1 = tdot(s, p) * inv;
  const V3 q = tcross(s, e1);
  const float b2 = tdot(d, q) * inv;
  t = tdot(e2, q) * inv;
  u = (1.0f - b1) - b2;
  v = b1;
  return (det != 0.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f);
}

struct Hit {
  float t, u, v;
  uint32_t prim;
  bool found;
};

// Node rows in ray order.  In the all-in-LDS mode every BVH4 node's x and y
// plane rows are staged in four copies, one per sign quadrant of (dir.x,
// dir.y), each pre-ordered (near, far) for rays of that quadrant; a ray reads
// the copy of its quadrant and its z rows in ray order by a row offset, so
// the box test pairs no planes by min/max (24 fewer VALU ops per node).
// Slab distances are monotone in the plane coordinate for a fixed direction
// (in both builds), so the quadrant's near plane is exactly the min of the
// pair and results are bit-identical.  (Eight octant copies measured -7.5 %
// on C2: the larger LDS image cost a resident block.)  The other modes (top
// nodes in LDS, the rest in global memory) read a node's plane rows in ray
// order through per-lane row offsets; their empty child slots are masked by
// their inverted box alone, global nodes are fetched with buffer loads
// (32-bit offsets from one descriptor), and LDS + spill stacks take plain LDS
// pushes / pops in steps where no lane can reach the spill area.  r4 A/B
// (C4 / C3 Mpaths/s, alternating in one call): buffer loads + spill fast
// path 2890 -> 2946 / 2686 -> 2735; the empty-box mask 3007-3033 / 2818-2823
// and plain pops 2971-2976 / 2791-2792 against 2922 / 2752 without either.
// Variants measured slower and removed in r6: unconditional three-entry
// pushes, an unsorted (slot-order) z row, a no-contraction triangle test.
constexpr uint32_t kQuadCopies = 4;                      // (x, y) sign quadrants
constexpr uint32_t kQuadCopyF4 = 7;                      // six plane rows + the refs row
constexpr uint32_t kQuadNodeF4 = kQuadCopies * kQuadCopyF4;

struct RayBox {   // precomputed slab-test terms
  V3 inv;
#if !MRT_PRECISE
  V3 oinv;
#endif
  uint32_t quad_f4;   // kQuadCopyF4 x quadrant; quadrant bit a set where direction component a (x, y) is negative
};

__device__ __forceinline__ float safe_inv(float d) {
  const float dd = fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d);
  return m_rcp(dd);
}

__device__ __forceinline__ RayBox make_raybox(V3 o, V3 d) {
  RayBox r;
  r.inv = mk(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
#if !MRT_PRECISE
  r.oinv = mk(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
#endif
  r.quad_f4 = kQuadCopyF4 * ((fbits(r.inv.x) >> 31) | ((fbits(r.inv.y) >> 31) << 1));
  return r;
}

// slab entry/exit on one axis; boxes are padded at build time so either form
// is conservative.
__device__ __forceinline__ float slab(float p, float o, float inv, float oinv) {
#if MRT_PRECISE
  (void)oinv;
  return (p - o) * inv;
#else
  (void)o;
  return fmaf(p, inv, -oinv);
#endif
}

// Box test of the four children of a BVH4 node (component-major node, see
// mrt_layout.h); returns each child's entry distance, +inf for a miss or an
// empty slot.  ORDERED: the x and y plane rows arrive as (near, far) (a
// quadrant copy of the all-in-LDS mode); otherwise as (lo, hi).
// LIVE = false (rows in ray order only): empty child slots are not masked by
// their ref but by their box — the builders store an inverted box (lo = +inf,
// hi = -inf) in every empty slot, whose near slab is +inf in every ray order
// (in the (lo, hi) order min/max would turn it into an infinite box)
template <int ORDERED, bool LIVE = true>   // 0: (lo, hi) rows; 2: x, y rows (near, far); 3: all rows (near, far)
__device__ __forceinline__ void box4(const float4* q, V3 o, const RayBox& rb, float tmin, float tmax, float tn[4]) {
#if MRT_PRECISE
  const float ox = o.x, oy = o.y, oz = o.z;
  const float oix = 0.0f, oiy = 0.0f, oiz = 0.0f;
#else
  const float ox = 0.0f, oy = 0.0f, oz = 0.0f;
  const float oix = rb.oinv.x, oiy = rb.oinv.y, oiz = rb.oinv.z;
  (void)o;
#endif
  const float* f = reinterpret_cast<const float*>(q);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x0 = slab(f[k], ox, rb.inv.x, oix), x1 = slab(f[4 + k], ox, rb.inv.x, oix);
    const float y0 = slab(f[8 + k], oy, rb.inv.y, oiy), y1 = slab(f[12 + k], oy, rb.inv.y, oiy);
    const float z0 = slab(f[16 + k], oz, rb.inv.z, oiz), z1 = slab(f[20 + k], oz, rb.inv.z, oiz);
    float tnear, tfar;
    if constexpr (ORDERED == 3) {
      tnear = fmaxf(fmaxf(x0, y0), fmaxf(z0, tmin));
      tfar = fminf(fminf(x1, y1), fminf(z1, tmax));
    } else if constexpr (ORDERED == 2) {
      tnear = fmaxf(fmaxf(x0, y0), fmaxf(fminf(z0, z1), tmin));
      tfar = fminf(fminf(x1, y1), fminf(fmaxf(z0, z1), tmax));
    } else {
      tnear = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), tmin));
      tfar = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tmax));
    }
    if constexpr (LIVE) {
      const bool live = (int32_t)fbits(f[24 + k]) != kEmptyChild;
      tn[k] = (live & (tnear <= tfar)) ? tnear : __builtin_inff();
    } else {
      static_assert(ORDERED == 3, "inverted empty boxes miss only with rows in ray order");
      tn[k] = (tnear <= tfar) ? tnear : __builtin_inff();
    }
  }
}

// LDS staging modes:
//   kGlobal  — only the per-lane traversal stack lives in LDS (stage ABI kernels);
//   kTopLds  — the first n BFS-ordered BVH nodes (top levels) are staged in
//              LDS; deeper nodes, leaf triangles and shading records are read
//              from global memory (L2 / Infinity Cache / HBM);
//   kAllLds  — small scenes: every node, leaf triangle, per-primitive shading
//              record, material and light entry is staged in LDS once per
//              block, so traversal and shading never leave the CU.
// LDS image: [nodes][triangles][prims][materials][lights] as float4, then the
// uint32 scratch (segment prefix), then the stack laid out [entry][lane]
// (consecutive lanes hit consecutive banks).  All LDS accesses index the
// __shared__ symbol directly so they lower to ds_read/ds_write (a pointer
// select between LDS and global lowers to flat_load).
enum LdsMode { kGlobal = 0, kTopLds = 1, kAllLds = 2 };
extern __shared__ float4 g_lds[];

struct LdsCtx {
  uint32_t n_lds_nodes;   // nodes [0, n) are in LDS
  uint32_t tri_base;      // float4 offsets (kAllLds)
  uint32_t prim_base;
  uint32_t mat_base;
  uint32_t light_base;
  uint32_t scratch_base;  // uint32 offset of the per-block scratch
  uint32_t stack_base;    // uint32 offset of the block's stack slot 0 (lane 0's); lanes add threadIdx.x
  uint32_t* spill;        // stack entries >= STACK: the block's rows of a global [lane][word] spill
                          //   area (null when STACK covers the BVH); lane threadIdx.x's row
  uint32_t spill_lane;    //   starts threadIdx.x * spill_lane words in (one word per entry)
};

__device__ __forceinline__ uint32_t* lds_u32() { return reinterpret_cast<uint32_t*>(g_lds); }

// float4s per staged node: the all-in-LDS BVH4 stages four
// quadrant copies of the six plane rows and the refs row (consecutive copies
// start 28 banks apart, so lanes of different quadrants reading the same node
// row hit disjoint banks)
__host__ __device__ constexpr uint32_t node_stride_f4(int mode, uint32_t node_f4) {
  return (mode == kAllLds && node_f4 == 8) ? kQuadNodeF4 : node_f4;
}

// float4 counts of the staged scene image for a mode
// (node_f4 = float4s per BVH4 node: 8; nodes / tri_records include the
// occluder tree's, prims are the scene's triangles)
__host__ __device__ inline uint32_t lds_scene_float4s(int mode, uint32_t node_f4, uint32_t nodes, uint32_t lds_nodes,
                                                      uint32_t tri_records, uint32_t prims, uint32_t mats,
                                                      uint32_t lights) {
  if (mode == kAllLds) return node_stride_f4(mode, node_f4) * nodes + 3 * tri_records + 6 * prims + 2 * mats + 7 * lights;
  if (mode == kTopLds) return node_f4 * lds_nodes;
  return 0;
}
// both trees' nodes and leaf-triangle records (mrt_layout.h DeviceScene)
__host__ __device__ inline uint32_t scene_nodes(const DeviceScene& sc) { return sc.num_nodes + sc.occ_nodes; }
__host__ __device__ inline uint32_t scene_tri_records(const DeviceScene& sc) { return sc.num_triangles + sc.occ_tris; }
__host__ __device__ inline uint32_t lds_scene_float4s(int mode, const DeviceScene& sc) {
  return lds_scene_float4s(mode, node_float4s(sc.width), scene_nodes(sc), sc.lds_nodes, scene_tri_records(sc),
                           sc.num_triangles, sc.num_materials, sc.num_lights + 1);
}

// 16-B buffer load at a 32-bit byte offset from a wave-uniform descriptor
// (no 64-bit address arithmetic per access); the host keeps every buffer
// read this way below 4 GiB (mrt_scene_create)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0xFFFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  return make_float4(bitsf(v[0]), bitsf(v[1]), bitsf(v[2]), bitsf(v[3]));
}

template <int MODE>
__device__ __forceinline__ void fetch_node4(const DeviceScene& sc, const LdsCtx& cx, int32_t node, const RayBox& rb,
                                            float4* q) {
  if (MODE == kAllLds) {   // the ray's quadrant copy
    const uint32_t sz = fbits(rb.inv.z) >> 31;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = g_lds[kQuadNodeF4 * node + rb.quad_f4 + i];
    q[4] = g_lds[kQuadNodeF4 * node + rb.quad_f4 + 4 + sz];
    q[5] = g_lds[kQuadNodeF4 * node + rb.quad_f4 + 5 - sz];
    q[6] = g_lds[kQuadNodeF4 * node + rb.quad_f4 + 6];
  } else {
    // top-nodes mode: rows in ray order, (near, far) per axis by the direction's signs
    const bool rowsel = MODE == kTopLds;
    const uint32_t sx = rowsel ? fbits(rb.inv.x) >> 31 : 0u, sy = rowsel ? fbits(rb.inv.y) >> 31 : 0u;
    const uint32_t sz = rowsel ? fbits(rb.inv.z) >> 31 : 0u;
    const uint32_t row[6] = {sx, 1u - sx, 2u + sy, 3u - sy, 4u + sz, 5u - sz};
    if (MODE == kAllLds || (MODE == kTopLds && (uint32_t)node < cx.n_lds_nodes)) {
#pragma unroll
      for (int i = 0; i < 6; ++i) q[i] = g_lds[8 * node + row[i]];
      q[6] = g_lds[8 * node + 6];
    } else {
      // one descriptor over the node array (kernel-argument values: wave-
      // uniform); per row a 32-bit offset node * 128 + row * 16
      const __amdgpu_buffer_rsrc_t rs = buf_rsrc(sc.nodes);
      const uint32_t b = (uint32_t)node << 7;
#pragma unroll
      for (int i = 0; i < 6; ++i) q[i] = buf_ld4(rs, b + (row[i] << 4));
      q[6] = buf_ld4(rs, b + 96u);
    }
  }
}

template <int MODE>
__device__ __forceinline__ void fetch_tri(const DeviceScene& sc, const LdsCtx& cx, uint32_t k, float4& t0,
                                          float4& t1, float4& t2) {
  if (MODE == kAllLds) {
    t0 = g_lds[cx.tri_base + 3 * k];
    t1 = g_lds[cx.tri_base + 3 * k + 1];
    t2 = g_lds[cx.tri_base + 3 * k + 2];
  } else {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(sc.tris);
    const uint32_t b = k * 48u;
    t0 = buf_ld4(rs, b);
    t1 = buf_ld4(rs, b + 16u);
    t2 = buf_ld4(rs, b + 32u);
  }
}

template <int MODE>
__device__ __forceinline__ float4 fetch_prim(const DeviceScene& sc, const LdsCtx& cx, uint32_t prim, uint32_t i) {
  if (MODE == kAllLds) return g_lds[cx.prim_base + 6 * prim + i];
  // (buffer loads here measured C4 -4 %, C3 -4.5 %: the shading records stay flat loads)
  return reinterpret_cast<const float4*>(sc.prims)[6 * (size_t)prim + i];
}
template <int MODE>
__device__ __forceinline__ float4 fetch_mat(const DeviceScene& sc, const LdsCtx& cx, uint32_t m, uint32_t i) {
  if (MODE == kAllLds) return g_lds[cx.mat_base + 2 * m + i];
  return reinterpret_cast<const float4*>(sc.materials)[2 * m + i];
}
template <int MODE>
__device__ __forceinline__ float4 fetch_light(const DeviceScene& sc, const LdsCtx& cx, uint32_t l, uint32_t i) {
  if (MODE == kAllLds) return g_lds[cx.light_base + 7 * l + i];
  return reinterpret_cast<const float4*>(sc.lights)[7 * l + i];
}

// STACK = LDS entries per lane; a negative STACK means |STACK| LDS entries
// plus the global spill area for deeper entries.
// A lane's spilled words are contiguous: its pushes and pops keep touching
// the same few cache lines (measured +1.1 % C4, +1.5 % C3 over [entry][lane]).
__device__ __forceinline__ uint32_t spill_index(const LdsCtx& cx, int w) {
  return threadIdx.x * cx.spill_lane + (uint32_t)w;
}
template <int STACK>
__device__ __forceinline__ void stack_push(const LdsCtx& cx, int sp, int32_t v) {
  constexpr int kL = STACK < 0 ? -STACK : STACK;
  if (STACK > 0 || sp < kL) lds_u32()[cx.stack_base + threadIdx.x + sp * kBlock] = (uint32_t)v;
  else cx.spill[spill_index(cx, sp - kL)] = (uint32_t)v;
}
template <int STACK>
__device__ __forceinline__ int32_t stack_get(const LdsCtx& cx, int sp) {
  constexpr int kL = STACK < 0 ? -STACK : STACK;
  if (STACK > 0 || sp < kL) return (int32_t)lds_u32()[cx.stack_base + threadIdx.x + sp * kBlock];
  uint32_t v = cx.spill[spill_index(cx, sp - kL)];
  // keeps the two loads apart: merged, they become one flat load whose wait
  // covers every outstanding global access (the spill stores included)
  asm("" : "+v"(v));
  return (int32_t)v;
}

// Stage the LDS image for `MODE` (every thread of the block calls it);
// `scratch_u32` uint32 words of per-block scratch follow the scene image.
template <int MODE>
__device__ __forceinline__ LdsCtx stage_lds(const DeviceScene& sc, uint32_t scratch_u32, uint32_t* spill = nullptr) {
  LdsCtx cx;
  const uint32_t nf4 = node_float4s(sc.width);   // float4s per node
  const uint32_t n_nodes = (MODE == kAllLds) ? scene_nodes(sc) : (MODE == kTopLds ? sc.lds_nodes : 0u);
  const uint32_t TR = (MODE == kAllLds) ? scene_tri_records(sc) : 0u;   // leaf triangles of both trees
  const uint32_t T = (MODE == kAllLds) ? sc.num_triangles : 0u;          // per-primitive records
  const uint32_t M = (MODE == kAllLds) ? sc.num_materials : 0u;
  const uint32_t NL = (MODE == kAllLds) ? sc.num_lights + 1 : 0u;
  cx.n_lds_nodes = n_nodes;
  const uint32_t node_f4 = node_stride_f4(MODE, nf4);
  const bool copies = node_f4 != nf4;
  cx.tri_base = node_f4 * n_nodes;
  cx.prim_base = cx.tri_base + 3 * TR;
  cx.mat_base = cx.prim_base + 6 * T;
  cx.light_base = cx.mat_base + 2 * M;
  const uint32_t f4 = cx.light_base + 7 * NL;
  cx.scratch_base = 4 * f4;
  cx.stack_base = cx.scratch_base + ((scratch_u32 + 3) & ~3u);
  cx.spill_lane = sc.max_stack;
  cx.spill = spill ? spill + (size_t)blockIdx.x * kBlock * cx.spill_lane : nullptr;
  if (MODE != kGlobal) {
    const float4* src[5] = {reinterpret_cast<const float4*>(sc.nodes), reinterpret_cast<const float4*>(sc.tris),
                            reinterpret_cast<const float4*>(sc.prims), reinterpret_cast<const float4*>(sc.materials),
                            reinterpret_cast<const float4*>(sc.lights)};
    const uint32_t base[5] = {0u, cx.tri_base, cx.prim_base, cx.mat_base, cx.light_base};
    const uint32_t len[5] = {nf4 * n_nodes, 3 * TR, 6 * T, 2 * M, 7 * NL};
    for (int r = copies ? 1 : 0; r < 5; ++r)
      for (uint32_t i = threadIdx.x; i < len[r]; i += kBlock) g_lds[base[r] + i] = src[r][i];
    if (copies) {   // quadrant copies: x, y rows (near, far), z rows (lo, hi), refs
      for (uint32_t i = threadIdx.x; i < node_f4 * n_nodes; i += kBlock) {
        const uint32_t node = i / node_f4, rem = i % node_f4;
        const uint32_t quad = rem / kQuadCopyF4, row = rem % kQuadCopyF4;
        const uint32_t axis = row >> 1;
        const uint32_t flip = axis < 2 ? (quad >> axis) & 1u : 0u;
        const uint32_t src_row = row < 6 ? 2 * axis + ((row & 1u) ^ flip) : 6u;
        g_lds[i] = src[0][8 * node + src_row];
      }
    }
    __syncthreads();
  }
  return cx;
}

// ---------------------------------------------------------------------------
// Diagnostic lane statistics (MRT_LANESTATS builds only; never the product):
// per wave, for each traversal loop, the loop iterations and the active lanes
// in them (lane utilisation of that loop = lanes / (64 x iterations)), and the
// lanes entering each phase.  Kept per wave in LDS by the wave's first active
// lane, summed into g_lanes at the wave's exit.  Slots (tools/lane_stats.py):
//   0-5   nearest query: lanes, wave calls, interior iterations, interior
//         lane-steps, leaf iterations, leaf lane-steps
//   6-11  the same for occlusion queries
//   12-13 shading: wave calls, lanes;  14-15 bounce_wave: calls, active lanes
//   16-17 shadow phase: lanes with a shadow ray, wave calls with any
//   18-19 camera-ray candidate lists: wave calls, lanes
//   20-25 path kernel: service rounds, lanes serviced, traversal rounds,
//         lanes traversing in them, lanes refilled, outer iterations
//   26-27 stream kernel: camera iterations, queue-level iterations
// ---------------------------------------------------------------------------
#ifndef MRT_LANESTATS
#define MRT_LANESTATS 0
#endif
#if MRT_LANESTATS
constexpr int kLaneStats = 32;
__shared__ unsigned long long s_lanes[kBlock / 64][kLaneStats];
__device__ unsigned long long g_lanes[kLaneStats];
__device__ __forceinline__ void ls_add(int k, uint32_t v) {
  const uint64_t m = __ballot(1);
  if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((unsigned long long)m) - 1)) s_lanes[threadIdx.x >> 6][k] += v;
}
__device__ __forceinline__ uint32_t ls_lanes() { return (uint32_t)__popcll(__ballot(1)); }
#define LS_ADD(k, v) ls_add((k), (v))
#define LS_INIT() do { if ((threadIdx.x & 63u) < (uint32_t)kLaneStats) s_lanes[threadIdx.x >> 6][threadIdx.x & 63u] = 0; } while (0)
#define LS_FLUSH() do { const uint32_t l_ = threadIdx.x & 63u; \
    if (l_ < (uint32_t)kLaneStats && s_lanes[threadIdx.x >> 6][l_]) atomicAdd(&g_lanes[l_], s_lanes[threadIdx.x >> 6][l_]); } while (0)
#else
#define LS_ADD(k, v) do {} while (0)
#define LS_INIT() do {} while (0)
#define LS_FLUSH() do {} while (0)
#endif

// While-while traversal with postponed leaves (Aila & Laine 2009, recast for
// 64-lane waves): a lane that reaches a leaf parks it and keeps descending
// interior nodes until every lane of the wave holds a leaf, then the wave
// tests leaves together — interior and leaf work are not interleaved lane by
// lane.  The per-lane stack is in LDS (entries beyond STACK spill to global
// memory); kDone marks an empty stack.
// ANY = false: nearest hit in [tmin, h.t]; ties -> lowest primitive index.
// ANY = true:  stop at the first primitive k != target with (t_k, k) <
//              (t_target, target) in [0, t_target] (shadow occlusion).
// Both results are independent of the visiting order, so every tree (host
// SAH, device LBVH / PLOC) returns the same (brute-force) answer.
constexpr int32_t kDone = 0x7FFFFFFF;   // empty-stack marker
// Traversal slack: the interior loop of a while-while round ends once at
// most this many lanes still seek a leaf, instead of waiting for the last
// one (the lanes holding a leaf test it; the others resume next round).  The
// path kernel's rounds are resumable anyway, and in deep global-memory trees
// the last lanes' descents are long: slack 12 (of 64) measured C4 1950 ->
// 2497 Mpaths/s (+28 %), C3 +7.5 %, C3g +5 %, C5 1/8 share +28 % (8 / 16 /
// 24 / 32 / 48: C4 2456 / 2488 / 2397 / 2281 / 1904).  Shallow all-in-LDS
// trees lose by it (C2, the stream kernel: slack 2 -1.3 %, 8 -3.4 %).
// r4, with the inline shadow finishes (service 32): path slack 8 / 12 / 16
// C4 2769 / 2852 / 2873, C3 2530 / 2616 / 2660; leaf slack 4 / 8 / 12 C4
// 2795 / 2852 / 2869, C3 2574 / 2616 / 2638 (one call, alternating)
#ifndef MRT_PATH_SLACK   // trav_round(): the path kernel
#define MRT_PATH_SLACK 16
#endif
#ifndef MRT_LEAF_SLACK   // trav_round(): the leaf loop's (a kept leaf is tested next round):
#define MRT_LEAF_SLACK 12 // r3, path slack 12: C4 2480 -> 2645 (+6.7 %), C3 2340 -> 2474 (+5.7 %);
#endif                   // 2 / 4 / 12 / 16 / 24 / 32: C4 2577 / 2605 / 2645 / 2640 / 2623 / 2611

template <int STACK>
__device__ __forceinline__ int32_t stack_pop(const LdsCtx& cx, int& sp) {
  // LDS + spill stacks: a plain LDS pop when no active lane's top entry is
  // in the spill area (wave-uniform test)
  if (STACK < 0 && !__any(sp > (STACK < 0 ? -STACK : STACK))) {
    const int32_t n = sp > 0 ? (int32_t)lds_u32()[cx.stack_base + threadIdx.x + (sp - 1) * kBlock] : kDone;
    sp = max(sp - 1, 0);
    return n;
  }
  const int32_t n = sp > 0 ? stack_get<STACK>(cx, sp - 1) : kDone;
  sp = max(sp - 1, 0);
  return n;
}

// One interior node: returns the next node to visit (nearest hit child, or a
// popped entry, or kDone); the other hit children are pushed far-to-near.
// Culling slack: a child is culled only when its entry lies beyond the
// current h.t by more than 2^-11 of it.  Box padding (bvh.cpp) is relative to
// the box's own coordinates, but the ray-triangle test's t error is relative
// to the ray's distance and grows for tiny or slanted triangles: on the
// 1M-triangle mesh (1e-3-sized triangles near x, z = 0) a test returned t
// 1.5e-5 before the padded box's entry, so whether that triangle was found
// depended on whether a farther hit had shortened h.t first — i.e. on the
// lane's visiting order, which the slack rounds make timing-dependent (C5:
// one pixel in 8.3 M differed between identical runs).  Visiting
// the few boxes just behind h.t makes the answer the brute-force one again in
// such cases (it never changes an answer: the leaf tests' t <= h.t rule
// decides).
[[maybe_unused]] constexpr float kCullScale = 1.0f + 0x1p-11f;
template <int STACK, int MODE, bool ANY>
__device__ __forceinline__ int32_t interior_step(const DeviceScene& sc, const LdsCtx& cx, int32_t node, V3 o,
                                                 const RayBox& rb, float tmin, float tmax, int& sp) {
  {
    float t[4];
    int32_t r[4];
    {
      float4 q[7];
      fetch_node4<MODE>(sc, cx, node, rb, q);
      tmax *= kCullScale;   // +inf stays +inf
      box4<MODE == kGlobal ? 0 : 3, MODE != kTopLds>(q, o, rb, tmin, tmax, t);
      r[0] = (int32_t)fbits(q[6].x); r[1] = (int32_t)fbits(q[6].y); r[2] = (int32_t)fbits(q[6].z); r[3] = (int32_t)fbits(q[6].w);
    }
    const float inf = __builtin_inff();
    // near-to-far order for occlusion rays too: measured +2.5 % (C2, r1) and
    // +4.5 % (C4) over slot order — near children hold the likely occluders
    // 4-input sorting network on (t, ref); misses (+inf) sink to the end
#define MRT_CE(i, j)                                      \
    {                                                     \
      const bool sw_ = t[j] < t[i];                       \
      const float ti_ = sw_ ? t[j] : t[i];                \
      const int32_t ri_ = sw_ ? r[j] : r[i];              \
      t[j] = sw_ ? t[i] : t[j];                           \
      r[j] = sw_ ? r[i] : r[j];                           \
      t[i] = ti_;                                         \
      r[i] = ri_;                                         \
    }
    if (MODE != kAllLds) {
      MRT_CE(0, 1) MRT_CE(2, 3) MRT_CE(0, 2) MRT_CE(1, 3) MRT_CE(1, 2)
    } else {
      // all-in-LDS trees: only the nearest hit child is picked, the others
      // are pushed in slot order — the full sort's 10 more VALU ops per node
      // cost more than the better pop order saves in a shallow tree (C2:
      // occlusion queries +0.5 %, 9661 / 9646 vs 9587 / 9613; nearest
      // queries too, another +2.8 %, 9895 / 9898 vs 9630 / 9635).
      // Global-memory trees keep the full sort (C4 = for occlusion).
      MRT_CE(0, 1) MRT_CE(0, 2) MRT_CE(0, 3)
    }
#undef MRT_CE
    // LDS + spill stacks (deep trees): when no lane of the wave can reach
    // the spill area in this step (sp + 3 <= LDS entries, wave-uniform),
    // the pushes and the pop are plain LDS accesses — no per-entry
    // LDS-or-spill branches (their exec-mask bookkeeping was ~40 of the ~250
    // instructions of a global-tree interior step)
    if (STACK < 0 && !__any(sp + 3 > (STACK < 0 ? -STACK : STACK))) {
      constexpr int kL = STACK < 0 ? -STACK : STACK;
      uint32_t* st = lds_u32() + cx.stack_base + threadIdx.x;
      if (t[3] < inf) { st[sp * kBlock] = (uint32_t)r[3]; ++sp; }
      if (t[2] < inf) { st[sp * kBlock] = (uint32_t)r[2]; ++sp; }
      if (t[1] < inf) { st[sp * kBlock] = (uint32_t)r[1]; ++sp; }
      int32_t next = r[0];
      if (!(t[0] < inf)) {
        next = sp > 0 ? (int32_t)st[(sp - 1) * kBlock] : kDone;
        sp = max(sp - 1, 0);
      }
      (void)kL;
      return next;
    }
    {
      if (t[3] < inf) { stack_push<STACK>(cx, sp, r[3]); ++sp; }
      if (t[2] < inf) { stack_push<STACK>(cx, sp, r[2]); ++sp; }
      if (t[1] < inf) { stack_push<STACK>(cx, sp, r[1]); ++sp; }
    }
    int32_t next = r[0];
    if (!(t[0] < inf)) next = stack_pop<STACK>(cx, sp);
    return next;
  }
}

// The triangles [first, first + cnt) of a leaf in index order, two at a time
// with both triangles' loads issued before either test (one memory or LDS
// round trip per pair; C4 +8 % with the flat-load fix below, C2 +3.9 % for
// LDS-resident leaves).  Nearest (any = false): updates h (ties ->
// lowest primitive index; (u, v) to uv[0], uv[kBlock] when uv is non-null).
// Occlusion (any = true): true at the first primitive k != target with
// (t_k, k) < (h.t, target).
// Leaf-ordered triangles ka and kb (kb tested only when `pair`), both loaded
// before either test.
template <int MODE>
__device__ __forceinline__ bool tri_pair(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, float tmin,
                                         uint32_t ka, uint32_t kb, bool pair, Hit& h, bool any, uint32_t target,
                                         uint32_t* uv) {
  float4 a0, a1, a2, b0, b1, b2;
  fetch_tri<MODE>(sc, cx, ka, a0, a1, a2);
  fetch_tri<MODE>(sc, cx, kb, b0, b1, b2);
  float t[2], u[2], v[2];
  bool ok[2];
  ok[0] = tri_bary(o, d, mk(a0), mk(a1), mk(a2), t[0], u[0], v[0]);
  ok[1] = tri_bary(o, d, mk(b0), mk(b1), mk(b2), t[1], u[1], v[1]) & pair;
  const uint32_t prim[2] = {fbits(a0.w), fbits(b0.w)};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool hit = ok[j] & (t[j] >= tmin) & (t[j] <= h.t);
    if (any) {
      if (hit & (prim[j] != target) & ((t[j] < h.t) | (prim[j] < target))) return true;
    } else if (hit & (!h.found | (t[j] < h.t) | (prim[j] < h.prim))) {
      h.found = true;
      h.t = t[j];
      if (uv) {
        uv[0] = fbits(u[j]);
        uv[kBlock] = fbits(v[j]);
      } else {
        h.u = u[j];
        h.v = v[j];
      }
      h.prim = prim[j];
    }
  }
  return false;
}

template <int MODE>
__device__ __forceinline__ bool leaf_tests(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, float tmin,
                                           uint32_t first, uint32_t cnt, Hit& h, bool any, uint32_t target,
                                           uint32_t* uv) {
  for (uint32_t k = 0; k < cnt; k += 2) {
    const uint32_t k1 = min(k + 1, cnt - 1);
    if (tri_pair<MODE>(sc, cx, o, d, tmin, first + k, first + k1, k1 != k, h, any, target, uv)) return true;
  }
  return false;
}

// Camera rays of one 8x8 pixel block through the block's candidate list
// (primary.h): the nearest hit over the listed triangles with the leaf test's
// arithmetic and tie rule — the traversal's answer, since the list holds
// every triangle a ray of the block can hit.  `list` / `cnt` are
// wave-uniform (scalar loads; LDS-resident triangles are broadcast reads).
template <int MODE>
__device__ __forceinline__ void primary_nearest(const DeviceScene& sc, const LdsCtx& cx, const uint32_t* list,
                                                uint32_t cnt, V3 o, V3 d, Hit& h) {
  h.t = __builtin_inff();
  h.u = h.v = 0.0f;
  h.prim = 0xFFFFFFFFu;
  h.found = false;
  for (uint32_t j = 0; j < cnt; j += 2) {
    const uint32_t j1 = min(j + 1, cnt - 1);
    tri_pair<MODE>(sc, cx, o, d, 0.0f, list[j], list[j1], j1 != j, h, false, 0u, nullptr);
  }
}

template <int STACK, int MODE, bool ANY>
__device__ __forceinline__ bool traverse(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, float tmin, Hit& h,
                                         uint32_t target, int32_t root) {
  const RayBox rb = make_raybox(o, d);
  int32_t node = root, leaf = 0;
  int sp = 0;
  constexpr int kLs = ANY ? 6 : 0;
  (void)kLs;
  LS_ADD(kLs + 0, ls_lanes());
  LS_ADD(kLs + 1, 1);
  if (node < 0) { leaf = node; node = kDone; }
  while (node != kDone || leaf != 0) {
    // interior nodes
    while (node != kDone && node >= 0) {
      LS_ADD(kLs + 2, 1);
      LS_ADD(kLs + 3, ls_lanes());
      node = interior_step<STACK, MODE, ANY>(sc, cx, node, o, rb, tmin, h.t, sp);
      if (node < 0 && leaf == 0) {   // park the leaf, keep descending
        leaf = node;
        node = stack_pop<STACK>(cx, sp);
      }
      if (__ballot(leaf == 0) == 0ull) break;
    }
    // leaves
    while (leaf < 0) {
      LS_ADD(kLs + 4, 1);
      LS_ADD(kLs + 5, ls_lanes());
      const uint32_t lr = ~(uint32_t)leaf;
      const uint32_t first = lr >> kLeafCountBits, cnt = (lr & (kMaxLeafSize - 1)) + 1;
      if (leaf_tests<MODE>(sc, cx, o, d, tmin, first, cnt, h, ANY, target, nullptr)) return true;
      leaf = 0;
      if (node < 0) {   // the next node is a leaf too: take it now
        leaf = node;
        node = stack_pop<STACK>(cx, sp);
      }
    }
  }
  return false;
}


template <int STACK, int MODE>
__device__ __forceinline__ Hit trace_nearest(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, float tmin,
                                             float tmax) {
  Hit h;
  h.t = tmax;
  h.u = h.v = 0.0f;
  h.prim = 0xFFFFFFFFu;
  h.found = false;
  traverse<STACK, MODE, false>(sc, cx, o, d, tmin, h, 0u, sc.root);
  return h;
}

// The tree a shadow ray from o traverses: the occluder tree when o is inside
// every culled plane by the margin (occluders.h: no triangle of those planes
// can then stand between o and a light) and the ray does not graze the
// light's plane (`graze`: cosine below occ_cos_min, where the light's own t
// error could reach a culled crossing), else the main tree.  The plane data
// is wave-uniform (kernel argument, scalar registers).
__device__ __forceinline__ int32_t shadow_root(const DeviceScene& sc, V3 o, bool graze) {
  if (sc.occ_planes == 0 || graze) return sc.root;
  bool inside = true;
  for (uint32_t k = 0; k < sc.occ_planes; ++k) {
    const float* p = sc.occ_plane[k];
    inside &= fmaf(p[0], o.x, fmaf(p[1], o.y, fmaf(p[2], o.z, -p[3]))) <= -sc.occ_margin;
  }
  return inside ? sc.occ_root : sc.root;
}

// The light triangles of an occluder tree built without them (DeviceScene::
// occ_lights): every shadow ray enters the light's own leaf box, so instead
// of a leaf visit per ray the other light triangles are tested here in one
// wave-uniform loop — the leaf test's arithmetic (a light record's vertices
// are its primitive's, in its order: v2 - v1, v3 - v1 are the leaf record's
// e1, e2 bit for bit, as in last_bounce_light_hit) and the occlusion rule
// (k != target, (t_k, k) < (t_T, target), t_k >= 0), so the query's answer
// is unchanged — bit for bit in the precise build; in the fast build the
// compiler may contract this inlined tri_bary differently from the leaf
// loop's (as origin_occludes), so a near-tie can flip within the 1e-2 gate.
// `tl` = the target's light index (its shading record's p1.w): the loop runs
// num_lights - 1 times, lane by lane over every light but the target (whose
// test the occlusion rule always rejected) — r6: one test instead of two per
// C2 shadow ray.
template <int MODE>
__device__ __forceinline__ bool lights_occlude(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t target,
                                               uint32_t tl, float tT) {
  bool occ = false;
  for (uint32_t j = 0; j + 1 < sc.num_lights; ++j) {   // wave-uniform trip count
    const uint32_t k = j < tl ? j : j + 1u;            // per lane: the j-th light other than the target
    const float4 LB = fetch_light<MODE>(sc, cx, k, 1), LD = fetch_light<MODE>(sc, cx, k, 3);
    const float4 LF = fetch_light<MODE>(sc, cx, k, 5);
    const uint32_t prim = fbits(LD.w);
    const V3 p0 = mk(LB);
    float t, u, v;
    const bool ok = tri_bary(o, d, p0, sub(mk(LD), p0), sub(mk(LF), p0), t, u, v);
    occ |= ok & (prim != target) & (t >= 0.0f) & (t <= tT) & ((t < tT) | (prim < target));
  }
  return occ;
}

// One face's triangles (conv_face_tris: two primitive ids, 0xFFFF = none)
// under the leaf test's arithmetic and occlusion rule, as lights_occlude.
template <int MODE>
__device__ __forceinline__ bool face_occludes(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t pair,
                                              uint32_t target, float tT) {
  bool occ = false;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t prim = (pair >> (16 * j)) & 0xFFFFu;
    if (prim != 0xFFFFu) {
      const V3 p0 = mk(fetch_prim<MODE>(sc, cx, prim, 0)), p1 = mk(fetch_prim<MODE>(sc, cx, prim, 1));
      const V3 p2 = mk(fetch_prim<MODE>(sc, cx, prim, 2));
      float t, u, v;
      const bool ok = tri_bary(o, d, p0, sub(p1, p0), sub(p2, p0), t, u, v);
      occ |= ok & (prim != target) & (t >= 0.0f) & (t <= tT) & ((t < tT) | (prim < target));
    }
  }
  return occ;
}

// Convex occluders (r6, occluders.h ConvexSet): the occlusion walk of the
// light samples was ~24 % of the C2 stream kernel (ablation MRT_DEBUG=32:
// 11.07 -> 8.45 ms per launch), paid per wave for its longest lane.  When
// every triangle of the occluder tree lies on a convex solid (the Cornell
// box's two blocks), a lane decides each solid in straight-line code:
//   * the segment [o, o + t_T d] against the solid's three bounding slabs
//     pushed out by delta (16x the BVH boxes' padding); an empty interval
//     means no triangle of the solid can report a hit — the padded-volume
//     argument the BVH's own culling rests on, with a wider margin;
//   * a ray from a face of a solid (the origin primitive's shading record:
//     p2.w = its face code, n0.w..n2.w = the face's outward unit normal n)
//     with d . n >= kConvexLeaveDot (1e-3) skips that solid: n's plane
//     supports the convex solid and the origin is ~1e-4 outside it (x >=
//     0.999, the flat shading normal's cosine to n, occluders.cpp), so the
//     segment moves away from the solid.  The leaf test's error is what
//     bounds the threshold: a ray grazing an adjacent face's plane near the
//     shared edge gets barycentrics off by ~u |s| |e| / (|cos| area), so over
//     3 M adversarial grazing rays from the blocks' faces (70 % within
//     1e-1 ... 1e-6 of an edge, tilted 1e-1 ... 1e-8 off the face) the largest
//     d . n of a ray that hits its own solid was 1.0e-5 (IEEE) / -4.2e-5
//     (FMA): 100x below the threshold (tests/test_convex_occluders.py).
//     (r6; before, the slab pair's axis normal with d . n >= 0.01: grazing
//     rays off a block's own face then fell through to the exhaustive test
//     of its other faces, in 15-20 % of C2's shadow waves at bounces >= 1);
//   * otherwise the face the segment enters the padded solid through (or, from
//     inside it, leaves it through) has its triangles leaf-tested with the
//     occlusion rule: a hit is the traversal's own answer ("occluded"); if
//     it does not hit, the face the segment leaves through, and then the
//     solid's other faces — the leaf test over every triangle of the solid,
//     which is what the walk would have tested.
// Returns whether a solid occludes; the occluder tree is not walked.
template <int MODE>
__device__ __forceinline__ bool convex_occlusion(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t target,
                                                 float tT, uint32_t origin) {
  const uint32_t own = fbits(fetch_prim<MODE>(sc, cx, origin, 2).w);   // c * 8 + face + 1 of the origin's solid
  const V3 own_n = mk(fetch_prim<MODE>(sc, cx, origin, 3).w, fetch_prim<MODE>(sc, cx, origin, 4).w,
                      fetch_prim<MODE>(sc, cx, origin, 5).w);   // its face's outward unit normal (0 off the solids)
  const uint32_t own_skip = ((own != 0u) & (dot(d, own_n) >= kConvexLeaveDot)) ? (own - 1u) >> 3 : 0xFFFFFFFFu;
  bool occluded = false;
  for (uint32_t c = 0; c < sc.conv_count; ++c) {   // wave-uniform; the three slabs unrolled (scalar operands)
    const float* B = sc.conv_obb[c];
    float t0 = 0.0f, t1 = tT;
    uint32_t fin = 8u, fout = 8u;   // entry / exit face (2a + side); 8 = none
#pragma unroll
    for (uint32_t a = 0; a < 3; ++a) {
      const float nd = (B[3 * a] * d.x + B[3 * a + 1] * d.y) + B[3 * a + 2] * d.z;
      const float no = (B[3 * a] * o.x + B[3 * a + 1] * o.y) + B[3 * a + 2] * o.z;
      const float inv = m_rcp(nd);
      const float tlo = (B[9 + 2 * a] - no) * inv, thi = (B[10 + 2 * a] - no) * inv;
      // along +n (the sign bit, so that nd = -0 pairs with inv = -inf): enters
      // through the lo face, leaves through the hi face; parallel rays get
      // (-inf, +inf) inside the slab, an empty interval outside, and NaN (no
      // constraint, the conservative side) exactly on a slab plane
      const bool pos = (fbits(nd) >> 31) == 0u;
      const float tn = pos ? tlo : thi, tf = pos ? thi : tlo;
      const bool in_ = tn > t0, out_ = tf < t1;
      t0 = in_ ? tn : t0;
      fin = in_ ? (pos ? 2u * a : 2u * a + 1u) : fin;
      t1 = out_ ? tf : t1;
      fout = out_ ? (pos ? 2u * a + 1u : 2u * a) : fout;
    }
    const bool leaves_own = own_skip == c;
    if ((t0 <= t1) & !leaves_own & !occluded) {
      uint32_t pin = 0xFFFFFFFFu, pout = 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t k = 0; k < 6; ++k) {
        pin = fin == k ? sc.conv_face_tris[c][k] : pin;
        pout = fout == k ? sc.conv_face_tris[c][k] : pout;
      }
      bool hit = face_occludes<MODE>(sc, cx, o, d, pin != 0xFFFFFFFFu ? pin : pout, target, tT);
      if (!hit & (pin != 0xFFFFFFFFu)) hit = face_occludes<MODE>(sc, cx, o, d, pout, target, tT);
      // neither face certifies (a near miss within delta, or an entry through
      // another face near an edge): the solid's other faces, which makes the
      // lane's answer the leaf test over every triangle of the solid
      if (!hit) {
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k)
          if (!hit & (k != fin) & (k != fout)) hit = face_occludes<MODE>(sc, cx, o, d, sc.conv_face_tris[c][k], target, tT);
      }
      occluded |= hit;
    }
  }
  return occluded;
}

template <int STACK, int MODE>
__device__ __forceinline__ bool trace_occluded(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t target,
                                               uint32_t tl, float t_target, bool graze, uint32_t origin,
                                               uint32_t dbg = 0u) {
  Hit h;
  h.t = t_target;
  h.found = false;
  int32_t root = shadow_root(sc, o, graze);
  const bool via_occ = root == sc.occ_root;
  if (sc.conv_count && via_occ) {
    if (!(dbg & 512u) && convex_occlusion<MODE>(sc, cx, o, d, target, t_target, origin)) return true;
    root = kDone;   // no walk (the light triangles are still tested below)
  }
  if (sc.occ_lights && via_occ && !(dbg & 1024u) && lights_occlude<MODE>(sc, cx, o, d, target, tl, t_target)) return true;
  return traverse<STACK, MODE, true>(sc, cx, o, d, 0.0f, h, target, root);
}

// The shadow ray's own surface first (exact early-out, r4).  The occlusion
// query answers "occluded" as soon as ANY primitive k != target passes the
// leaf test with (t_k, k) < (t_T, target) in [0, t_T]; the triangle the ray
// leaves is such a k whenever the light lies behind that triangle's plane
// (the ray re-crosses the surface ~1e-4 from its origin: about half of a
// closed mesh's shadow rays, each of which would otherwise descend the tree
// to the origin's own leaf).  It is tested with the leaf test's arithmetic
// (tri_bary over the shading record's vertices: the leaf record's v0,
// e1 = v1 - v0, e2 = v2 - v0 are the same float operations, bvh.cpp) and its
// acceptance rule, so "occluded" here is the traversal's answer and
// "not occluded" changes nothing — bit-exactly in the precise build (no FMA
// contraction).  In the fast build (-ffp-contract=fast) the compiler may fuse
// this inlined copy of tri_bary differently from the leaf loop's, so on a
// near-tie (t within an ulp of t_T or 0) the two can disagree; the fast
// build's 1e-2 image gate covers such flips.  Scenes of >= kOriginTestTriangles only
// (DeviceScene::origin_test).
// the last bounce's occlusion query of a light hit through the occluder tree
// (shadow_root) instead of the main tree
template <int MODE>
__device__ __forceinline__ bool origin_occludes(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t prim,
                                                uint32_t target, float tT) {
  if (!sc.origin_test) return false;   // wave-uniform (kernel argument)
  const V3 p0 = mk(fetch_prim<MODE>(sc, cx, prim, 0)), p1 = mk(fetch_prim<MODE>(sc, cx, prim, 1));
  const V3 p2 = mk(fetch_prim<MODE>(sc, cx, prim, 2));
  float t, u, v;
  const bool ok = tri_bary(o, d, p0, sub(p1, p0), sub(p2, p0), t, u, v);
  return ok & (prim != target) & (t >= 0.0f) & (t <= tT) & ((t < tT) | (prim < target));
}

// Shadow-ray resolve under MPS nearest-hit semantics + lightSamplingHandler
// (renderer/Shaders.metal:214-231): contributes iff the nearest hit of the
// shadow ray (tmin 0, tmax inf) is the target triangle at t >= 1e-4.
// `origin` = the primitive the ray leaves (origin_occludes).
template <int STACK, int MODE>
__device__ bool shadow_reaches_target(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, uint32_t target,
                                      uint32_t origin, bool graze, uint32_t dbg = 0u) {
  const float4 P1 = fetch_prim<MODE>(sc, cx, target, 1);   // .w: the target's light index
  const V3 p0 = mk(fetch_prim<MODE>(sc, cx, target, 0)), p1 = mk(P1);
  const V3 p2 = mk(fetch_prim<MODE>(sc, cx, target, 2));
  float tT, u, v;
  if (!tri_test(o, d, p0, sub(p1, p0), sub(p2, p0), 0.0f, __builtin_inff(), tT, u, v)) return false;
  if (!(tT >= kDistanceEpsilon)) return false;
  if (!(dbg & 128u) && origin_occludes<MODE>(sc, cx, o, d, origin, target, tT)) return false;
  if (dbg & 32u) return true;   // ablation: no occlusion traversal
  return !trace_occluded<STACK, MODE>(sc, cx, o, d, target, fbits(P1.w), tT, graze, origin, dbg);
}

// Last bounce (bounce + 1 == MAX_PATH_LENGTH): intersectionHandler adds no
// light sample and makes no next ray there (Shaders.metal:150,199), so the
// nearest hit matters only if it is an emitter — every emitter is a light
// triangle (scene flattening) — and only through its emission.  So the
// nearest query becomes: the nearest (t, prim) over the light triangles
// alone (leaf-test arithmetic and tie rule over their shading records), then
// — if one is hit at t >= 1e-4 — the occlusion query "does any other
// triangle k beat it, (t_k, k) < (t_L, L)" (the shadow query's any-hit
// traversal).  Not beaten: the nearest hit is that light (emission follows
// as before); beaten, missed, or nearer than 1e-4: no emission, which is
// all the reference's nearest hit could add.  Exact (precise build
// bitwise); scenes with <= kLightShortcutMax light triangles
// (DeviceScene::light_shortcut), not with DEBUG_MATERIAL (which shades
// every hit).  Returns true when the occlusion query is still to run (h
// holds the light hit); false: h.found says whether there is emission.
// Measured (r4, alternating in one call): C2 (stream kernel) 9738 / 9743 ->
// 10772 / 10778 Mpaths/s (+10.6 %); the path kernel keeps the full query
// (its variant measured C4 -1.3 %, C3 -3.4 %, removed in r6).
// `graze`: the hit light's cosine to the ray is below the occluder tree's
// guard (shadow_root; |d . n| / |n| over the geometric normal n = e1 x e2,
// which occluders.cpp's cos_min covers as it covers the interpolated normal).
template <int MODE>
__device__ __forceinline__ bool last_bounce_light_hit(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, Hit& h,
                                                      bool& graze) {
  h.t = __builtin_inff();
  h.u = h.v = 0.0f;
  h.prim = 0xFFFFFFFFu;
  h.found = false;
  float gd = 0.0f, gn = 1.0f;   // the nearest light's (d . n)^2 and n . n
  for (uint32_t k = 0; k < sc.num_lights; ++k) {   // wave-uniform
    // the light record's vertices are the primitive's, in its order
    // (scene flattening, Renderer.mm:394-413): three independent loads, and
    // v2 - v1, v3 - v1 are the leaf record's e1, e2 bit for bit
    const float4 LB = fetch_light<MODE>(sc, cx, k, 1), LD = fetch_light<MODE>(sc, cx, k, 3);
    const float4 LF = fetch_light<MODE>(sc, cx, k, 5);
    const uint32_t prim = fbits(LD.w);   // lights[k].index
    const V3 p0 = mk(LB), e1 = sub(mk(LD), p0), e2 = sub(mk(LF), p0);
    float t, u, v;
    const bool ok = tri_bary(o, d, p0, e1, e2, t, u, v);
    const bool hit = ok & (t >= 0.0f) & (t <= h.t);
    if (hit & (!h.found | (t < h.t) | (prim < h.prim))) {
      h.found = true;
      h.t = t;
      h.u = u;
      h.v = v;
      h.prim = prim;
      const V3 n = tcross(e1, e2);
      const float dn = tdot(d, n);
      gd = dn * dn;
      gn = tdot(n, n);
    }
  }
  if (h.found && h.t < kDistanceEpsilon) h.found = false;   // no emission whatever is nearer
  graze = !(gd >= sc.occ_cos_min2 * gn);
  return h.found;
}

// ---------------------------------------------------------------------------
// Shading helpers — renderer/KernelHelpers.h, renderer/Raytracing.h
// ---------------------------------------------------------------------------
// fresnel — KernelHelpers.h:7-21
__device__ __forceinline__ float fresnel(V3 n, V3 i, float etaOut, float etaIn) {
  float result = 1.0f;
  const float etaScale = m_div(etaOut, etaIn);
  const float cosThetaI = fminf(fmaxf(dot(n, i), -1.0f), 1.0f);
  const float sinThetaTSquared = (etaScale * etaScale) * (1.0f - cosThetaI * cosThetaI);
  if (sinThetaTSquared < 1.0f) {
    const float cosThetaT = m_sqrt(1.0f - sinThetaTSquared);
    const float rS = m_div(etaIn * cosThetaI - etaOut * cosThetaT, etaIn * cosThetaI + etaOut * cosThetaT);
    const float rP = m_div(etaIn * cosThetaT - etaOut * cosThetaI, etaIn * cosThetaT + etaOut * cosThetaI);
    result = 0.5f * (rS * rS + rP * rP);
  }
  return result;
}
// triangleSamplePDF — Raytracing.h:168-171
__device__ __forceinline__ float triangleSamplePDF(float area, float cosTheta, float dist) {
  return m_div(dist * dist, area * cosTheta);
}
// balanceHeuristic (power heuristic) — Raytracing.h:173-178
__device__ __forceinline__ float balanceHeuristic(float f, float g) {
  const float f2 = f * f, g2 = g * g;
  return m_div(f2, f2 + g2);
}
// buildOrthonormalBasis — Raytracing.h:189-205
__device__ __forceinline__ void buildOrthonormalBasis(V3 n, V3& u, V3& v) {
  if (n.z < 0.0f) {
    const float a = m_rcp(1.0f - n.z);
    const float b = n.x * n.y * a;
    u = mk(1.0f - n.x * n.x * a, -b, n.x);
    v = mk(b, n.y * n.y * a - 1.0f, -n.y);
  } else {
    const float a = m_rcp(1.0f + n.z);
    const float b = -n.x * n.y * a;
    u = mk(1.0f - n.x * n.x * a, b, -n.x);
    v = mk(b, 1.0f - n.y * n.y * a, -n.y);
  }
}
// generateDiffuseBounce + alignWithNormal — Raytracing.h:207-223 (smp = noise.zw)
__device__ __forceinline__ V3 diffuseBounce(float sx, float sy, V3 n) {
  const float cosTheta = m_sqrt(sy);
  const float phi = sx * kPi * 2.0f;
  const float sinTheta = m_sqrt(1.0f - cosTheta * cosTheta);
  V3 u, v;
  buildOrthonormalBasis(n, u, v);
  const float cp = m_cos(phi), sp = m_sin(phi);
  return add(mul(add(mul(u, cp), mul(v, sp)), sinTheta), mul(n, cosTheta));
}
__device__ __forceinline__ bool isMirrorDir(V3 wI, V3 n, V3 wO) {
  return fabsf(dot(reflect(wI, n), wO) - 1.0f) < kAngleEpsilon;
}

struct Mat {
  V3 kd, le;
  float ior;
  uint32_t type;
};
template <int MODE>
__device__ __forceinline__ Mat load_material(const DeviceScene& sc, const LdsCtx& cx, uint32_t m) {
  const float4 a = fetch_mat<MODE>(sc, cx, m, 0), b = fetch_mat<MODE>(sc, cx, m, 1);
  return {mk(a), mk(b), a.w, fbits(b.w)};
}

// sampleMaterial — KernelHelpers.h:56-114
__device__ __forceinline__ void sampleMaterial(const Mat& m, V3 wI, V3 wO, V3 n, const float4& ns, float& bsdf,
                                               float& pdf) {
  const float cosTheta = dot(wO, n);
  constexpr float invPi = 1.0f / kPi;
  bool diffuse_lobe = (m.type == kDiffuse);
  bool zero_lobe = false;
  if (m.type == kPlastic || m.type == kDielectric) {
    const float fI = fresnel(n, neg(wI), 1.0f, m.ior);
    if (fI < ns.y) {
      diffuse_lobe = (m.type == kPlastic);
      zero_lobe = (m.type == kDielectric);
    }
  }
  if (zero_lobe) {
    bsdf = pdf = 0.0f;
  } else if (diffuse_lobe) {
    bsdf = pdf = invPi * cosTheta;
  } else {   // mirror lobe
    bsdf = isMirrorDir(wI, n, wO) ? cosTheta : 0.0f;
    pdf = 1.0f;
  }
}

// generateNextBounce — KernelHelpers.h:116-179
__device__ __forceinline__ V3 generateNextBounce(const Mat& m, V3 wI, float currentIoR, V3 n, const float4& ns,
                                                 float& bsdf, float& pdf, float& ior) {
  constexpr float invPi = 1.0f / kPi;
  ior = currentIoR;
  int lobe = 0;   // 0 diffuse, 1 mirror, 2 pass-through
  if (m.type == kMirror) {
    lobe = 1;
  } else if (m.type == kPlastic || m.type == kDielectric) {
    const float fI = fresnel(n, neg(wI), currentIoR, m.ior);
    lobe = (fI < ns.y) ? (m.type == kPlastic ? 0 : 2) : 1;
  }
  V3 wO;
  if (lobe == 0) {
    wO = diffuseBounce(ns.z, ns.w, n);
    bsdf = pdf = invPi * dot(wO, n);
  } else if (lobe == 1) {
    wO = reflect(wI, n);
    bsdf = dot(wO, n);
    pdf = 1.0f;
  } else {
    ior = m.ior;
    wO = wI;
    bsdf = pdf = 1.0f;
  }
  return wO;
}

// lightTriangleSamplePDF — KernelHelpers.h:181-190
__device__ __forceinline__ float lightTriangleSamplePDF(float tpdf, float area, V3 source, V3 sv, V3 sn,
                                                        V3& dirOut, float& LdotD) {
  const V3 d = sub(sv, source);
  const float dist = length(d);
  dirOut = normalize(d);
  LdotD = -dot(dirOut, sn);
  const float valid = float(dist >= kDistanceEpsilon) * float(LdotD >= kAngleEpsilon);
  return valid * tpdf * triangleSamplePDF(area, LdotD, dist);
}

// selectLightTriangle — KernelHelpers.h:49-54.  The linear scan returns the
// first index with !(cdf[index+1] <= xi) (or count); cdf is non-decreasing, so
// a binary search returns the same index.
template <int MODE>
__device__ __forceinline__ uint32_t selectLightTriangle(const DeviceScene& sc, const LdsCtx& cx, uint32_t count,
                                                        float xi) {
  uint32_t lo = 0, hi = count;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (fetch_light<MODE>(sc, cx, mid + 1, 2).w <= xi) lo = mid + 1;   // entry mid+1: (v1.n, cdf)
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------------------
// Path state + the per-hit shading of intersectionHandler
// ---------------------------------------------------------------------------
struct PathState {
  V3 o, d, T, R;
  float pdf;          // Ray.params.x
  float ior;          // Ray.params.w
  float prevDiffuse;  // Ray.params.y (0 or 1)
  uint32_t mtype;     // material type of the surface the next ray leaves (set with the next ray)
};
struct ShadowRay {
  V3 o, d, L;
  uint32_t target;
  bool valid;
  bool graze;   // cosine to the light below the occluder tree's guard (shadow_root)
};

// rayGenerator — renderer/Shaders.metal:75-103 (camera fixed at t = 0)
__device__ __forceinline__ void camera_ray(uint32_t x, uint32_t y, uint32_t W, uint32_t H, const float4& ns,
                                           V3& o, V3& d) {
  const float aspect = m_div(float(H), float(W));
  const float wm1 = float(W - 1), hm1 = float(H - 1);
  const float dudvx = m_div(ns.x * 2.0f - 1.0f, wm1);
  const float dudvy = m_div(ns.y * 2.0f - 1.0f, hm1);
  const float ncx = m_div(float(2 * x), wm1) - 1.0f;
  const float ncy = m_div(float(2 * y), hm1) - 1.0f;
  d = normalize(mk(dudvx + ncx, dudvy + ncy * aspect, -1.0f));
  o = mk(kCameraX, kCameraY, kCameraZ);   // up - view * 2.35
}

// Owned slots: slot s of a frame = owned tile k = s >> 12 (global tile
// rank + k * count) and pixel p = s & 4095 inside it in 8x8-block order (a
// wave's 64 lanes cover one 8x8 block).  A ray's tag is its global slot
// g = frame_in_batch * num_slots + s — at bounce 0 simply the launch index.
__device__ __forceinline__ void slot_pixel(uint32_t s, uint32_t rank, uint32_t count, uint32_t tiles_x, uint32_t& x,
                                           uint32_t& y) {
  const uint32_t k = s >> 12, p = s & 4095u;
  const uint32_t t = rank + k * count;
  const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
  const uint32_t blk = p >> 6, q = p & 63u;
  x = tx * kTile + (blk & 7u) * 8u + (q & 7u);
  y = ty * kTile + (blk >> 3) * 8u + (q >> 3);
}

// n / d for n < 2^31 through the launch's magic (kernels.h MagicDiv; draw_n
// checks every multiplier against its divisor d)
__device__ __forceinline__ uint32_t mdiv(uint32_t n, MagicDiv m, uint32_t d) {
  (void)d;
  return m.m ? (__umulhi(n, m.m) >> m.sh) : n;
}
// slot_pixel with the launch's magic for tiles_x
__device__ __forceinline__ void slot_pixel_a(uint32_t s, const BounceArgs& a, uint32_t& x, uint32_t& y) {
  const uint32_t k = s >> 12, p = s & 4095u;
  const uint32_t t = a.shard_rank + k * a.shard_count;
  const uint32_t ty = mdiv(t, a.div_tiles, a.tiles_x), tx = t - ty * a.tiles_x;
  const uint32_t blk = p >> 6, q = p & 63u;
  x = tx * kTile + (blk & 7u) * 8u + (q & 7u);
  y = ty * kTile + (blk >> 3) * 8u + (q >> 3);
}

// noise table of frame (batch frame fj) - back, back in {0, 1, 2}
__device__ __forceinline__ const float4* noise_table(const BounceArgs& a, uint32_t fj, uint32_t back) {
  return a.noise_window + (a.noise_offset + fj - back) * (kNoiseDim * kNoiseDim);
}

__device__ __forceinline__ uint32_t shade_noise_cell(uint32_t x, uint32_t y, uint32_t bounce, uint32_t f) {
  // renderer/Shaders.metal:135-136
  return ((x + bounce + f / 3) % kNoiseDim) + ((y + bounce + f / 5) % kNoiseDim) * kNoiseDim;
}

// intersectionHandler body for a ray with a valid hit (distance >= 1e-4),
// renderer/Shaders.metal:128-211.  Emits the NEE shadow ray (when
// bounce + 1 < L), adds MIS-weighted emission, and — when `next` — samples
// the next bounce and updates the throughput.
template <int MODE, bool SKIP_ZERO = true>
__device__ __forceinline__ void shade_hit(const DeviceScene& sc, const LdsCtx& cx, const Hit& h, PathState& s,
                                          const float4& ns, uint32_t bounce, uint32_t L, bool next, ShadowRay& sh,
                                          bool debug_material) {
  // Loads are staged behind scheduling barriers: hoisting all 13 float4
  // record loads together would pin ~50 VGPRs and halve occupancy.
  // interpolate(float2) — KernelHelpers.h:23-47
  const float wu = h.u, wv = h.v, ww = (1.0f - h.u) - h.v;
  uint32_t mat_index, light_index;
  V3 hv, hn;
  {
    const float4 P0 = fetch_prim<MODE>(sc, cx, h.prim, 0), P1 = fetch_prim<MODE>(sc, cx, h.prim, 1);
    const float4 P2 = fetch_prim<MODE>(sc, cx, h.prim, 2);
    mat_index = fbits(P0.w);
    light_index = fbits(P1.w);
    hv = add(add(mul(mk(P0), wu), mul(mk(P1), wv)), mul(mk(P2), ww));
  }
  {
    const float4 N0 = fetch_prim<MODE>(sc, cx, h.prim, 3), N1 = fetch_prim<MODE>(sc, cx, h.prim, 4);
    const float4 N2 = fetch_prim<MODE>(sc, cx, h.prim, 5);
    hn = normalize(add(add(mul(mk(N0), wu), mul(mk(N1), wv)), mul(mk(N2), ww)));
  }
  const Mat m = load_material<MODE>(sc, cx, mat_index);
  const V3 wI = s.d;
  if (debug_material) {   // DEBUG_MATERIAL (Shaders.metal:7,142-147): radiance := Fresnel, emission and NEE add to it
    const float f = fresnel(hn, neg(wI), 1.0f, 1.5f);
    s.R = mk(f, f, f);
  }
  sh.valid = false;
  sh.graze = true;
  // light sampling — Shaders.metal:150-176
  if (bounce + 1 < L) {
    const uint32_t li = selectLightTriangle<MODE>(sc, cx, sc.num_lights, ns.z);
    // barycentric(noise.wx) — Raytracing.h:182-187
    const float r1 = m_sqrt(ns.w), r2 = ns.x;
    const float bu = 1.0f - r1, bv = r1 * (1.0f - r2), bw = r1 * r2;
    V3 lv, ln;
    float lpdf;
    uint32_t lindex;
    {
      const float4 LB = fetch_light<MODE>(sc, cx, li, 1), LD = fetch_light<MODE>(sc, cx, li, 3);
      const float4 LF = fetch_light<MODE>(sc, cx, li, 5);
      lv = add(add(mul(mk(LB), bu), mul(mk(LD), bv)), mul(mk(LF), bw));
      lpdf = LB.w;
      lindex = fbits(LD.w);
    }
    {
      const float4 LC = fetch_light<MODE>(sc, cx, li, 2), LE = fetch_light<MODE>(sc, cx, li, 4);
      const float4 LG = fetch_light<MODE>(sc, cx, li, 6);
      ln = normalize(add(add(mul(mk(LC), bu), mul(mk(LE), bv)), mul(mk(LG), bw)));
    }
    const float4 LA = fetch_light<MODE>(sc, cx, li, 0);
    V3 dirToLight;
    float cosL;
    const float lightPdf = lightTriangleSamplePDF(lpdf, LA.w, hv, lv, ln, dirToLight, cosL);
    sh.graze = !(cosL >= sc.occ_cos_min);
    float materialBsdf, materialPdf;
    sampleMaterial(m, wI, dirToLight, hn, ns, materialBsdf, materialPdf);
    const float weight = balanceHeuristic(lightPdf, materialPdf);
    const float scale = m_div(weight * materialBsdf, lightPdf);
    sh.L = mk(((LA.x * m.kd.x) * s.T.x) * scale, ((LA.y * m.kd.y) * s.T.y) * scale,
              ((LA.z * m.kd.z) * s.T.z) * scale);
    sh.o = add(hv, mul(hn, kDistanceEpsilon));
    sh.d = dirToLight;
    sh.target = lindex;
    // A light sample of exactly zero (a mirror, a plastic mirror lobe or a
    // dielectric pass-through: the material's BSDF is 0 toward the light)
    // changes nothing whether or not it is occluded — R + 0 == R bit for bit,
    // R never being -0 (it starts at +0 and +0 + -0 == +0) — so its shadow
    // query is not traced (except by the B-2 stage kernel, whose shadow-ray
    // records follow the reference: traced as the reference does)
    sh.valid = (lightPdf > 0.0f) && (lindex != h.prim);
    if (SKIP_ZERO) sh.valid = sh.valid && !((sh.L.x == 0.0f) & (sh.L.y == 0.0f) & (sh.L.z == 0.0f));
  }
  // emission with MIS — Shaders.metal:180-197 (the light vertex re-derived
  // there is the hit vertex itself: lights[ref.lightTriangleIndex].index == prim)
  if (light_index != 0xFFFFFFFFu) {
    const float area = fetch_light<MODE>(sc, cx, light_index, 0).w, tpdf = fetch_light<MODE>(sc, cx, light_index, 1).w;
    V3 dirToLight;
    float cosE;
    const float mPdf = s.pdf;
    const float lPdf = s.prevDiffuse * lightTriangleSamplePDF(tpdf, area, s.o, hv, hn, dirToLight, cosE);
    const float weight = balanceHeuristic(mPdf, lPdf);
    const float k = weight * mPdf;
    s.R = add(s.R, mk((m.le.x * s.T.x) * k, (m.le.y * s.T.y) * k, (m.le.z * s.T.z) * k));
  }
  // next ray — Shaders.metal:199-211
  if (next) {
    float bsdf, pdf, ior;
    const V3 wO = generateNextBounce(m, wI, s.ior, hn, ns, bsdf, pdf, ior);
    s.d = wO;
    s.o = add(hv, mul(hn, kDistanceEpsilon));
    s.pdf = pdf;
    s.prevDiffuse = float(m.type == kDiffuse);
    s.mtype = m.type;
    s.ior = ior;
    const float q = m_div(bsdf, pdf);
    s.T = mk(s.T.x * (m.kd.x * q), s.T.y * (m.kd.y * q), s.T.z * (m.kd.z * q));
  }
}

// accumulateImage — renderer/Shaders.metal:233-249: the value written for
// frame f given the stored pixel
__device__ __forceinline__ float4 accumulate_value(const float4& stored, V3 c, uint32_t f) {
  if (f > 0) {
    const float factor = m_div(float(f), float(f + 1));
    return make_float4(mixf(c.x, stored.x, factor), mixf(c.y, stored.y, factor), mixf(c.z, stored.z, factor), 1.0f);
  }
  return make_float4(c.x, c.y, c.z, 1.0f);
}
__device__ __forceinline__ void accumulate_pixel(float4* image, uint32_t pix, V3 c, uint32_t f) {
  image[pix] = accumulate_value(f > 0 ? image[pix] : make_float4(0.0f, 0.0f, 0.0f, 0.0f), c, f);
}

// ---------------------------------------------------------------------------
// Diagnostic phase stamps (MRT_STAMPS builds only; never in the product):
// s_memtime around each wave-uniform phase of the bounce loop, summed per
// wave in SGPRs and stored once per wave (plain stores into g_wave_t) at
// exit, with the wave's launch timeline.  The stamp waits for
// vmcnt/lgkmcnt(0), so read the SHARES, not the length.
// ---------------------------------------------------------------------------
#ifndef MRT_STAMPS
#define MRT_STAMPS 0
#endif
#if MRT_STAMPS
__device__ __forceinline__ uint64_t stamp_now() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
// per-wave timeline of the last launch of each bounce index (b % 4), in
// s_memrealtime ticks (100 MHz, chip-wide), wave id = block * 4 + wave:
// {first iteration start, exit, iterations | exit reason << 32 (1 = input
// exhausted, 2 = output segment full), last grab, end of the last grab's
// work, summed grab latency, max grab latency, last grab's latency, phase
// cycles 0..4 (s_memtime), kernel entry (before the LDS staging)} — plain stores, so the exit is not a storm of
// atomics on a few words
constexpr uint32_t kStampWaves = 8192;
constexpr uint32_t kStampFields = 16;
__device__ unsigned long long g_wave_t[4][kStampWaves][kStampFields];
__device__ __forceinline__ uint64_t stamp_real() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define STAMP_DECL() uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}; uint64_t st_prev = 0; uint64_t st_iters = 0; \
    const uint64_t st_t0 = stamp_real(); uint64_t st_why = 0, st_grab = 0, st_work = 0, st_ab = 0, \
    st_asum = 0, st_amax = 0
#define STAMP_BEGIN() do { st_prev = stamp_now(); ++st_iters; } while (0)
#define STAMP(k) do { const uint64_t t_ = stamp_now(); st_acc[k] += t_ - st_prev; st_prev = t_; } while (0)
#define STAMP_FLUSH() do { if ((threadIdx.x & 63u) == 0) { \
    const uint32_t w_ = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u; \
    if (w_ < kStampWaves) { unsigned long long* e_ = g_wave_t[a.bounce & 3u][w_]; \
      e_[0] = st_t0; e_[1] = stamp_real(); e_[2] = st_iters | (st_why << 32); e_[3] = st_grab; \
      e_[4] = st_work; e_[5] = st_asum; e_[6] = st_amax; e_[7] = st_grab - st_ab; \
      for (int k_ = 0; k_ < 5; ++k_) e_[8 + k_] = st_acc[k_]; e_[13] = st_entry; } } } while (0)
#define STAMP_ENTRY() const uint64_t st_entry = stamp_real()
struct StampRef { uint64_t* acc; uint64_t* prev; };   // a kernel's phase accumulators, for a callee
#define STAMP_REF() StampRef{st_acc, &st_prev}
#define STAMP_AT(r, k) do { const uint64_t t_ = stamp_now(); (r).acc[k] += t_ - *(r).prev; *(r).prev = t_; } while (0)
#define STAMP_ATOMIC_BEGIN() do { st_ab = stamp_real(); } while (0)
#define STAMP_EXIT(got) do { st_why = (got) == 0xFFFFFFFEu ? 2u : 1u; } while (0)
#define STAMP_GRAB() do { st_grab = stamp_real(); st_asum += st_grab - st_ab; \
    st_amax = st_grab - st_ab > st_amax ? st_grab - st_ab : st_amax; } while (0)
#define STAMP_WORK() do { st_work = stamp_real(); } while (0)
#else
#define STAMP_DECL() do {} while (0)
#define STAMP_BEGIN() do {} while (0)
#define STAMP(k) do {} while (0)
#define STAMP_FLUSH() do {} while (0)
#define STAMP_EXIT(got) do {} while (0)
#define STAMP_GRAB() do {} while (0)
#define STAMP_WORK() do {} while (0)
#define STAMP_ATOMIC_BEGIN() do {} while (0)
#define STAMP_ENTRY() do {} while (0)
struct StampRef {};
#define STAMP_REF() StampRef{}
#define STAMP_AT(r, k) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// Fused wavefront bounce kernel (the hot path).
//
// One launch per (frame, bounce) over a persistent grid of G blocks.  Each
// ray: [bounce 0: generate the camera ray | else load its SoA state] ->
// nearest hit -> shade (NEE shadow ray, MIS emission, next direction) ->
// shadow visibility -> either accumulate the pixel (path ends: miss, near
// hit, or last bounce) or append the ray to the next queue.
//
// Queue compaction without global atomics: the N input rays are split into
// G contiguous block ranges of `chunk` rays; block g appends its survivors to
// [g*chunk, g*chunk + count_g) of the next queue with one LDS atomic per wave
// (ballot + popcount prefix inside the wave), and publishes count_g once.
// The next launch prefix-scans the G counts in LDS and maps its own dense
// index i to (segment j, offset) with a binary search.  Ray order inside a
// block segment is not deterministic; every ray carries its pixel, so the
// image is.
// ---------------------------------------------------------------------------
// exclusive prefix of v[0..n) in place (LDS), returns the total; n <= 16*kBlock
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t* v, uint32_t n, uint32_t* wave_tmp) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t per = (n + kBlock - 1) / kBlock;
  const uint32_t b = tid * per, e = min(n, b + per);
  uint32_t local = 0;
  for (uint32_t i = b; i < e; ++i) local += v[i];
  uint32_t incl = local;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t up = __shfl_up(incl, off);
    if ((int)lane >= off) incl += up;
  }
  if (lane == 63) wave_tmp[wave] = incl;
  __syncthreads();
  uint32_t wave_prefix = 0, total = 0;
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    if (w < wave) wave_prefix += wave_tmp[w];
    total += wave_tmp[w];
  }
  uint32_t run = wave_prefix + incl - local;
  for (uint32_t i = b; i < e; ++i) {
    const uint32_t x = v[i];
    v[i] = run;
    run += x;
  }
  __syncthreads();
  return total;
}

// One wave iteration of the fused bounce: up to 64 rays of bounce `bounce`.
// Each active lane generates its camera ray (bounce 0: `idx` = the launch's
// dense index = global slot) or loads its ray from `slot` of `in_q`, finds
// the nearest hit, shades it (NEE shadow ray, MIS emission, next ray), writes
// the radiance of a path that ends here, appends a survivor to the block's
// output segment [out_base, out_base + cap) of `out_q` through the LDS
// cursors (class 0 = left a diffuse surface, from the front; class 1 from
// the back) and traces the shadow ray.  Returns the survivors written.
// Used by bounce_kernel (one launch per bounce) and, with WAVEQ (the wave's
// own queue: survivors at out_base + their rank among the wave's survivors,
// no cursors, no class split), by stream_kernel.
template <int STACK, int MODE, bool WAVEQ = false>
__device__ __forceinline__ uint32_t bounce_wave(const DeviceScene& sc, const LdsCtx& cx, const BounceArgs& a,
                                               uint32_t bounce, bool active, uint32_t idx, uint32_t slot,
                                               const RayQueue& in_q, const RayQueue& out_q, uint32_t* cursor,
                                               uint32_t out_base, uint32_t cap,
                                               StampRef st) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool last = (bounce + 1 == a.max_path_length);
  LS_ADD(14, 1);
  LS_ADD(15, (uint32_t)__popcll(__ballot(active)));
  // -- phase 0: generate (bounce 0) or load (SoA queue planes 0-1) the ray
  PathState s;
  uint32_t tag = 0;   // tag = global owned slot | prevDiffuse << 31
  uint32_t pblk = 0xFFFFFFFFu;   // bounce 0: the pixel's 8x8 block (camera-ray candidate lists)
  if (active) {
    if (bounce == 0) {
      // frame fj of the batch (num_slots is a multiple of 4096: waves never
      // straddle frames, so fj is wave-uniform)
      const uint32_t fj = a.batch == 1u ? 0u : __builtin_amdgcn_readfirstlane(mdiv(idx, a.div_slots, a.num_slots));
      uint32_t x, y;
      slot_pixel_a(idx - fj * a.num_slots, a, x, y);
      active = (x < a.width) && (y < a.height);
      if (active) {
        tag = idx;
        pblk = (x / kPrimaryBlock) + (y / kPrimaryBlock) * a.primary_bx;
        const float4 ns = noise_table(a, fj, 0u)[(x % kNoiseDim) + (y % kNoiseDim) * kNoiseDim];
        camera_ray(x, y, a.width, a.height, ns, s.o, s.d);
      }
    } else {
      // planes 2-3 (throughput, pdf, radiance, ior) are loaded after the
      // traversal: they are not needed there, and keeping them out of the
      // traversal's live set saves 8 VGPRs
      const float4 q0 = in_q.plane[0][slot], q1 = in_q.plane[1][slot];
      s.o = mk(q0);
      tag = fbits(q0.w);
      s.d = mk(q1);
      s.prevDiffuse = (tag >> 31) ? 1.0f : 0.0f;
    }
  }
  STAMP_AT(st, 0);
  // -- phase 1: nearest hit of the path ray (MPS intersect, Renderer.mm:519-523)
  Hit h;
  h.found = false;
  bool listed = false;
  if (bounce == 0 && a.primary) {
    // a wave of camera rays is one 8x8 pixel block (slot_pixel): its
    // candidate list, when every active lane is in the same block
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(pblk);
    const bool uniform = b0 != 0xFFFFFFFFu && __ballot(active && pblk != b0) == 0;
    const uint32_t hd = uniform ? __builtin_amdgcn_readfirstlane(a.primary[b0]) : kPrimaryFallback;
    const uint32_t cnt = hd & 0xFFu;
    if (cnt != kPrimaryFallback) {
      listed = true;
      LS_ADD(18, 1);
      LS_ADD(19, (uint32_t)__popcll(__ballot(active)));
      if (active) primary_nearest<MODE>(sc, cx, a.primary + (hd >> 8), cnt, s.o, s.d, h);
    }
  }
  if (active && !listed) {
    if (last && sc.light_shortcut && !(a.flags & kShadeDebugMaterial)) {
      // the last bounce: light triangles, then one occlusion query (last_bounce_light_hit)
      bool graze;
      if (last_bounce_light_hit<MODE>(sc, cx, s.o, s.d, h, graze)) {
        // the light hit is the target of a shadow query from s.o: the
        // occluder tree when shadow_root allows it (the other lights lost to
        // it in last_bounce_light_hit already, so no lights_occlude here)
        Hit hh;
        hh.t = h.t;
        hh.found = false;
        const int32_t root = shadow_root(sc, s.o, graze);
        if (!(a.debug & 64u) && traverse<STACK, MODE, true>(sc, cx, s.o, s.d, 0.0f, hh, h.prim, root)) h.found = false;
      }
    } else {
      h = trace_nearest<STACK, MODE>(sc, cx, s.o, s.d, 0.0f, __builtin_inff());
    }
  }
  STAMP_AT(st, 1);
  // -- phase 2: intersectionHandler (Shaders.metal:105-212); a miss or a
  //    near hit ends the path (:122-126)
  const uint32_t gslot = tag & 0x7FFFFFFFu;
  if (active) {
    if (bounce == 0) {
      s.T = mk(1.0f, 1.0f, 1.0f);
      s.R = mk(0.0f, 0.0f, 0.0f);
      s.pdf = 1.0f;
      s.prevDiffuse = 0.0f;
      s.ior = 1.00029f;
    } else {
      const float4 q2 = in_q.plane[2][slot], q3 = in_q.plane[3][slot];
      s.T = mk(q2);
      s.pdf = q2.w;
      s.R = mk(q3);
      s.ior = q3.w;
    }
  }
  const bool hit_ok = active && h.found && !(h.t < kDistanceEpsilon);
  ShadowRay sh;
  sh.valid = false;
  if (__ballot(hit_ok)) {
    LS_ADD(12, 1);
    LS_ADD(13, (uint32_t)__popcll(__ballot(hit_ok)));
  }
  if (hit_ok) {
    const uint32_t fj = a.batch == 1u ? 0u : mdiv(gslot, a.div_slots, a.num_slots);   // frame in batch
    uint32_t x, y;
    slot_pixel_a(gslot - fj * a.num_slots, a, x, y);
    const uint32_t back = (bounce % 3u) == 0 ? 0u : ((bounce % 3u) == 1 ? 2u : 1u);   // uniform
    const float4 ns = noise_table(a, fj, back)[shade_noise_cell(x, y, bounce, a.frame_index + fj)];
    if (a.debug & 2u) {   // ablation: no shading, reflect back along the ray
      s.o = add(s.o, mul(s.d, h.t * 0.999f));
      s.d = mk(-s.d.x, -s.d.y, -s.d.z);
    } else {
      shade_hit<MODE>(sc, cx, h, s, ns, bounce, a.max_path_length, !last, sh, (a.flags & kShadeDebugMaterial) != 0);
    }
  }
  STAMP_AT(st, 2);
  // -- phase 3: paths that end here (miss, near hit, last bounce: none of
  //    them carries a shadow ray) go to accumulateImage (:233-249);
  //    survivors are compacted into this block's segment of the next queue.
  //    Planes 0-2 are written before the shadow traversal so the next ray
  //    is not live across it; plane 3 (radiance, ior) after it.
  if (active && (!hit_ok || last)) a.radiance[gslot] = make_float4(s.R.x, s.R.y, s.R.z, 0.0f);
  const bool alive = hit_ok && !last;
  // re-sort by material between bounces: survivors that left a diffuse
  // surface (class 0) fill the block's segment from the front, the others
  // (mirror / plastic / dielectric: specular and refracted rays) from the
  // back; the next bounce reads all class-0 runs first, so its waves see
  // rays of one class (MRT_DEBUG bit 16: no partition)
  const bool cls1 = !WAVEQ && (s.prevDiffuse == 0.0f) && !(a.debug & 16u);
  const uint64_t mask0 = __ballot(alive && !cls1), mask1 = __ballot(alive && cls1);
  uint32_t o = 0, wrote = 0;
  if (mask0 | mask1) {
    uint32_t w0 = 0, w1 = 0;
    if (!WAVEQ && lane == 0) {
      if (mask0) w0 = atomicAdd(&cursor[0], (uint32_t)__popcll(mask0));
      if (mask1) w1 = atomicAdd(&cursor[1], (uint32_t)__popcll(mask1));
    }
    w0 = __shfl(w0, 0);
    w1 = __shfl(w1, 0);
    o = cls1 ? out_base + cap - 1u - (w1 + lanes_below_in(mask1)) : out_base + w0 + lanes_below_in(mask0);
    if (alive && !(a.debug & 4u)) {
      out_q.plane[0][o] = make_float4(s.o.x, s.o.y, s.o.z, bitsf(gslot | (s.prevDiffuse != 0.0f ? 0x80000000u : 0u)));
      out_q.plane[1][o] = make_float4(s.d.x, s.d.y, s.d.z, 0.0f);
      out_q.plane[2][o] = make_float4(s.T.x, s.T.y, s.T.z, s.pdf);
    }
    wrote = (uint32_t)__popcll(mask0 | mask1);
  }
  STAMP_AT(st, 3);
  // -- phase 4: shadow ray (MPS intersect :545-553 + lightSamplingHandler :214-231)
  if (__ballot(sh.valid)) {
    LS_ADD(16, (uint32_t)__popcll(__ballot(sh.valid)));
    LS_ADD(17, 1);
  }
  if (sh.valid && ((a.debug & 1u) || shadow_reaches_target<STACK, MODE>(sc, cx, sh.o, sh.d, sh.target, h.prim, sh.graze, a.debug))) {
    s.R = add(s.R, sh.L);
  }
  if (alive && !(a.debug & 4u)) out_q.plane[3][o] = make_float4(s.R.x, s.R.y, s.R.z, s.ior);
  STAMP_AT(st, 4);
  return wrote;
}

// Device-measured execution span of a frame batch's render launch(es): the
// earliest block start and the latest wave end on the chip's wall clock.
// With batches on two streams the next launch's blocks start while this one
// drains, so host events around a launch would time the wait as well.
__device__ __forceinline__ void span_begin(const BounceArgs& a) {
  if (a.span && threadIdx.x == 0) atomicMax(a.span, ~(unsigned long long)wall_clock64());
}
__device__ __forceinline__ void span_end(const BounceArgs& a) {
  if (a.span && (threadIdx.x & 63u) == 0) atomicMax(a.span + 1, (unsigned long long)wall_clock64());
}

template <int STACK, int MODE>
__global__ __launch_bounds__(kBlock, MRT_BOUNCE_WAVES) void bounce_kernel(DeviceScene sc, BounceArgs a) {
  __shared__ uint32_t s_wave[kBlock / 64];
  __shared__ uint32_t s_cursor[2], s_res, s_closed;
  STAMP_ENTRY();
  span_begin(a);
  LS_INIT();
  const uint32_t tid = threadIdx.x;
  const uint32_t G = gridDim.x;
  const uint32_t nseg = (a.bounce == 0) ? 0u : a.in_segments;
  const LdsCtx cx = stage_lds<MODE>(sc, nseg + 1, a.stack_spill);
  uint32_t* seg = lds_u32() + cx.scratch_base;   // exclusive prefix of the input segments
  if (tid == 0) s_cursor[0] = s_cursor[1] = s_res = s_closed = 0;

  uint32_t N, in_chunk = 0;
  if (a.bounce == 0) {
    N = a.num_slots * a.batch;
    __syncthreads();
  } else {
    for (uint32_t i = tid; i < nseg; i += kBlock) seg[i] = a.in_seg_count[i];
    __syncthreads();
    N = block_exclusive_scan(seg, nseg, s_wave);
    if (tid == 0) seg[nseg] = N;   // sentinel: count of segment j = seg[j+1] - seg[j]
    __syncthreads();
    in_chunk = *a.in_chunk;
  }
  const uint32_t chunk = ((N + G - 1) / G + kBlock - 1) / kBlock * kBlock;
  // Work assignment (see kernels.h): dynamic — waves grab kGrab rays at a
  // time from kGrabRanges ranges, so the launch ends with at most one grab of
  // imbalance instead of a tail of slow blocks; block output capacity
  // cap = chunk + kSegSlack.  A wave reserves kGrab output slots in LDS
  // before it grabs and returns what it did not use; a wave that cannot
  // reserve stops.  A stopped block holds > cap - kGrab - 3*kGrab > chunk
  // survivors, so not every block can stop while input remains (survivors
  // <= N <= G*chunk): the input is always drained.
  // MRT_DEBUG bit 8: static interleaved assignment (64-ray groups
  // g*4 + w, + 4G, ...), capacity chunk.
  const bool dynamic = (a.debug & 8u) == 0;
  const uint32_t cap = dynamic ? chunk + kSegSlack : chunk;
  const uint32_t out_base = blockIdx.x * cap;
  const uint32_t rlen = ((N + kGrabRanges - 1) / kGrabRanges + kGrab - 1) / kGrab * kGrab;
  uint32_t cur_range = blockIdx.x % kGrabRanges, ranges_left = kGrabRanges;
  uint32_t static_base = blockIdx.x * kBlock + (tid & ~63u);

  const uint32_t lane = tid & 63u;

  STAMP_DECL();
  for (;;) {
    uint32_t start, end, niter;
    if (dynamic) {
      uint32_t got = 0xFFFFFFFFu;
      STAMP_ATOMIC_BEGIN();
      if (lane == 0) {
        if (atomicAdd(&s_res, kGrab) + kGrab <= cap) {
          // s_closed: ranges a wave of this block found exhausted, so the
          // block's other waves skip them without a device atomic (walking
          // the exhausted ranges one atomic at a time delayed the launch's
          // last exits by ~30 us: C2 +1.6 %, one GPU's 1/8 share +3.5 %;
          // publishing closed ranges in a launch-wide mask word measured
          // slower than the per-block mask alone)
          while (ranges_left) {
            const uint32_t r0 = cur_range * rlen;
            if (r0 < N && !(__hip_atomic_load(&s_closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & (1u << cur_range))) {
              const uint32_t i = atomicAdd(a.grab + cur_range * kGrabStride, kGrab);
              if (i < rlen && r0 + i < N) { got = r0 + i; break; }
              atomicOr(&s_closed, 1u << cur_range);
            }
            cur_range = cur_range + 1 == kGrabRanges ? 0u : cur_range + 1;
            --ranges_left;
          }
          if (got == 0xFFFFFFFFu) atomicSub(&s_res, kGrab);   // input exhausted
        } else {
          got = 0xFFFFFFFEu;                                   // block's output segment full
        }
      }
      got = __builtin_amdgcn_readfirstlane(got);
      if (got >= 0xFFFFFFFEu) { STAMP_EXIT(got); break; }
      cur_range = __builtin_amdgcn_readfirstlane(cur_range);
      ranges_left = __builtin_amdgcn_readfirstlane(ranges_left);
      STAMP_GRAB();
      start = got;
      end = min(N, cur_range * rlen + rlen);
      niter = kGrab / 64;
    } else {
      if (static_base >= N) break;
      start = static_base;
      end = N;
      niter = 1;
      static_base += G * kBlock;
    }
    uint32_t wrote = 0;
    for (uint32_t it = 0; it < niter; ++it) {
      const uint32_t idx = start + it * 64u + lane;
      bool active = idx < end;
      uint32_t slot = 0;
      if (active && a.bounce != 0) {
        uint32_t lo = 0, hi = nseg;   // last j with seg[j] <= idx
        while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (seg[mid] <= idx) lo = mid; else hi = mid; }
        // segments [0, G): class 0 from the start of block j's range;
        // [G, 2G): class 1, packed at the end of block j - G's range
        const uint32_t g_in = nseg >> 1;
        slot = lo < g_in ? lo * in_chunk + (idx - seg[lo])
                         : (lo - g_in) * in_chunk + in_chunk - (seg[lo + 1] - seg[lo]) + (idx - seg[lo]);
      }
      STAMP_BEGIN();
      wrote += bounce_wave<STACK, MODE>(sc, cx, a, a.bounce, active, idx, slot, a.in_q, a.out_q, s_cursor,
                                               out_base, cap, STAMP_REF());
    }
    STAMP_WORK();
    if (dynamic && lane == 0) atomicSub(&s_res, kGrab - wrote);
  }
  STAMP_FLUSH();
  __syncthreads();
  if (tid == 0) {
    a.out_seg_count[blockIdx.x] = s_cursor[0];
    a.out_seg_count[G + blockIdx.x] = s_cursor[1];
    const uint32_t total = s_cursor[0] + s_cursor[1];
    if (total) atomicAdd(a.out_total, total);   // stats: one atomic per block per launch
    if (blockIdx.x == 0) *a.out_chunk = cap;
  }
  LS_FLUSH();
  span_end(a);
}


// ---------------------------------------------------------------------------
// Wave-local streaming wavefront: every bounce of a frame batch in ONE launch
// over the persistent bounce grid, with no hand-off between waves (the
// whole-scene-in-LDS class: C1, C2).
//
// bounce_kernel ends every bounce at a launch boundary: the last grabs drain
// at falling occupancy and the next launch ramps up again — 60-110 us per
// launch on one GPU's 1/8 tile share of C2 (launches of 0.35-1 ms), 1-3 % of
// a whole-frame launch.  Here each wave keeps its own small queue per bounce
// level (kStreamCap slots in HBM, written and re-read by the same CU, so
// mostly L2 hits) and always runs a full wave of ONE bounce: the deepest
// level holding >= 64 rays, else 64 new camera rays from the launch's grab
// ranges.  Survivors go to the next level at the wave's own count (ballot +
// popcount, no atomics).  Every iteration is a coherent 64-lane wave of one
// bounce as in bounce_kernel (shading code path, noise table), the queues
// never exceed 2 * 64 - 1 rays per level (a level is run as soon as it holds
// 64 and deeper levels first), and only the end of the launch drains: once
// the camera rays are gone a wave runs its partial levels, deepest first.
// No wave ever waits for another, so any grid and any residency is safe.
// ---------------------------------------------------------------------------
template <int STACK, int MODE>
// Waves per SIMD the stream kernel's registers allow: 6 (80 VGPRs, 6 values
// spilled to scratch, reloaded outside the traversal loops: tools/
// scratch_sites.py) under the max-ILP scheduler of its unit (Makefile):
// C2 +1.7…+3.4 %, L = 5 +4…6 % over 5 waves (96 VGPRs, no spill); 7 / 8
// waves (23 / 37 spills) lose 6 / 27 %, and 6 waves under the default
// scheduler only tie (r5, alternating in one call); re-swept at the r6
// library: 5 / 7 waves -6 / -10 %, 0 / 2 spare block slots -2 / -1.3 %
#ifndef MRT_STREAM_WAVES
#define MRT_STREAM_WAVES 6
#endif
#ifndef MRT_STREAM_SPARE   // block slots per CU the stream kernel's persistent grid leaves free (stream_grid_t)
#define MRT_STREAM_SPARE 1
#endif
__global__ __launch_bounds__(kBlock, MRT_STREAM_WAVES) void stream_kernel(DeviceScene sc, BounceArgs a) {
  __shared__ uint32_t s_cnt[kBlock / 64][kStreamMaxL];    // rays queued per level (wave-private rows)
  __shared__ uint32_t s_alive[kBlock / 64][kStreamMaxL];  // survivors per bounce (stats)
  __shared__ uint32_t s_closed;
  span_begin(a);
  LS_INIT();
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t L = a.max_path_length;
  const LdsCtx cx = stage_lds<MODE>(sc, 0, a.stack_spill);
  for (uint32_t i = lane; i < L; i += 64u) { s_cnt[wave][i] = 0; s_alive[wave][i] = 0; }
  if (tid == 0) s_closed = 0;
  __syncthreads();
  uint32_t* cnt = s_cnt[wave];
  const uint32_t N0 = a.num_slots * a.batch;
  const uint32_t rlen = ((N0 + kGrabRanges - 1) / kGrabRanges + kGrab - 1) / kGrab * kGrab;
  uint32_t cur_range = blockIdx.x % kGrabRanges, ranges_left = kGrabRanges;
  // this wave's queue: level k (1..L-1) at slots qbase + (k - 1) * kStreamCap
  const uint32_t qbase = (blockIdx.x * (kBlock / 64u) + wave) * (L > 1 ? L - 1 : 1u) * kStreamCap;
  uint32_t pend = 0, pend_end = 0;   // camera rays [pend, pend_end) of the wave's last grab not yet run
  bool input = true;
  STAMP_DECL();   // stamp builds: phase cycles accumulate but are not flushed for this kernel
  const StampRef st = STAMP_REF();
  for (;;) {
    // the deepest level holding a full wave (wave-uniform LDS reads)
    uint32_t lvl = 0;
    for (uint32_t k = L - 1; k >= 1; --k)
      if (cnt[k] >= 64u) { lvl = k; break; }
    if (lvl == 0 && input && pend >= pend_end) {
      // grab kGrab camera rays from the launch's ranges (as bounce_kernel)
      uint32_t got = 0xFFFFFFFFu, gend = 0;
      if (lane == 0) {
        while (ranges_left) {
          const uint32_t r0 = cur_range * rlen;
          if (r0 < N0 && !(__hip_atomic_load(&s_closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & (1u << cur_range))) {
            const uint32_t i = atomicAdd(a.grab + cur_range * kGrabStride, kGrab);
            if (i < rlen && r0 + i < N0) { got = r0 + i; gend = min(N0, min(r0 + rlen, got + kGrab)); break; }
            atomicOr(&s_closed, 1u << cur_range);
          }
          cur_range = cur_range + 1 == kGrabRanges ? 0u : cur_range + 1;
          --ranges_left;
        }
      }
      got = __builtin_amdgcn_readfirstlane(got);
      cur_range = __builtin_amdgcn_readfirstlane(cur_range);
      ranges_left = __builtin_amdgcn_readfirstlane(ranges_left);
      if (got == 0xFFFFFFFFu) {
        input = false;
      } else {
        pend = got;
        pend_end = __builtin_amdgcn_readfirstlane(gend);
      }
    }
    uint32_t n, first;   // this iteration: n rays of level lvl
    bool camera = false;
    if (lvl == 0 && pend < pend_end) {
      camera = true;
      first = pend;
      n = min(64u, pend_end - pend);
      pend += n;
    } else {
      if (lvl == 0) {   // camera rays exhausted: the deepest non-empty level
        for (uint32_t k = L - 1; k >= 1; --k)
          if (cnt[k] > 0u) { lvl = k; break; }
        if (lvl == 0) break;   // every level empty: the wave is done
      }
      n = min(64u, cnt[lvl]);
      first = cnt[lvl] - n;   // run the top n, the rest stays in place
      cnt[lvl] = first;
    }
    const bool active = lane < n;
    const uint32_t idx = first + lane;                                  // camera: the launch's dense index
    const uint32_t slot = qbase + (lvl - 1u) * kStreamCap + first + lane;   // level lvl >= 1: the queue slot
    const uint32_t out = lvl + 1u < L ? qbase + lvl * kStreamCap + cnt[lvl + 1u] : 0u;
    // The wave reads rays its own lanes wrote: their stores first.  This
    // relies on gfx9 (CDNA) memory ordering: a wave's vector stores are
    // counted by vmcnt and the CU's L1 is write-through, so after
    // s_waitcnt vmcnt(0) the wave's own later loads see them.  On gfx10+
    // (stores counted by vscnt) it would need a wavefront-scope
    // release/acquire fence instead (measured within +0.5 % here, DESIGN.md
    // §2.1a).
#if MRT_LANESTATS
    // diagnostic: cycles this wait costs the wave (slot 28) over its level iterations (slot 29)
    uint64_t w0_, w1_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w0_)::"memory");
    if (!camera) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w1_)::"memory");
    if (!camera) { LS_ADD(28, (uint32_t)(w1_ - w0_)); LS_ADD(29, 1); }
#else
    if (!camera) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    LS_ADD(camera ? 26 : 27, 1);
    const uint32_t wrote = bounce_wave<STACK, MODE, true>(sc, cx, a, camera ? 0u : lvl, active, idx, slot,
                                                                 a.in_q, a.in_q, nullptr, out, 0u, st);
    if (lvl + 1u < L && lane == 0) {
      cnt[lvl + 1u] += wrote;
      s_alive[wave][lvl] += wrote;
    }
  }
  // stats: survivors of bounce b = rays alive at the start of bounce b + 1
  for (uint32_t b = lane; b + 1 < L; b += 64u)
    if (s_alive[wave][b]) atomicAdd(a.bounce_counts + b, s_alive[wave][b]);
  LS_FLUSH();
  span_end(a);
}

struct Trav {
  int32_t node, leaf;
  int sp;
};
__device__ __forceinline__ void trav_begin(int32_t root, Trav& tr) {
  tr.node = root;
  tr.leaf = 0;
  tr.sp = 0;
  if (tr.node < 0) { tr.leaf = tr.node; tr.node = kDone; }
}
__device__ __forceinline__ bool trav_done(const Trav& tr) { return tr.node == kDone && tr.leaf == 0; }

// One round of the while-while walk of traverse(): interior nodes (parking
// one leaf) until every lane still descending holds a leaf, then the parked
// leaves.  any = occlusion query: stops at the first triangle k != target
// with (t_k, k) < (h.t, target) and sets `occluded`.
// uv: when non-null, the nearest hit's barycentrics go to uv[0], uv[kBlock]
// (the lane's LDS path state) instead of h.u, h.v.
template <int STACK, int MODE>
__device__ __forceinline__ void trav_round(const DeviceScene& sc, const LdsCtx& cx, V3 o, V3 d, const RayBox& rb,
                                           Hit& h, bool any, uint32_t target, bool& occluded, Trav& tr,
                                           uint32_t* uv = nullptr, bool trl = false) {
  (void)trl;
#if MRT_TRACE_PX
  if (trl) printf("TR round node=%d leaf=%d sp=%d ht=%08x\n", tr.node, tr.leaf, tr.sp, fbits(h.t));
#endif
  while (tr.node != kDone && tr.node >= 0) {
    LS_ADD(2, 1);
    LS_ADD(3, (uint32_t)__popcll(__ballot(!any)));
    LS_ADD(9, (uint32_t)__popcll(__ballot(any)));
#if MRT_TRACE_PX
    const int32_t n0_ = tr.node;
#endif
    tr.node = interior_step<STACK, MODE, false>(sc, cx, tr.node, o, rb, 0.0f, h.t, tr.sp);
#if MRT_TRACE_PX
    if (trl) printf("TR   int %d -> %d sp=%d leaf=%d\n", n0_, tr.node, tr.sp, tr.leaf);
#endif
    if (tr.node < 0 && tr.leaf == 0) {
      tr.leaf = tr.node;
      tr.node = stack_pop<STACK>(cx, tr.sp);
#if MRT_TRACE_PX
      if (trl) printf("TR   park %d pop %d sp=%d\n", tr.leaf, tr.node, tr.sp);
#endif
    }
    if ((uint32_t)__popcll(__ballot(tr.leaf == 0)) <= (uint32_t)MRT_PATH_SLACK) break;
  }
  while (tr.leaf < 0) {
    LS_ADD(4, 1);
    LS_ADD(5, (uint32_t)__popcll(__ballot(!any)));
    LS_ADD(11, (uint32_t)__popcll(__ballot(any)));
    const uint32_t lr = ~(uint32_t)tr.leaf;
    const uint32_t first = lr >> kLeafCountBits, cnt = (lr & (kMaxLeafSize - 1)) + 1;
    if (leaf_tests<MODE>(sc, cx, o, d, 0.0f, first, cnt, h, any, target, uv)) {   // occluded: the query is over
      occluded = true;
      tr.node = kDone;
      tr.leaf = 0;
      break;
    }
#if MRT_TRACE_PX
    if (trl) printf("TR   leaf %d first=%u cnt=%u -> ht=%08x prim=%u\n", tr.leaf, first, cnt, fbits(h.t), h.prim);
#endif
    tr.leaf = 0;
    if (tr.node < 0) {
      tr.leaf = tr.node;
      tr.node = stack_pop<STACK>(cx, tr.sp);
#if MRT_TRACE_PX
      if (trl) printf("TR   next leaf %d pop %d sp=%d\n", tr.leaf, tr.node, tr.sp);
#endif
    }
#if MRT_LEAF_SLACK > 0
    if ((uint32_t)__popcll(__ballot(tr.leaf < 0)) <= (uint32_t)MRT_LEAF_SLACK) break;
#endif
  }
}

// ---------------------------------------------------------------------------
// Path megakernel: all MAX_PATH_LENGTH bounces of a batch of frames in ONE
// launch.  Each lane carries a whole path — camera ray, then per bounce the
// nearest-hit query, intersectionHandler, the NEE shadow query and
// lightSamplingHandler, in the reference's order (renderer/Renderer.mm:
// 500-585) — as a sequence of resumable traversal queries (trav_round); when
// MRT_PATH_SERVICE lanes have finished their query the wave services them
// together (shading or the shadow resolve, then the next query of the same
// path), and a lane whose path ended takes the next pixel sample from the
// wave's grab pool.  Compared with the wavefront of per-bounce launches there
// are no ray queues in HBM (the path state lives in LDS, 64 B per lane), no
// compaction and segment scans, and one launch (one ramp and drain) per
// batch instead of one per bounce.  The arithmetic of every path is the
// same, so the image is identical (precise build: bitwise).
// LDS path state per lane ([word][lane] after the stack): T (0-2), R (3-5),
// material pdf (6), ior (7), next-ray direction (8-10), pixel slot tag |
// prevDiffuse << 31 (11).  The next ray's origin needs no word: it is the
// shadow ray's origin (both are p + n * 1e-4, Shaders.metal:171,205), which
// stays in the lane's ray registers through the shadow query.
// ---------------------------------------------------------------------------
[[maybe_unused]] constexpr uint32_t kPathStateWords = 12;
#ifndef MRT_PATH_WAVES   // 5: 96 VGPRs with 1-3 spilled values (C4 +11 %, C3 +8 % over 4 waves)
#define MRT_PATH_WAVES 5
#endif
// Service threshold: finished nearest queries a wave collects before it
// shades them together.  With finished shadow queries handled inside the
// traversal loop (r4) a service round shades 22 of
// 64 lanes on C3 instead of 16: C4 2803 -> 2849 Mpaths/s (+1.6 %), C3 2491
// -> 2601 (+4.4 %) at 24, 2848 / 2620 at 32 (16: 2770 / 2471), alternating
// in one call.
#ifndef MRT_PATH_SERVICE
#define MRT_PATH_SERVICE 32
#endif

// Start the nearest query of the lane's ray: phase 1, a full traversal.
// (The last-bounce light shortcut of the wavefront kernels,
// last_bounce_light_hit, measured C4 -1.3 % / C3 -3.4 % here: removed in r6.)
__device__ __forceinline__ void begin_nearest(const DeviceScene& sc, Hit& h, Trav& tr, uint32_t& phase) {
  phase = 1;
  trav_begin(sc.root, tr);
  h.t = __builtin_inff(); h.u = h.v = 0.0f; h.prim = 0xFFFFFFFFu; h.found = false;
}

// Diagnostic path trace (MRT_TRACE_PX builds only, never the product): the
// queries of one pixel-frame (MRT_TRACE_X, MRT_TRACE_Y, absolute frame
// MRT_TRACE_F) printed with their float bits.
#ifndef MRT_TRACE_PX
#define MRT_TRACE_PX 0
#endif
#if MRT_TRACE_PX
__device__ __forceinline__ bool trace_lane(const BounceArgs& a, uint32_t tagv) {
  const uint32_t gslot = tagv & 0x7FFFFFFFu;
  const uint32_t fj = a.batch == 1u ? 0u : mdiv(gslot, a.div_slots, a.num_slots);
  uint32_t x, y;
  slot_pixel_a(gslot - fj * a.num_slots, a, x, y);
  return x == MRT_TRACE_X && y == MRT_TRACE_Y && a.frame_index + fj == MRT_TRACE_F;
}
#define MRT_TRACE(tagv, ...) do { if (trace_lane(a, (tagv))) printf(__VA_ARGS__); } while (0)
#else
#define MRT_TRACE(tagv, ...) do {} while (0)
#endif

template <int STACK, int MODE>
__global__ __launch_bounds__(kBlock, MRT_PATH_WAVES) void path_kernel(DeviceScene sc, BounceArgs a) {
  __shared__ uint32_t s_closed;
  __shared__ uint32_t s_count[64];   // rays alive at the start of bounce b + 1 (stats)
  span_begin(a);
  LS_INIT();
  const uint32_t tid = threadIdx.x;
  const LdsCtx cx = stage_lds<MODE>(sc, 1, a.stack_spill);
  if (tid == 0) s_closed = 0;
  if (tid < 64) s_count[tid] = 0;
  __syncthreads();
  const uint32_t N = a.num_slots * a.batch;
  const uint32_t L = a.max_path_length;
  const uint32_t rlen = ((N + kGrabRanges - 1) / kGrabRanges + kGrab - 1) / kGrab * kGrab;
  uint32_t cur_range = blockIdx.x % kGrabRanges, ranges_left = kGrabRanges;
  const uint32_t lane = tid & 63u;
  uint32_t* const ps = lds_u32() + cx.stack_base + threadIdx.x + (uint32_t)(STACK < 0 ? -STACK : STACK) * kBlock;

  uint32_t pool_next = 0, pool_end = 0;   // wave-uniform pool of pixel-sample indices
  bool exhausted = false;
  uint32_t phase = 0;                     // 0 idle, 1 nearest query, 2 shadow query
  uint32_t bounce = 0;
  V3 ro = mk(0.0f, 0.0f, 0.0f), rd = mk(0.0f, 0.0f, 1.0f);
  Trav tr{kDone, 0, 0};
  Hit h;                                  // nearest: the hit; shadow: h.t = t_target, (h.u, h.v, bits h.prim) = L
  h.t = 0.0f; h.u = h.v = 0.0f; h.prim = 0u; h.found = false;
  bool occluded = false;
  uint32_t target = 0;

  for (;;) {
    LS_ADD(25, 1);
    // ---- refill idle lanes with new camera rays (rayGenerator, Shaders.metal:75-103)
    for (;;) {
      const uint64_t idle = __ballot(phase == 0);
      if (!idle || exhausted) break;
      if (pool_next >= pool_end) {
        uint32_t got = 0xFFFFFFFFu;
        if (lane == 0) {
          while (ranges_left) {
            const uint32_t r0 = cur_range * rlen;
            if (r0 < N && !(__hip_atomic_load(&s_closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & (1u << cur_range))) {
              const uint32_t i = atomicAdd(a.grab + cur_range * kGrabStride, kGrab);
              if (i < rlen && r0 + i < N) { got = r0 + i; break; }
              atomicOr(&s_closed, 1u << cur_range);
            }
            cur_range = cur_range + 1 == kGrabRanges ? 0u : cur_range + 1;
            --ranges_left;
          }
        }
        got = __builtin_amdgcn_readfirstlane(got);
        cur_range = __builtin_amdgcn_readfirstlane(cur_range);
        ranges_left = __builtin_amdgcn_readfirstlane(ranges_left);
        if (got == 0xFFFFFFFFu) { exhausted = true; break; }
        pool_next = got;
        pool_end = min(N, min(got + kGrab, cur_range * rlen + rlen));
      }
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
      const uint32_t take = min((uint32_t)__popcll(idle), pool_end - pool_next);
      LS_ADD(24, (uint32_t)__popcll(__ballot(phase == 0 && rank < take)));
      if (phase == 0 && rank < take) {
        const uint32_t idx = pool_next + rank;
        // sample index -> (frame fj, slot sl): frame-major, or (sc.region_grabs)
        // block-major — 8x8 pixel block, then frame, then pixel — so that a
        // grab range (1/kGrabRanges of the launch) is one band of the image
        // over all the batch's frames, and the blocks of one XCD (block ids
        // = x mod 8) start on ranges x and x + 8: their rays meet the same
        // geometry in that XCD's L2
        uint32_t fj, sl;
        if (sc.region_grabs) {
          const uint32_t q = idx >> 6, blk = mdiv(q, a.div_batch, a.batch);
          fj = q - blk * a.batch;
          sl = (blk << 6) | (idx & 63u);
        } else {
          fj = a.batch == 1u ? 0u : mdiv(idx, a.div_slots, a.num_slots);
          sl = idx - fj * a.num_slots;
        }
        uint32_t x, y;
        slot_pixel_a(sl, a, x, y);
        if ((x < a.width) && (y < a.height)) {
          const float4 ns = noise_table(a, fj, 0u)[(x % kNoiseDim) + (y % kNoiseDim) * kNoiseDim];
          camera_ray(x, y, a.width, a.height, ns, ro, rd);
          ps[0 * kBlock] = fbits(1.0f); ps[1 * kBlock] = fbits(1.0f); ps[2 * kBlock] = fbits(1.0f);
          ps[3 * kBlock] = 0u; ps[4 * kBlock] = 0u; ps[5 * kBlock] = 0u;
          ps[6 * kBlock] = fbits(1.0f); ps[7 * kBlock] = fbits(1.00029f);
          ps[11 * kBlock] = fj * a.num_slots + sl;   // the global slot; prevDiffuse 0
          bounce = 0;
          begin_nearest(sc, h, tr, phase);
        }
      }
      pool_next += take;
    }
    if (!__any(phase != 0)) break;   // every lane idle and no samples left

    // ---- traversal rounds until enough lanes have finished their query
    bool fin = phase != 0 && trav_done(tr);
    for (;;) {
      // a finished shadow query needs no shading: its light sample is added
      // (lightSamplingHandler, Shaders.metal:214-231) and the path's next
      // nearest query starts at once, inside the traversal loop, so service
      // rounds (whose shading cost is the same however few lanes they shade)
      // are spent on finished nearest queries only
      if (fin && phase == 2) {
        MRT_TRACE(ps[11 * kBlock], "TR O inline b=%u occluded=%d\n", bounce, (int)occluded);
        if (!occluded) {
          ps[3 * kBlock] = fbits(bitsf(ps[3 * kBlock]) + h.u);
          ps[4 * kBlock] = fbits(bitsf(ps[4 * kBlock]) + h.v);
          ps[5 * kBlock] = fbits(bitsf(ps[5 * kBlock]) + bitsf(h.prim));
        }
        bounce += 1;
        atomicAdd(&s_count[bounce - 1], 1u);   // stats: rays alive at the start of this bounce
        rd = mk(bitsf(ps[8 * kBlock]), bitsf(ps[9 * kBlock]), bitsf(ps[10 * kBlock]));
        begin_nearest(sc, h, tr, phase);
        fin = trav_done(tr);
      }
      // (phase 3 — the last-bounce light shortcut's occlusion query — no
      // longer occurs here; this check of it stays because without it the
      // compiler allocates the kernel worse: SGPR spills 26 -> 34, scratch
      // 20 -> 36 B per lane, r6)
      if (fin && phase == 3) {
        h.found = !occluded;
        phase = 1;
      }
      const uint64_t going = __ballot(phase != 0 && !fin);
      if (!going) break;
      if ((uint32_t)__popcll(__ballot(fin)) >= (exhausted ? 1u : (uint32_t)MRT_PATH_SERVICE)) break;
      LS_ADD(22, 1);
      LS_ADD(23, (uint32_t)__popcll(going));
      if (phase != 0 && !fin) {
        const RayBox rb = make_raybox(ro, rd);
#if MRT_TRACE_PX
        const bool trl = phase == 1 && bounce == MRT_TRACE_B && trace_lane(a, ps[11 * kBlock]);
#else
        const bool trl = false;
#endif
        trav_round<STACK, MODE>(sc, cx, ro, rd, rb, h, phase >= 2, target, occluded, tr, nullptr, trl);
        fin = trav_done(tr);
      }
    }
    if (!__any(fin)) continue;
    LS_ADD(20, 1);
    LS_ADD(21, (uint32_t)__popcll(__ballot(fin)));

    // ---- service: finished shadow queries (MPS nearest hit + lightSamplingHandler,
    //      Shaders.metal:214-231), then the path's next bounce
    bool next_query = false;
    if (fin && phase == 2) {
      MRT_TRACE(ps[11 * kBlock], "TR O service b=%u occluded=%d\n", bounce, (int)occluded);
      if (!occluded) {
        ps[3 * kBlock] = fbits(bitsf(ps[3 * kBlock]) + h.u);
        ps[4 * kBlock] = fbits(bitsf(ps[4 * kBlock]) + h.v);
        ps[5 * kBlock] = fbits(bitsf(ps[5 * kBlock]) + bitsf(h.prim));
      }
      next_query = true;
    }
    // ---- service: finished nearest queries (intersectionHandler, Shaders.metal:105-212)
    if (fin && phase == 1) {
      PathState s;
      s.o = ro;
      s.d = rd;
      s.T = mk(bitsf(ps[0 * kBlock]), bitsf(ps[1 * kBlock]), bitsf(ps[2 * kBlock]));
      s.R = mk(bitsf(ps[3 * kBlock]), bitsf(ps[4 * kBlock]), bitsf(ps[5 * kBlock]));
      s.pdf = bitsf(ps[6 * kBlock]);
      s.ior = bitsf(ps[7 * kBlock]);
      const uint32_t tagv = ps[11 * kBlock];
      s.prevDiffuse = (tagv >> 31) ? 1.0f : 0.0f;
      const uint32_t gslot = tagv & 0x7FFFFFFFu;
      const bool last = bounce + 1 == L;
      const bool hit_ok = h.found && !(h.t < kDistanceEpsilon);   // :122-126
      MRT_TRACE(tagv, "TR N b=%u found=%d t=%08x prim=%u u=%08x v=%08x o=%08x %08x %08x d=%08x %08x %08x\n", bounce,
                (int)h.found, fbits(h.t), h.prim, fbits(h.u), fbits(h.v), fbits(ro.x), fbits(ro.y), fbits(ro.z),
                fbits(rd.x), fbits(rd.y), fbits(rd.z));
      ShadowRay sh;
      sh.valid = false;
      LS_ADD(13, (uint32_t)__popcll(__ballot(hit_ok)));
      if (hit_ok) {
        const uint32_t fj = a.batch == 1u ? 0u : mdiv(gslot, a.div_slots, a.num_slots);
        uint32_t x, y;
        slot_pixel_a(gslot - fj * a.num_slots, a, x, y);
        const uint32_t back = (bounce % 3u) == 0 ? 0u : ((bounce % 3u) == 1 ? 2u : 1u);
        const float4 ns = noise_table(a, fj, back)[shade_noise_cell(x, y, bounce, a.frame_index + fj)];
        shade_hit<MODE>(sc, cx, h, s, ns, bounce, L, !last, sh, (a.flags & kShadeDebugMaterial) != 0);
      }
      if (!hit_ok || last) {   // the path ends: accumulateImage input (Shaders.metal:233-249)
        // streamed once to the accumulate pass: a non-temporal store, so the
        // 2 GB of radiance per launch do not evict BVH lines from L2 (C4
        // +1.2 %, 1960 -> 1984 Mpaths/s, A/B twice in one call)
        typedef float v4f __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4f{s.R.x, s.R.y, s.R.z, 0.0f}, reinterpret_cast<v4f*>(a.radiance + gslot));
        MRT_TRACE(tagv, "TR E b=%u R=%08x %08x %08x\n", bounce, fbits(s.R.x), fbits(s.R.y), fbits(s.R.z));
        phase = 0;
      } else {
        ps[0 * kBlock] = fbits(s.T.x); ps[1 * kBlock] = fbits(s.T.y); ps[2 * kBlock] = fbits(s.T.z);
        ps[3 * kBlock] = fbits(s.R.x); ps[4 * kBlock] = fbits(s.R.y); ps[5 * kBlock] = fbits(s.R.z);
        ps[6 * kBlock] = fbits(s.pdf); ps[7 * kBlock] = fbits(s.ior);
        ps[8 * kBlock] = fbits(s.d.x); ps[9 * kBlock] = fbits(s.d.y); ps[10 * kBlock] = fbits(s.d.z);
        ps[11 * kBlock] = gslot | (s.prevDiffuse != 0.0f ? 0x80000000u : 0u);
        ro = s.o;   // the next ray's origin (also the shadow ray's, below)
        // the shadow ray: MPS nearest hit == target test + occlusion query
        // (MRT_DEBUG bit 1, ablation only: no shadow queries)
        bool shadow = false;
        if (sh.valid && !(a.debug & 1u)) {
          const float4 P1 = fetch_prim<MODE>(sc, cx, sh.target, 1);   // .w: the target's light index
          const V3 p0 = mk(fetch_prim<MODE>(sc, cx, sh.target, 0)), p1 = mk(P1);
          const V3 p2 = mk(fetch_prim<MODE>(sc, cx, sh.target, 2));
          float tT, u, v;
          const int32_t sroot = shadow_root(sc, ro, sh.graze);
          if (tri_test(ro, sh.d, p0, sub(p1, p0), sub(p2, p0), 0.0f, __builtin_inff(), tT, u, v) &&
              !(tT < kDistanceEpsilon) && !origin_occludes<MODE>(sc, cx, ro, sh.d, h.prim, sh.target, tT) &&
              !(sc.occ_lights && sroot == sc.occ_root &&
                lights_occlude<MODE>(sc, cx, ro, sh.d, sh.target, fbits(P1.w), tT))) {
            shadow = true;
            phase = 2;
            MRT_TRACE(tagv, "TR S b=%u target=%u tT=%08x root=%d L=%08x %08x %08x\n", bounce, sh.target, fbits(tT),
                      sroot, fbits(sh.L.x), fbits(sh.L.y), fbits(sh.L.z));
            rd = sh.d;   // ro = s.o = sh.o
            trav_begin(sroot, tr);
            h.t = tT;
            h.u = sh.L.x;
            h.v = sh.L.y;
            h.prim = fbits(sh.L.z);
            h.found = false;
            target = sh.target;
            occluded = false;
          }
        }
        next_query = !shadow;
      }
    }
    // ---- the path's next bounce: its nearest-hit query
    if (next_query) {
      bounce += 1;
      atomicAdd(&s_count[bounce - 1], 1u);   // stats: rays alive at the start of this bounce
      // ro already holds the next ray's origin (set at shading, unchanged by a shadow query)
      rd = mk(bitsf(ps[8 * kBlock]), bitsf(ps[9 * kBlock]), bitsf(ps[10 * kBlock]));
      begin_nearest(sc, h, tr, phase);
    }
  }
  __syncthreads();
  if (tid < 64 && tid + 1 < L && s_count[tid]) atomicAdd(a.bounce_counts + tid, s_count[tid]);
  LS_FLUSH();
  span_end(a);
}

// accumulateImage (renderer/Shaders.metal:233-249) for a batch of frames over
// the owned tiles: image = f == 0 ? c : mix(c, image, f/(f+1)).  Frames are
// accumulated strictly in order (the running mean is order-dependent): one
// thread applies the batch's frames to its pixel in frame order.
// At most 32 VGPRs (four frames' loads in flight instead of eight): the
// render kernels hold 5 waves x 96 of a SIMD's 512 VGPRs (the path kernel;
// the stream kernel since r5 5 persistent blocks x 80), so a 32-VGPR
// accumulate wave fits beside them and batch b's accumulate (main stream)
// runs while batch b + 1 renders on the other stream instead of waiting for
// its drain (the 2-stream period was launch + ~0.33 ms on C2).  One call,
// alternating: C2 10755 / 10762 -> 11024 / 11033 Mpaths/s (+2.5 %), C2 L=5
// +2.0 %, C2 1/8 share 10340 -> 10733 (+3.7 %), C4 +0.5 %.
constexpr uint32_t kAccLoads = 4;
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_vgpr(32))) void accumulate_frame_kernel(AccumArgs a) {
  if (a.counters && blockIdx.x == 0) {   // the draw's render launches have completed (stream order)
    for (uint32_t i = threadIdx.x; i < a.copy_words; i += kBlock) a.host_counters[i] = a.counters[i];
    for (uint32_t i = threadIdx.x; i < a.span_words; i += kBlock)
      a.host_counters[a.span_word + i] = a.counters[a.span_word + i];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.zero_words; i += kBlock) a.counters[i] = 0u;
    __threadfence_system();
  }
  for (uint32_t idx = blockIdx.x * kBlock + threadIdx.x; idx < a.num_slots; idx += gridDim.x * kBlock) {
    uint32_t x, y;
    slot_pixel(idx, a.shard_rank, a.shard_count, a.tiles_x, x, y);
    if (x >= a.width || y >= a.height) continue;
    const uint32_t pix = y * a.width + x;
    // the running mean stays in registers across the batch's frames (one
    // image read and one write per pixel); radiance rows are read once,
    // eight frames' loads in flight at a time
    const float4* rad = a.radiance + idx;
    if (!a.accumulate) {   // ACCUMULATE_IMAGE false (Shaders.metal:241): the batch's last frame alone
      const float4 c = rad[(size_t)(a.batch - 1) * a.num_slots];
      a.image[pix] = make_float4(c.x, c.y, c.z, 1.0f);
      continue;
    }
    float4 cur = a.frame_index > 0 ? a.image[pix] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t j = 0;
    for (; j + kAccLoads <= a.batch; j += kAccLoads) {
      float4 c[kAccLoads];
#pragma unroll
      for (uint32_t k = 0; k < kAccLoads; ++k) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(rad + (size_t)(j + k) * a.num_slots));
        c[k] = make_float4(v.x, v.y, v.z, v.w);
      }
#pragma unroll
      for (uint32_t k = 0; k < kAccLoads; ++k) cur = accumulate_value(cur, mk(c[k]), a.frame_index + j + k);
    }
    for (; j < a.batch; ++j) cur = accumulate_value(cur, mk(rad[(size_t)j * a.num_slots]), a.frame_index + j);
    a.image[pix] = cur;
  }
}

// ---------------------------------------------------------------------------
// Stage kernels over the reference AoS records (B-2 ABI, parity replay)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void raygen_kernel(uint32_t W, uint32_t H, const float4* noise, RefRay* rays) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= W * H) return;
  const uint32_t x = i % W, y = i / W;
  V3 o, d;
  camera_ray(x, y, W, H, noise[(x % kNoiseDim) + (y % kNoiseDim) * kNoiseDim], o, d);
  RefRay& r = rays[i];
  r.origin[0] = o.x; r.origin[1] = o.y; r.origin[2] = o.z;
  r.direction[0] = d.x; r.direction[1] = d.y; r.direction[2] = d.z;
  r.maxDistance = __builtin_inff();
  r.params[0] = 1.0f; r.params[1] = 0.0f; r.params[2] = 0.0f; r.params[3] = 1.00029f;
  for (int k = 0; k < 3; ++k) { r.throughput[k] = 1.0f; r.radiance[k] = 0.0f; }
}

template <int STACK>
__global__ __launch_bounds__(kBlock) void intersect_kernel(DeviceScene sc, const uint8_t* rays, uint32_t stride,
                                                           uint32_t count, RefIntersection* out, uint32_t* spill) {
  const LdsCtx cx = stage_lds<kGlobal>(sc, 0, spill);
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < count; i += gridDim.x * kBlock) {
    const float* r = reinterpret_cast<const float*>(rays + (size_t)i * stride);
    RefIntersection res{-1.0f, 0xFFFFFFFFu, {0.0f, 0.0f}};
    const float tmax = r[7];
    if (tmax >= 0.0f) {   // maxDistance < 0 disables the ray (Shaders.metal:124,173)
      const V3 o = mk(r[0], r[1], r[2]), d = mk(r[4], r[5], r[6]);
      const Hit h = trace_nearest<STACK, kGlobal>(sc, cx, o, d, r[3], tmax);
      if (h.found) {
        res.distance = h.t;
        res.triangleIndex = h.prim;
        res.coordinates[0] = h.u;
        res.coordinates[1] = h.v;
      }
    }
    out[i] = res;
  }
}

__global__ __launch_bounds__(kBlock) void shade_kernel(DeviceScene sc, uint32_t W, uint32_t H, uint32_t f,
                                                       uint32_t L, const float4* noise,
                                                       const RefIntersection* isect, RefRay* rays,
                                                       RefShadowRay* srays, uint32_t flags) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= W * H) return;
  const uint32_t x = i % W, y = i / W;
  RefShadowRay& sr = srays[i];
  RefRay& r = rays[i];
  sr.maxDistance = -1.0f;                                   // Shaders.metal:119
  const RefIntersection is = isect[i];
  if (is.distance < kDistanceEpsilon) { r.maxDistance = -1.0f; return; }   // :122-126
  PathState s;
  s.o = mk(r.origin[0], r.origin[1], r.origin[2]);
  s.d = mk(r.direction[0], r.direction[1], r.direction[2]);
  s.T = mk(r.throughput[0], r.throughput[1], r.throughput[2]);
  s.R = mk(r.radiance[0], r.radiance[1], r.radiance[2]);
  s.pdf = r.params[0];
  s.prevDiffuse = r.params[1];
  s.ior = r.params[3];
  const uint32_t bounce = (uint32_t)r.params[2];
  Hit h;
  h.t = is.distance; h.prim = is.triangleIndex; h.u = is.coordinates[0]; h.v = is.coordinates[1]; h.found = true;
  ShadowRay sh;
  const LdsCtx cx = stage_lds<kGlobal>(sc, 0);
  shade_hit<kGlobal, false>(sc, cx, h, s, noise[shade_noise_cell(x, y, bounce, f)], bounce, L, true, sh,
                     (flags & kShadeDebugMaterial) != 0);
  if (bounce + 1 < L) {
    sr.origin[0] = sh.o.x; sr.origin[1] = sh.o.y; sr.origin[2] = sh.o.z;
    sr.direction[0] = sh.d.x; sr.direction[1] = sh.d.y; sr.direction[2] = sh.d.z;
    sr.maxDistance = sh.valid ? __builtin_inff() : -1.0f;
    sr.targetIndex = sh.target;
    sr.throughput[0] = sh.L.x; sr.throughput[1] = sh.L.y; sr.throughput[2] = sh.L.z;
  }
  r.radiance[0] = s.R.x; r.radiance[1] = s.R.y; r.radiance[2] = s.R.z;
  r.direction[0] = s.d.x; r.direction[1] = s.d.y; r.direction[2] = s.d.z;
  r.origin[0] = s.o.x; r.origin[1] = s.o.y; r.origin[2] = s.o.z;
  r.maxDistance = __builtin_inff();
  r.params[0] = s.pdf; r.params[1] = s.prevDiffuse; r.params[2] = float(bounce + 1); r.params[3] = s.ior;
  r.throughput[0] = s.T.x; r.throughput[1] = s.T.y; r.throughput[2] = s.T.z;
}

// lightSamplingHandler — Shaders.metal:214-231
__global__ __launch_bounds__(kBlock) void resolve_kernel(uint32_t count, const RefIntersection* isect, RefRay* rays,
                                                         const RefShadowRay* srays) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= count) return;
  const RefIntersection is = isect[i];
  if (is.distance >= kDistanceEpsilon && is.triangleIndex == srays[i].targetIndex)
    for (int k = 0; k < 3; ++k) rays[i].radiance[k] += srays[i].throughput[k];
}

__global__ __launch_bounds__(kBlock) void accumulate_kernel(uint32_t W, uint32_t H, uint32_t f, const RefRay* rays,
                                                            float4* image, bool accumulate) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= W * H) return;
  accumulate_pixel(image, i, mk(rays[i].radiance[0], rays[i].radiance[1], rays[i].radiance[2]), accumulate ? f : 0u);
}

inline uint32_t blocks_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

constexpr size_t kAllLdsBudget = 48 * 1024;   // scene bytes staged whole in LDS

int choose_mode(const DeviceScene& sc) {
  static const int forced = [] {   // MRT_MODE=0/1/2 forces kGlobal/kTopLds/kAllLds (profiling)
    const char* v = mrt::diag_env("MRT_MODE");
    return v ? std::atoi(v) : -1;
  }();
  if (forced >= 0 && forced <= 2) return forced;
  if ((size_t)lds_scene_float4s(kAllLds, sc) * 16 <= kAllLdsBudget)
    return kAllLds;
  return sc.lds_nodes > 0 ? kTopLds : kGlobal;
}

size_t bounce_lds_bytes(const DeviceScene& sc, int mode, uint32_t stack, uint32_t grid) {
  const size_t scene = (size_t)lds_scene_float4s(mode, sc) * 16;
  const size_t scratch = ((size_t)2 * grid + 1 + 3) / 4 * 16;   // segment counts per block (2 classes) + sentinel
  return scene + scratch + (size_t)stack * kBlock * 4;           // stack = LDS entries (|STACK|)
}

#if MRT_EMIT_MAIN   // the per-bounce and path kernels' host side (not in the stream unit)
// kTopLds: stage only as many top BVH nodes as keep the block's LDS within
// 1/MRT_BOUNCE_WAVES of the CU less a 2-KB margin for allocation granularity
// (the VGPR budget allows MRT_BOUNCE_WAVES resident blocks of 4 waves); the
// BFS order makes any prefix the top levels.  Full occupancy beats more
// staged nodes (at 6 blocks/CU: C4 with 80 nodes 828, ~100 nodes (at the
// edge) 780, 128 nodes 715 Mpaths/s).
#ifndef MRT_LDS_BLOCKS
#define MRT_LDS_BLOCKS MRT_BOUNCE_WAVES
#endif
DeviceScene fit_lds_nodes(const DeviceScene& sc, int mode, uint32_t stack, uint32_t grid) {
  if (mode != kTopLds) return sc;
  DeviceScene f = sc;
  const size_t kLdsPerBlockTarget = 160 * 1024 / MRT_LDS_BLOCKS - 2048;
  const size_t fixed = bounce_lds_bytes(sc, kGlobal, stack, grid) + 64;   // scratch + stack + static
  const size_t node_bytes = (size_t)node_float4s(sc.width) * 16;
  const size_t fit = fixed < kLdsPerBlockTarget ? (kLdsPerBlockTarget - fixed) / node_bytes : 0;
  f.lds_nodes = (uint32_t)std::min<size_t>(sc.lds_nodes, fit);
  return f;
}

template <int STACK, int MODE>
hipError_t grid_for(const DeviceScene& sc, uint32_t blocks_per_cu, uint32_t* grid) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return e;
  // the LDS scratch (2 segment counts per block) depends on the grid: take
  // the largest blocks/CU n whose own LDS footprint still allows n resident
  // blocks (and the VGPR budget allows)
  const uint32_t cus = (uint32_t)prop.multiProcessorCount;
  const int stack = STACK < 0 ? -STACK : STACK;
  int n = 1;
  for (int want = 8; want >= 1; --want) {
    const uint32_t g = cus * (uint32_t)want;
    const size_t lds = bounce_lds_bytes(fit_lds_nodes(sc, MODE, stack, g), MODE, stack, g);
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bounce_kernel<STACK, MODE>, kBlock, lds) != hipSuccess)
      occ = 0;
    if (occ >= want) { n = want; break; }
  }
  // one launch at a time: every resident block slot (the dynamic work
  // distribution leaves no tail to fill); with frames in flight the caller
  // asks for fewer blocks per CU per launch
  *grid = (uint32_t)(prop.multiProcessorCount * (blocks_per_cu ? std::min<uint32_t>(n, blocks_per_cu) : n));
  return hipSuccess;
}

// path kernel: LDS = scene image + stack + the per-lane path state; the
// kTopLds node budget fits MRT_PATH_WAVES resident blocks per CU
size_t path_lds_bytes(const DeviceScene& sc, int mode, uint32_t stack) {
  const size_t scene = (size_t)lds_scene_float4s(mode, sc) * 16;
  return scene + 16 + (size_t)stack * kBlock * 4 + (size_t)kPathStateWords * kBlock * 4;
}
DeviceScene fit_path_lds_nodes(const DeviceScene& sc, int mode, uint32_t stack) {
  if (mode != kTopLds) return sc;
  DeviceScene f = sc;
  const size_t target = 160 * 1024 / MRT_PATH_WAVES - 2048;
  const size_t fixed = path_lds_bytes(sc, kGlobal, stack) + 64 + 256;   // + static (s_count, s_closed)
  const size_t fit = fixed < target ? (target - fixed) / ((size_t)node_float4s(sc.width) * 16) : 0;
  f.lds_nodes = (uint32_t)std::min<size_t>(sc.lds_nodes, fit);
  return f;
}

template <int STACK, int MODE>
hipError_t path_grid_t(const DeviceScene& sc, uint32_t* grid) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return e;
  const int stack = STACK < 0 ? -STACK : STACK;
  const size_t lds = path_lds_bytes(fit_path_lds_nodes(sc, MODE, stack), MODE, stack);
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, path_kernel<STACK, MODE>, kBlock, lds) != hipSuccess || occ < 1)
    occ = 1;
  *grid = (uint32_t)prop.multiProcessorCount * (uint32_t)std::min(occ, 8);
  return hipSuccess;
}

template <int STACK, int MODE>
hipError_t launch_path_t(const DeviceScene& sc, const BounceArgs& a, uint32_t grid, hipStream_t s) {
  const int stack = STACK < 0 ? -STACK : STACK;
  const DeviceScene f = fit_path_lds_nodes(sc, MODE, stack);
  path_kernel<STACK, MODE><<<dim3(grid), dim3(kBlock), path_lds_bytes(f, MODE, stack), s>>>(f, a);
  return hipGetLastError();
}

template <int STACK>
hipError_t path_dispatch_mode(const DeviceScene& sc, const BounceArgs* a, uint32_t grid, uint32_t* grid_out,
                              hipStream_t s) {
  switch (choose_mode(sc)) {
    case kAllLds:
      return a ? launch_path_t<STACK, kAllLds>(sc, *a, grid, s) : path_grid_t<STACK, kAllLds>(sc, grid_out);
    case kTopLds:
      return a ? launch_path_t<STACK, kTopLds>(sc, *a, grid, s) : path_grid_t<STACK, kTopLds>(sc, grid_out);
    default:
      return a ? launch_path_t<STACK, kGlobal>(sc, *a, grid, s) : path_grid_t<STACK, kGlobal>(sc, grid_out);
  }
}

// LDS stack capacity variants (negative: |STACK| LDS entries + global spill)
hipError_t path_dispatch(const DeviceScene& sc, const BounceArgs* a, uint32_t stack_entries, uint32_t grid,
                         uint32_t* grid_out, hipStream_t s) {
  if (sc.width != 4) return hipErrorInvalidValue;
  if (sc.max_stack > stack_entries) {
    if (stack_entries <= 8) return path_dispatch_mode<-8>(sc, a, grid, grid_out, s);
    if (stack_entries <= 12) return path_dispatch_mode<-12>(sc, a, grid, grid_out, s);
    if (stack_entries <= 16) return path_dispatch_mode<-16>(sc, a, grid, grid_out, s);
    return path_dispatch_mode<-32>(sc, a, grid, grid_out, s);
  }
  if (stack_entries <= 8) return path_dispatch_mode<8>(sc, a, grid, grid_out, s);
  if (stack_entries <= 12) return path_dispatch_mode<12>(sc, a, grid, grid_out, s);
  if (stack_entries <= 16) return path_dispatch_mode<16>(sc, a, grid, grid_out, s);
  if (stack_entries <= 24) return path_dispatch_mode<24>(sc, a, grid, grid_out, s);
  return path_dispatch_mode<32>(sc, a, grid, grid_out, s);
}

template <int STACK, int MODE>
hipError_t launch_bounce_t(const DeviceScene& sc, const BounceArgs& a, uint32_t grid, hipStream_t s) {
  const DeviceScene f = fit_lds_nodes(sc, MODE, STACK < 0 ? -STACK : STACK, grid);
  const size_t lds = bounce_lds_bytes(f, MODE, STACK < 0 ? -STACK : STACK, grid);
  bounce_kernel<STACK, MODE><<<dim3(grid), dim3(kBlock), lds, s>>>(f, a);
  return hipGetLastError();
}

template <int STACK>
hipError_t dispatch_mode(const DeviceScene& sc, const BounceArgs* a, uint32_t grid, uint32_t* grid_out,
                         hipStream_t s) {
  switch (choose_mode(sc)) {
    case kAllLds:
      return a ? launch_bounce_t<STACK, kAllLds>(sc, *a, grid, s) : grid_for<STACK, kAllLds>(sc, grid, grid_out);
    case kTopLds:
      return a ? launch_bounce_t<STACK, kTopLds>(sc, *a, grid, s) : grid_for<STACK, kTopLds>(sc, grid, grid_out);
    default:
      return a ? launch_bounce_t<STACK, kGlobal>(sc, *a, grid, s) : grid_for<STACK, kGlobal>(sc, grid, grid_out);
  }
}

// stack_entries = LDS stack capacity (8/16/24/32); when the BVH's bound is
// larger, the spill variants (8, 16 or 32 LDS entries + global) are used
hipError_t dispatch(const DeviceScene& sc, const BounceArgs* a, uint32_t stack_entries, uint32_t grid,
                    uint32_t* grid_out, hipStream_t s) {
  if (sc.width != 4) return hipErrorInvalidValue;
  if (sc.max_stack > stack_entries) {
    if (stack_entries <= 8) return dispatch_mode<-8>(sc, a, grid, grid_out, s);
    if (stack_entries <= 16) return dispatch_mode<-16>(sc, a, grid, grid_out, s);
    return dispatch_mode<-32>(sc, a, grid, grid_out, s);
  }
  if (stack_entries <= 8) return dispatch_mode<8>(sc, a, grid, grid_out, s);
  if (stack_entries <= 12) return dispatch_mode<12>(sc, a, grid, grid_out, s);
  if (stack_entries <= 16) return dispatch_mode<16>(sc, a, grid, grid_out, s);
  if (stack_entries <= 24) return dispatch_mode<24>(sc, a, grid, grid_out, s);
  return dispatch_mode<32>(sc, a, grid, grid_out, s);
}

#endif  // MRT_EMIT_MAIN

// wave-local streaming wavefront: whole-scene-in-LDS scenes, the stack in LDS
template <int STACK>
hipError_t launch_stream_t(const DeviceScene& sc, const BounceArgs& a, uint32_t grid, hipStream_t s) {
  stream_kernel<STACK, kAllLds><<<dim3(grid), dim3(kBlock), bounce_lds_bytes(sc, kAllLds, STACK, 0), s>>>(sc, a);
  return hipGetLastError();
}
// the stream kernel's own persistent grid: every block slot its LDS (scene
// image + stack, no segment scratch) and registers leave on a CU
template <int STACK>
hipError_t stream_grid_t(const DeviceScene& sc, uint32_t* grid) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return e;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, stream_kernel<STACK, kAllLds>, kBlock,
                                                   bounce_lds_bytes(sc, kAllLds, STACK, 0)) != hipSuccess || occ < 1)
    occ = 1;
  // one block slot per CU is left to the other render stream's launch and
  // the accumulate kernel (MRT_STREAM_SPARE): with 6-wave registers the
  // kernel fits 6 blocks per CU, and 5 of them persistent measured best —
  // C2 11937 vs 11740 Mpaths/s with all 6 (1344 / 1408 blocks: within
  // ±0.3 %), per-frame draws 9585 vs 8856 (r5, alternating in one call)
  const int spare = occ > 1 ? MRT_STREAM_SPARE : 0;
  *grid = (uint32_t)prop.multiProcessorCount * (uint32_t)std::min(occ - spare, 8);
  return hipSuccess;
}

bool stream_ok(const DeviceScene& sc, uint32_t stack_entries) {
  return sc.width == 4 && choose_mode(sc) == kAllLds && sc.max_stack <= stack_entries && stack_entries <= 32;
}

}  // namespace

// Translation units (Makefile): MRT_TU 0 = every entry point (precise and
// diagnostic builds); the fast build is split in two — MRT_TU 1 everything
// but the stream kernel, MRT_TU 2 the stream kernel alone, compiled with the
// max-ILP machine scheduler (-amdgpu-sched-strategy=max-ilp: C2 +0.45 %,
// alternating in one call, while the path kernel loses 0.5 % under it).
#if MRT_EMIT_MAIN
hipError_t launch_raygen(uint32_t W, uint32_t H, const float* noise, RefRay* rays, hipStream_t s) {
  raygen_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(W, H,
                     reinterpret_cast<const float4*>(noise), rays);
  return hipGetLastError();
}

hipError_t launch_intersect(const DeviceScene& sc, const void* rays, uint32_t stride, uint32_t count,
                            RefIntersection* out, uint32_t* spill, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (sc.width != 4) return hipErrorInvalidValue;
  const uint8_t* r = reinterpret_cast<const uint8_t*>(rays);
  if (sc.max_stack <= (uint32_t)kMaxStack) {   // whole stack in LDS
    const size_t lds = (size_t)kMaxStack * kBlock * 4;
    intersect_kernel<kMaxStack><<<dim3(blocks_for(count)), dim3(kBlock), lds, s>>>(sc, r, stride, count, out, nullptr);
  } else {                                      // 32 LDS entries + global spill, persistent grid
    if (!spill) return hipErrorInvalidValue;
    const size_t lds = (size_t)32 * kBlock * 4;
    const dim3 g(std::min<uint32_t>(blocks_for(count), kIntersectSpillGrid));
    intersect_kernel<-32><<<g, dim3(kBlock), lds, s>>>(sc, r, stride, count, out, spill);
  }
  return hipGetLastError();
}

hipError_t launch_shade(const DeviceScene& sc, uint32_t W, uint32_t H, uint32_t frame_index, uint32_t max_path_length,
                        const float* noise, const RefIntersection* isect, RefRay* rays, RefShadowRay* srays,
                        uint32_t flags, hipStream_t s) {
  shade_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(sc, W, H, frame_index,
                     max_path_length, reinterpret_cast<const float4*>(noise), isect, rays, srays, flags);
  return hipGetLastError();
}

hipError_t launch_resolve(uint32_t count, const RefIntersection* isect, RefRay* rays, const RefShadowRay* srays,
                          hipStream_t s) {
  if (count == 0) return hipSuccess;
  resolve_kernel<<<dim3(blocks_for(count)), dim3(kBlock), 0, s>>>(count, isect, rays, srays);
  return hipGetLastError();
}

hipError_t launch_accumulate(uint32_t W, uint32_t H, uint32_t frame_index, const RefRay* rays, float* image,
                             bool accumulate, hipStream_t s) {
  accumulate_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(W, H, frame_index, rays,
                     reinterpret_cast<float4*>(image), accumulate);
  return hipGetLastError();
}

hipError_t launch_accumulate_frame(const AccumArgs& a, hipStream_t s) {
  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(blocks_for(a.num_slots), 4096));
  accumulate_frame_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(a);
  return hipGetLastError();
}

// blitFragment — renderer/Shaders.metal:33-70 with the compile-time switches
// of Raytracing.h:11-12,25-31 as runtime flags (include/mrt.h MRT_DISPLAY_*):
// tone map 1 - exp(-c) (ENABLE_TONE_MAPPING), toSRGB on rgb (MANUAL_SRGB,
// Raytracing.h:130-135), then the COMPARISON_MODE against a reference image
// scaled by COMPARISON_SCALE.  One output pixel per image pixel (the
// reference samples the W x H texture with a nearest filter).
__device__ __forceinline__ float to_srgb(float v) {   // Raytracing.h:130-135
  if (v <= 0.0f) return 0.0f;
  if (v >= 1.0f) return 1.0f;
#if MRT_PRECISE
  return (v < 0.0031308f) ? (12.92f * v) : (1.055f * powf(v, 1.0f / 2.4f) - 0.055f);
#else
  return (v < 0.0031308f) ? (12.92f * v) : (1.055f * __powf(v, 1.0f / 2.4f) - 0.055f);
#endif
}
__device__ __forceinline__ float4 display_map(float4 c, uint32_t flags) {
  if (flags & 1u) {   // tone mapping (applies to all four channels, as color = 1 - exp(-color))
#if MRT_PRECISE
    c = make_float4(1.0f - expf(-c.x), 1.0f - expf(-c.y), 1.0f - expf(-c.z), 1.0f - expf(-c.w));
#else
    c = make_float4(1.0f - __expf(-c.x), 1.0f - __expf(-c.y), 1.0f - __expf(-c.z), 1.0f - __expf(-c.w));
#endif
  }
  if (flags & 2u) c = make_float4(to_srgb(c.x), to_srgb(c.y), to_srgb(c.z), c.w);
  return c;
}
__global__ __launch_bounds__(kBlock) void display_kernel(const float4* image, const float4* reference, float4* out,
                                                         uint32_t n, uint32_t flags, float scale) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float4 c = display_map(image[i], flags);
  const uint32_t mode = (flags >> 8) & 0xFFu;
  if (mode == 0u || !reference) { out[i] = c; return; }
  const float4 r = display_map(reference[i], flags);   // the reference texture goes through the same blit
  float4 o;
  if (mode == 1u) {          // COMPARE_ABSOLUTE_VALUE
    o = make_float4(fabsf(c.x - r.x), fabsf(c.y - r.y), fabsf(c.z - r.z), fabsf(c.w - r.w));
  } else if (mode == 2u) {   // COMPARE_REF_TO_COLOR
    o = make_float4(fmaxf(0.0f, r.x - c.x), fmaxf(0.0f, r.y - c.y), fmaxf(0.0f, r.z - c.z), fmaxf(0.0f, r.w - c.w));
  } else if (mode == 3u) {   // COMPARE_COLOR_TO_REF
    o = make_float4(fmaxf(0.0f, c.x - r.x), fmaxf(0.0f, c.y - r.y), fmaxf(0.0f, c.z - r.z), fmaxf(0.0f, c.w - r.w));
  } else {                   // COMPARE_LUMINANCE: red = output brighter, green = reference brighter
    const float lc = (c.x * (1.0f / 3.0f) + c.y * (1.0f / 3.0f)) + c.z * (1.0f / 3.0f);
    const float lr = (r.x * (1.0f / 3.0f) + r.y * (1.0f / 3.0f)) + r.z * (1.0f / 3.0f);
    o = make_float4(fmaxf(0.0f, lc - lr), fmaxf(0.0f, lr - lc), 0.0f, 1.0f);
  }
  out[i] = make_float4(o.x * scale, o.y * scale, o.z * scale, o.w * scale);
}

hipError_t launch_display(const float4* image, const float4* reference, float4* out, uint32_t n, uint32_t flags,
                          float compare_scale, hipStream_t s) {
  if (n == 0) return hipSuccess;
  display_kernel<<<dim3(blocks_for(n)), dim3(kBlock), 0, s>>>(image, reference, out, n, flags, compare_scale);
  return hipGetLastError();
}

// owned-tile pack/unpack for the multi-GPU exchange (renderer.cpp
// mrt_tiles_pack / mrt_tiles_unpack): packed index = k * 4096 + ty * 64 + tx
// for the k-th owned tile (global tile rank + k * count, row-major tiles)
__global__ __launch_bounds__(kBlock) void tiles_move_kernel(const float4* src, float4* dst, uint32_t W, uint32_t H,
                                                            uint32_t rank, uint32_t count, uint32_t tiles_x,
                                                            uint32_t owned, bool pack) {
  const uint64_t n = (uint64_t)owned * kTile * kTile;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = (uint32_t)(i >> 12), p = (uint32_t)(i & 4095u);
    const uint32_t t = rank + k * count;
    const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
    const uint32_t x = tx * kTile + (p & 63u), y = ty * kTile + (p >> 6);
    const bool in = x < W && y < H;
    if (pack) dst[i] = in ? src[(size_t)y * W + x] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    else if (in) dst[(size_t)y * W + x] = src[i];
  }
}

hipError_t launch_tiles_move(const float4* src, float4* dst, uint32_t W, uint32_t H, uint32_t rank, uint32_t count,
                             bool pack, hipStream_t s) {
  const uint32_t tx = (W + kTile - 1) / kTile, ty = (H + kTile - 1) / kTile, T = tx * ty;
  const uint32_t owned = rank < T ? (T - rank + count - 1) / count : 0u;
  if (!owned) return hipSuccess;
  const uint32_t blocks = std::min<uint32_t>(4096u, owned * 16u);
  tiles_move_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(src, dst, W, H, rank, count, tx, owned, pack);
  return hipGetLastError();
}

hipError_t read_wave_times(unsigned long long* out, size_t n) {
#if MRT_STAMPS
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), std::min(n, (size_t)4 * kStampWaves * kStampFields) * sizeof(unsigned long long));
#else
  for (size_t k = 0; k < n; ++k) out[k] = 0;
  return hipSuccess;
#endif
}

hipError_t read_lane_stats(unsigned long long* out, size_t n, bool reset) {
  for (size_t k = 0; k < n; ++k) out[k] = 0;
#if MRT_LANESTATS
  unsigned long long v[kLaneStats];
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_lanes), sizeof(v));
  if (e != hipSuccess) return e;
  for (size_t k = 0; k < n && k < (size_t)kLaneStats; ++k) out[k] = v[k];
  if (reset) {
    for (int k = 0; k < kLaneStats; ++k) v[k] = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_lanes), v, sizeof(v));
  }
  return e;
#else
  (void)reset;
  return hipSuccess;
#endif
}

hipError_t read_stamps(unsigned long long* out8, bool reset) {
  for (int k = 0; k < 8; ++k) out8[k] = 0;
#if MRT_STAMPS
  // phase cycles and iterations summed over the per-wave records of the last
  // launch of each bounce index
  std::vector<unsigned long long> w((size_t)4 * kStampWaves * kStampFields);
  hipError_t e = hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_wave_t), w.size() * sizeof(unsigned long long));
  if (e != hipSuccess) return e;
  for (size_t i = 0; i < (size_t)4 * kStampWaves; ++i) {
    const unsigned long long* r = &w[i * kStampFields];
    for (int k = 0; k < 5; ++k) out8[k] += r[8 + k];
    out8[5] += r[2] & 0xFFFFFFFFull;
  }
  if (reset) {
    std::fill(w.begin(), w.end(), 0ull);
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_t), w.data(), w.size() * sizeof(unsigned long long));
  }
  return e;
#else
  (void)reset;
  return hipSuccess;
#endif
}

hipError_t bounce_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t blocks_per_cu, uint32_t* grid) {
  // (dispatch passes `grid` through as blocks_per_cu when no launch is given)
  return dispatch(sc, nullptr, stack_entries, blocks_per_cu, grid, nullptr);
}

hipError_t launch_bounce(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries, uint32_t grid,
                         hipStream_t s) {
  return dispatch(sc, &a, stack_entries, grid, nullptr, s);
}

hipError_t launch_paths(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries, uint32_t grid,
                        hipStream_t s) {
  return path_dispatch(sc, &a, stack_entries, grid, nullptr, s);
}

hipError_t path_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t* grid) {
  return path_dispatch(sc, nullptr, stack_entries, 0, grid, nullptr);
}

bool path_preferred(const DeviceScene& sc) { return choose_mode(sc) != kAllLds; }

#endif  // MRT_EMIT_MAIN
#if MRT_EMIT_STREAM
bool stream_supported(const DeviceScene& sc, uint32_t stack_entries) { return stream_ok(sc, stack_entries); }

hipError_t stream_grid(const DeviceScene& sc, uint32_t stack_entries, uint32_t* grid) {
  if (!stream_ok(sc, stack_entries)) return hipErrorNotSupported;
  if (stack_entries <= 8) return stream_grid_t<8>(sc, grid);
  if (stack_entries <= 12) return stream_grid_t<12>(sc, grid);
  if (stack_entries <= 16) return stream_grid_t<16>(sc, grid);
  if (stack_entries <= 24) return stream_grid_t<24>(sc, grid);
  return stream_grid_t<32>(sc, grid);
}

hipError_t launch_stream(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries, uint32_t grid,
                         hipStream_t s) {
  if (!stream_ok(sc, stack_entries) || a.max_path_length > kStreamMaxL) return hipErrorNotSupported;
  if (stack_entries <= 8) return launch_stream_t<8>(sc, a, grid, s);
  if (stack_entries <= 12) return launch_stream_t<12>(sc, a, grid, s);
  if (stack_entries <= 16) return launch_stream_t<16>(sc, a, grid, s);
  if (stack_entries <= 24) return launch_stream_t<24>(sc, a, grid, s);
  return launch_stream_t<32>(sc, a, grid, s);
}
#endif  // MRT_EMIT_STREAM

}  // namespace MRT_NS
}  // namespace mrt
