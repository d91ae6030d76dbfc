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

#include "kernels.h"

#ifndef MRT_PRECISE
#error "compile with -DMRT_PRECISE=0 or 1"
#endif
#if MRT_PRECISE
#define MRT_NS precise
#else
#define MRT_NS fast
#endif

namespace mrt {
namespace MRT_NS {
namespace {

constexpr int kBlock = 256;   // 4 waves of 64 lanes

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

// ---------------------------------------------------------------------------
// Geometry: MPS nearest-hit semantics (renderer/Renderer.mm:464-469)
// ---------------------------------------------------------------------------
// Moller-Trumbore, cull none; (u, v) are the weights of (V0, V1) as
// interpolate() expects (renderer/KernelHelpers.h:37-47).
__device__ __forceinline__ bool tri_test(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float tmin, float tmax, float& t,
                                         float& u, float& v) {
  const V3 p = cross(d, e2);
  const float det = dot(e1, p);
  if (det == 0.0f) return false;
  const float inv = m_rcp(det);
  const V3 s = sub(o, v0);
  const float b1 = dot(s, p) * inv;
  if (!(b1 >= 0.0f && b1 <= 1.0f)) return false;
  const V3 q = cross(s, e1);
  const float b2 = dot(d, q) * inv;
  if (!(b2 >= 0.0f && b1 + b2 <= 1.0f)) return false;
  const float tt = dot(e2, q) * inv;
  if (!(tt >= tmin && tt <= tmax)) return false;
  t = tt;
  u = (1.0f - b1) - b2;
  v = b1;
  return true;
}

struct Hit {
  float t, u, v;
  uint32_t prim;
  bool found;
};

struct RayBox {   // precomputed slab-test terms
  V3 inv;
#if !MRT_PRECISE
  V3 oinv;
#endif
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

// Box test of both children of a node; returns entry distances.
__device__ __forceinline__ void box2(const float4& a, const float4& b, const float4& c, V3 o, const RayBox& rb,
                                     float tmin, float tmax, bool& hl, bool& hr, float& tnl, float& tnr) {
#if MRT_PRECISE
  const V3 oi = o;
  const float ox = o.x, oy = o.y, oz = o.z;
  const float oix = 0.0f, oiy = 0.0f, oiz = 0.0f;
  (void)oi;
#else
  const float ox = 0.0f, oy = 0.0f, oz = 0.0f;
  const float oix = rb.oinv.x, oiy = rb.oinv.y, oiz = rb.oinv.z;
#endif
  const float lx0 = slab(a.x, ox, rb.inv.x, oix), lx1 = slab(a.y, ox, rb.inv.x, oix);
  const float ly0 = slab(a.z, oy, rb.inv.y, oiy), ly1 = slab(a.w, oy, rb.inv.y, oiy);
  const float lz0 = slab(c.x, oz, rb.inv.z, oiz), lz1 = slab(c.y, oz, rb.inv.z, oiz);
  const float rx0 = slab(b.x, ox, rb.inv.x, oix), rx1 = slab(b.y, ox, rb.inv.x, oix);
  const float ry0 = slab(b.z, oy, rb.inv.y, oiy), ry1 = slab(b.w, oy, rb.inv.y, oiy);
  const float rz0 = slab(c.z, oz, rb.inv.z, oiz), rz1 = slab(c.w, oz, rb.inv.z, oiz);
  tnl = fmaxf(fmaxf(fminf(lx0, lx1), fminf(ly0, ly1)), fmaxf(fminf(lz0, lz1), tmin));
  const float tfl = fminf(fminf(fmaxf(lx0, lx1), fmaxf(ly0, ly1)), fminf(fmaxf(lz0, lz1), tmax));
  tnr = fmaxf(fmaxf(fminf(rx0, rx1), fminf(ry0, ry1)), fmaxf(fminf(rz0, rz1), tmin));
  const float tfr = fminf(fminf(fmaxf(rx0, rx1), fmaxf(ry0, ry1)), fminf(fmaxf(rz0, rz1), tmax));
  hl = tnl <= tfl;
  hr = tnr <= tfr;
}

// Traversal context: LDS-staged top nodes + a per-lane LDS stack laid out
// [entry][lane] (consecutive lanes hit consecutive banks).
struct TraversalCtx {
  const float4* lds_nodes;
  uint32_t n_lds;
  uint32_t* stack;       // &lds_stack[threadIdx.x]
};

__device__ __forceinline__ void fetch_node(const DeviceScene& sc, const TraversalCtx& cx, int32_t node, float4& a,
                                           float4& b, float4& c, float4& e) {
  const float4* p = ((uint32_t)node < cx.n_lds) ? cx.lds_nodes + 4 * node
                                                : reinterpret_cast<const float4*>(sc.nodes) + 4 * (size_t)node;
  a = p[0];
  b = p[1];
  c = p[2];
  e = p[3];
}

// Nearest hit in [tmin, tmax]; ties -> lowest primitive index.
template <int STACK>
__device__ Hit trace_nearest(const DeviceScene& sc, const TraversalCtx& cx, V3 o, V3 d, float tmin, float tmax) {
  Hit h;
  h.t = tmax;
  h.u = h.v = 0.0f;
  h.prim = 0xFFFFFFFFu;
  h.found = false;
  const RayBox rb = make_raybox(o, d);
  const float4* tris = reinterpret_cast<const float4*>(sc.tris);
  int32_t node = sc.root;
  int sp = 0;
  while (true) {
    if (node >= 0) {
      float4 a, b, c, e;
      fetch_node(sc, cx, node, a, b, c, e);
      bool hl, hr;
      float tnl, tnr;
      box2(a, b, c, o, rb, tmin, h.t, hl, hr, tnl, tnr);
      const int32_t rl = (int32_t)fbits(e.x), rr = (int32_t)fbits(e.y);
      if (hl && hr) {
        const bool swap = tnr < tnl;
        const int32_t nearer = swap ? rr : rl, farther = swap ? rl : rr;
        if (sp < STACK) { cx.stack[sp * kBlock] = (uint32_t)farther; ++sp; }
        node = nearer;
        continue;
      }
      if (hl) { node = rl; continue; }
      if (hr) { node = rr; continue; }
    } else {
      const uint32_t leaf = ~(uint32_t)node;
      const uint32_t first = leaf >> kLeafCountBits, cnt = (leaf & (kMaxLeafSize - 1)) + 1;
      for (uint32_t k = 0; k < cnt; ++k) {
        const float4 t0 = tris[3 * (first + k)], t1 = tris[3 * (first + k) + 1], t2 = tris[3 * (first + k) + 2];
        float t, u, v;
        if (tri_test(o, d, mk(t0), mk(t1), mk(t2), tmin, h.t, t, u, v)) {
          const uint32_t prim = fbits(t0.w);
          if (!h.found || t < h.t || prim < h.prim) {
            h.found = true;
            h.t = t;
            h.u = u;
            h.v = v;
            h.prim = prim;
          }
        }
      }
    }
    if (sp == 0) break;
    --sp;
    node = (int32_t)cx.stack[sp * kBlock];
  }
  return h;
}

// Is any primitive k != target hit with (t_k, k) < (t_target, target)?
// (the shadow ray's MPS nearest hit is then not the target)
template <int STACK>
__device__ bool trace_occluded(const DeviceScene& sc, const TraversalCtx& cx, V3 o, V3 d, uint32_t target,
                               float t_target) {
  const RayBox rb = make_raybox(o, d);
  const float4* tris = reinterpret_cast<const float4*>(sc.tris);
  int32_t node = sc.root;
  int sp = 0;
  while (true) {
    if (node >= 0) {
      float4 a, b, c, e;
      fetch_node(sc, cx, node, a, b, c, e);
      bool hl, hr;
      float tnl, tnr;
      box2(a, b, c, o, rb, 0.0f, t_target, hl, hr, tnl, tnr);
      const int32_t rl = (int32_t)fbits(e.x), rr = (int32_t)fbits(e.y);
      if (hl && hr) {
        const bool swap = tnr < tnl;
        const int32_t nearer = swap ? rr : rl, farther = swap ? rl : rr;
        if (sp < STACK) { cx.stack[sp * kBlock] = (uint32_t)farther; ++sp; }
        node = nearer;
        continue;
      }
      if (hl) { node = rl; continue; }
      if (hr) { node = rr; continue; }
    } else {
      const uint32_t leaf = ~(uint32_t)node;
      const uint32_t first = leaf >> kLeafCountBits, cnt = (leaf & (kMaxLeafSize - 1)) + 1;
      for (uint32_t k = 0; k < cnt; ++k) {
        const float4 t0 = tris[3 * (first + k)], t1 = tris[3 * (first + k) + 1], t2 = tris[3 * (first + k) + 2];
        const uint32_t prim = fbits(t0.w);
        if (prim == target) continue;
        float t, u, v;
        if (tri_test(o, d, mk(t0), mk(t1), mk(t2), 0.0f, t_target, t, u, v) && (t < t_target || prim < target))
          return true;
      }
    }
    if (sp == 0) break;
    --sp;
    node = (int32_t)cx.stack[sp * kBlock];
  }
  return false;
}

// Shadow-ray resolve under MPS nearest-hit semantics + lightSamplingHandler
// (renderer/Shaders.metal:214-231): contributes iff the nearest hit of the
// shadow ray (tmin 0, tmax inf) is the target triangle at t >= 1e-4.
template <int STACK>
__device__ bool shadow_reaches_target(const DeviceScene& sc, const TraversalCtx& cx, V3 o, V3 d, uint32_t target) {
  const float4* pr = reinterpret_cast<const float4*>(sc.prims) + 6 * (size_t)target;
  const V3 p0 = mk(pr[0]), p1 = mk(pr[1]), p2 = mk(pr[2]);
  float tT, u, v;
  if (!tri_test(o, d, p0, sub(p1, p0), sub(p2, p0), 0.0f, __builtin_inff(), tT, u, v)) return false;
  if (!(tT >= kDistanceEpsilon)) return false;
  return !trace_occluded<STACK>(sc, cx, o, d, target, tT);
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
__device__ __forceinline__ Mat load_material(const DeviceScene& sc, uint32_t m) {
  const float4* p = reinterpret_cast<const float4*>(sc.materials) + 2 * m;
  const float4 a = p[0], b = p[1];
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
                                                        V3& dirOut) {
  const V3 d = sub(sv, source);
  const float dist = length(d);
  dirOut = normalize(d);
  const float LdotD = -dot(dirOut, sn);
  const float valid = float(dist >= kDistanceEpsilon) * float(LdotD >= kAngleEpsilon);
  return valid * tpdf * triangleSamplePDF(area, LdotD, dist);
}

// selectLightTriangle — KernelHelpers.h:49-54.  The linear scan returns the
// first index with !(cdf[index+1] <= xi) (or count); cdf is non-decreasing, so
// a binary search returns the same index.
__device__ __forceinline__ uint32_t selectLightTriangle(const float4* lights, uint32_t count, float xi) {
  uint32_t lo = 0, hi = count;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (lights[7 * (mid + 1) + 2].w <= xi) lo = mid + 1;   // entry mid+1: (v1.n, cdf)
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
};
struct ShadowRay {
  V3 o, d, L;
  uint32_t target;
  bool valid;
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
  o = mk(0.0f, 1.0f, 2.35f);   // up - view * 2.35
}

__device__ __forceinline__ uint32_t shade_noise_cell(uint32_t x, uint32_t y, uint32_t bounce, uint32_t f) {
  // renderer/Shaders.metal:135-136
  return ((x + bounce + f / 3) % kNoiseDim) + ((y + bounce + f / 5) % kNoiseDim) * kNoiseDim;
}

// intersectionHandler body for a ray with a valid hit (distance >= 1e-4),
// renderer/Shaders.metal:128-211.  Emits the NEE shadow ray (when
// bounce + 1 < L), adds MIS-weighted emission, and — when `next` — samples
// the next bounce and updates the throughput.
__device__ __forceinline__ void shade_hit(const DeviceScene& sc, const Hit& h, PathState& s, const float4& ns,
                                          uint32_t bounce, uint32_t L, bool next, ShadowRay& sh) {
  const float4* pr = reinterpret_cast<const float4*>(sc.prims) + 6 * (size_t)h.prim;
  const float4 P0 = pr[0], P1 = pr[1], P2 = pr[2], N0 = pr[3], N1 = pr[4], N2 = pr[5];
  const uint32_t mat_index = fbits(P0.w);
  const uint32_t light_index = fbits(P1.w);
  const Mat m = load_material(sc, mat_index);
  // interpolate(float2) — KernelHelpers.h:23-47
  const float wu = h.u, wv = h.v, ww = (1.0f - h.u) - h.v;
  const V3 hv = add(add(mul(mk(P0), wu), mul(mk(P1), wv)), mul(mk(P2), ww));
  const V3 hn = normalize(add(add(mul(mk(N0), wu), mul(mk(N1), wv)), mul(mk(N2), ww)));
  const V3 wI = s.d;
  const float4* lights = reinterpret_cast<const float4*>(sc.lights);
  sh.valid = false;
  // light sampling — Shaders.metal:150-176
  if (bounce + 1 < L) {
    const uint32_t li = selectLightTriangle(lights, sc.num_lights, ns.z);
    const float4* lt = lights + 7 * li;
    const float4 LA = lt[0], LB = lt[1], LC = lt[2], LD = lt[3], LE = lt[4], LF = lt[5], LG = lt[6];
    // barycentric(noise.wx) — Raytracing.h:182-187
    const float r1 = m_sqrt(ns.w), r2 = ns.x;
    const float bu = 1.0f - r1, bv = r1 * (1.0f - r2), bw = r1 * r2;
    const V3 lv = add(add(mul(mk(LB), bu), mul(mk(LD), bv)), mul(mk(LF), bw));
    const V3 ln = normalize(add(add(mul(mk(LC), bu), mul(mk(LE), bv)), mul(mk(LG), bw)));
    V3 dirToLight;
    const float lightPdf = lightTriangleSamplePDF(LB.w, LA.w, hv, lv, ln, dirToLight);
    float materialBsdf, materialPdf;
    sampleMaterial(m, wI, dirToLight, hn, ns, materialBsdf, materialPdf);
    const float weight = balanceHeuristic(lightPdf, materialPdf);
    const uint32_t lindex = fbits(LD.w);
    const float scale = m_div(weight * materialBsdf, lightPdf);
    sh.L = mk(((LA.x * m.kd.x) * s.T.x) * scale, ((LA.y * m.kd.y) * s.T.y) * scale,
              ((LA.z * m.kd.z) * s.T.z) * scale);
    sh.o = add(hv, mul(hn, kDistanceEpsilon));
    sh.d = dirToLight;
    sh.target = lindex;
    sh.valid = (lightPdf > 0.0f) && (lindex != h.prim);
  }
  // emission with MIS — Shaders.metal:180-197 (the light vertex re-derived
  // there is the hit vertex itself: lights[ref.lightTriangleIndex].index == prim)
  if (light_index != 0xFFFFFFFFu) {
    const float4* lt = lights + 7 * light_index;
    const float area = lt[0].w, tpdf = lt[1].w;
    V3 dirToLight;
    const float mPdf = s.pdf;
    const float lPdf = s.prevDiffuse * lightTriangleSamplePDF(tpdf, area, s.o, hv, hn, dirToLight);
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
    s.ior = ior;
    const float q = m_div(bsdf, pdf);
    s.T = mk(s.T.x * (m.kd.x * q), s.T.y * (m.kd.y * q), s.T.z * (m.kd.z * q));
  }
}

// accumulateImage — renderer/Shaders.metal:233-249
__device__ __forceinline__ void accumulate_pixel(float4* image, uint32_t pix, V3 c, uint32_t f) {
  float4 out;
  if (f > 0) {
    const float factor = m_div(float(f), float(f + 1));
    const float4 stored = image[pix];
    out = make_float4(mixf(c.x, stored.x, factor), mixf(c.y, stored.y, factor), mixf(c.z, stored.z, factor), 1.0f);
  } else {
    out = make_float4(c.x, c.y, c.z, 1.0f);
  }
  image[pix] = out;
}

// ---------------------------------------------------------------------------
// Fused wavefront bounce kernel (the hot path).
//
// One launch per (frame, bounce).  Each ray slot: [bounce 0: generate camera
// ray | else load SoA state] -> nearest hit -> shade (NEE shadow ray, MIS
// emission, next direction) -> shadow visibility -> either accumulate the
// pixel (path ends: miss, near hit, or last bounce) or append the ray to the
// next queue.  Appends are compacted per wave with a ballot + popcount
// prefix and ONE atomicAdd per wave.  Lanes are processed in wave-uniform
// grid-stride chunks so every ballot sees a converged wave.
// ---------------------------------------------------------------------------
template <int STACK>
__global__ __launch_bounds__(kBlock) void bounce_kernel(DeviceScene sc, BounceArgs a) {
  extern __shared__ float4 lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t n_lds = sc.lds_nodes;
  for (uint32_t i = tid; i < 4 * n_lds; i += kBlock) lds[i] = reinterpret_cast<const float4*>(sc.nodes)[i];
  __syncthreads();
  TraversalCtx cx;
  cx.lds_nodes = lds;
  cx.n_lds = n_lds;
  cx.stack = reinterpret_cast<uint32_t*>(lds + 4 * n_lds) + tid;

  const uint32_t lane = tid & 63u;
  const uint32_t wave_in_grid = blockIdx.x * (kBlock / 64) + (tid >> 6);
  const uint32_t wave_stride = gridDim.x * kBlock;
  const uint32_t count = (a.bounce == 0) ? a.num_slots : *a.in_count;
  const bool last = (a.bounce + 1 == a.max_path_length);
  const uint64_t lanes_below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  for (uint32_t base = wave_in_grid * 64; base < count; base += wave_stride) {
    const uint32_t slot = base + lane;
    bool active = slot < count;
    PathState s;
    uint32_t pix = 0, x = 0, y = 0;
    if (active) {
      if (a.bounce == 0) {
        // owned tile k -> global tile rank + k*count; 8x8 pixel blocks per wave
        const uint32_t k = slot >> 12, p = slot & 4095u;
        const uint32_t t = a.shard_rank + k * a.shard_count;
        const uint32_t tx = t % a.tiles_x, ty = t / a.tiles_x;
        const uint32_t blk = p >> 6, q = p & 63u;
        x = tx * kTile + (blk & 7u) * 8u + (q & 7u);
        y = ty * kTile + (blk >> 3) * 8u + (q >> 3);
        active = (x < a.width) && (y < a.height);
        if (active) {
          pix = y * a.width + x;
          const float4 ns = a.noise_raygen[(x % kNoiseDim) + (y % kNoiseDim) * kNoiseDim];
          camera_ray(x, y, a.width, a.height, ns, s.o, s.d);
          s.T = mk(1.0f, 1.0f, 1.0f);
          s.R = mk(0.0f, 0.0f, 0.0f);
          s.pdf = 1.0f;
          s.prevDiffuse = 0.0f;
          s.ior = 1.00029f;
        }
      } else {
        const float4 q0 = a.in_q.plane[0][slot], q1 = a.in_q.plane[1][slot];
        const float4 q2 = a.in_q.plane[2][slot], q3 = a.in_q.plane[3][slot];
        s.o = mk(q0);
        s.pdf = q0.w;
        s.d = mk(q1);
        s.ior = q1.w;
        s.T = mk(q2);
        const uint32_t tag = fbits(q2.w);
        pix = tag & 0x7FFFFFFFu;
        s.prevDiffuse = (tag >> 31) ? 1.0f : 0.0f;
        s.R = mk(q3);
        y = pix / a.width;
        x = pix - y * a.width;
      }
    }
    bool alive = false;
    if (active) {
      const Hit h = trace_nearest<STACK>(sc, cx, s.o, s.d, 0.0f, __builtin_inff());
      if (!h.found || h.t < kDistanceEpsilon) {
        accumulate_pixel(a.image, pix, s.R, a.frame_index);   // path terminated (Shaders.metal:122-126)
      } else {
        const float4 ns = a.noise_shade[shade_noise_cell(x, y, a.bounce, a.frame_index)];
        ShadowRay sh;
        shade_hit(sc, h, s, ns, a.bounce, a.max_path_length, !last, sh);
        if (sh.valid && shadow_reaches_target<STACK>(sc, cx, sh.o, sh.d, sh.target)) s.R = add(s.R, sh.L);
        if (last) accumulate_pixel(a.image, pix, s.R, a.frame_index);
        else alive = true;
      }
    }
    // wave-level stream compaction of the survivors
    const uint64_t mask = __ballot(alive);
    if (mask) {
      uint32_t wbase = 0;
      if (lane == 0) wbase = atomicAdd(a.out_count, (uint32_t)__popcll(mask));
      wbase = __shfl(wbase, 0);
      if (alive) {
        const uint32_t o = wbase + (uint32_t)__popcll(mask & lanes_below);
        a.out_q.plane[0][o] = make_float4(s.o.x, s.o.y, s.o.z, s.pdf);
        a.out_q.plane[1][o] = make_float4(s.d.x, s.d.y, s.d.z, s.ior);
        a.out_q.plane[2][o] = make_float4(s.T.x, s.T.y, s.T.z, bitsf(pix | (s.prevDiffuse != 0.0f ? 0x80000000u : 0u)));
        a.out_q.plane[3][o] = make_float4(s.R.x, s.R.y, s.R.z, 0.0f);
      }
    }
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

__global__ __launch_bounds__(kBlock) void intersect_kernel(DeviceScene sc, const uint8_t* rays, uint32_t stride,
                                                           uint32_t count, RefIntersection* out) {
  __shared__ uint32_t stack[kMaxStack * kBlock];
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= count) return;
  TraversalCtx cx{nullptr, 0u, stack + threadIdx.x};
  const float* r = reinterpret_cast<const float*>(rays + (size_t)i * stride);
  RefIntersection res{-1.0f, 0xFFFFFFFFu, {0.0f, 0.0f}};
  const float tmax = r[7];
  if (tmax >= 0.0f) {   // maxDistance < 0 disables the ray (Shaders.metal:124,173)
    const Hit h = trace_nearest<kMaxStack>(sc, cx, mk(r[0], r[1], r[2]), mk(r[4], r[5], r[6]), r[3], tmax);
    if (h.found) {
      res.distance = h.t;
      res.triangleIndex = h.prim;
      res.coordinates[0] = h.u;
      res.coordinates[1] = h.v;
    }
  }
  out[i] = res;
}

__global__ __launch_bounds__(kBlock) void shade_kernel(DeviceScene sc, uint32_t W, uint32_t H, uint32_t f,
                                                       uint32_t L, const float4* noise,
                                                       const RefIntersection* isect, RefRay* rays,
                                                       RefShadowRay* srays) {
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
  shade_hit(sc, h, s, noise[shade_noise_cell(x, y, bounce, f)], bounce, L, true, sh);
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
                                                            float4* image) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= W * H) return;
  accumulate_pixel(image, i, mk(rays[i].radiance[0], rays[i].radiance[1], rays[i].radiance[2]), f);
}

inline uint32_t blocks_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

template <int STACK>
hipError_t launch_bounce_t(const DeviceScene& sc, const BounceArgs& a, hipStream_t s) {
  const size_t lds_bytes = (size_t)sc.lds_nodes * 64 + (size_t)STACK * kBlock * 4;
  // occupancy-sized persistent grid, cached per (device, LDS footprint)
  static int cached_dev = -1, blocks_per_cu = 1, cus = 0;
  static size_t cached_lds = 0;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev != cached_dev || lds_bytes != cached_lds) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return e;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bounce_kernel<STACK>, kBlock, lds_bytes) != hipSuccess || n <= 0)
      n = 1;
    cus = prop.multiProcessorCount;
    blocks_per_cu = n;
    cached_dev = dev;
    cached_lds = lds_bytes;
  }
  uint32_t grid = (uint32_t)(cus * blocks_per_cu);
  if (a.bounce == 0) grid = std::min<uint32_t>(grid, std::max<uint32_t>(1, blocks_for(a.num_slots)));
  bounce_kernel<STACK><<<dim3(grid), dim3(kBlock), lds_bytes, s>>>(sc, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_raygen(uint32_t W, uint32_t H, const float* noise, RefRay* rays, hipStream_t s) {
  raygen_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(W, H,
                     reinterpret_cast<const float4*>(noise), rays);
  return hipGetLastError();
}

hipError_t launch_intersect(const DeviceScene& sc, const void* rays, uint32_t stride, uint32_t count,
                            RefIntersection* out, hipStream_t s) {
  if (count == 0) return hipSuccess;
  intersect_kernel<<<dim3(blocks_for(count)), dim3(kBlock), 0, s>>>(sc,
                     reinterpret_cast<const uint8_t*>(rays), stride, count, out);
  return hipGetLastError();
}

hipError_t launch_shade(const DeviceScene& sc, uint32_t W, uint32_t H, uint32_t frame_index, uint32_t max_path_length,
                        const float* noise, const RefIntersection* isect, RefRay* rays, RefShadowRay* srays,
                        hipStream_t s) {
  shade_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(sc, W, H, frame_index,
                     max_path_length, reinterpret_cast<const float4*>(noise), isect, rays, srays);
  return hipGetLastError();
}

hipError_t launch_resolve(uint32_t count, const RefIntersection* isect, RefRay* rays, const RefShadowRay* srays,
                          hipStream_t s) {
  if (count == 0) return hipSuccess;
  resolve_kernel<<<dim3(blocks_for(count)), dim3(kBlock), 0, s>>>(count, isect, rays, srays);
  return hipGetLastError();
}

hipError_t launch_accumulate(uint32_t W, uint32_t H, uint32_t frame_index, const RefRay* rays, float* image,
                             hipStream_t s) {
  accumulate_kernel<<<dim3(blocks_for(W * H)), dim3(kBlock), 0, s>>>(W, H, frame_index, rays,
                     reinterpret_cast<float4*>(image));
  return hipGetLastError();
}

hipError_t launch_bounce(const DeviceScene& sc, const BounceArgs& a, uint32_t stack_entries, hipStream_t s) {
  if (stack_entries <= 8) return launch_bounce_t<8>(sc, a, s);
  if (stack_entries <= 16) return launch_bounce_t<16>(sc, a, s);
  if (stack_entries <= 24) return launch_bounce_t<24>(sc, a, s);
  return launch_bounce_t<32>(sc, a, s);
}

}  // namespace MRT_NS
}  // namespace mrt
