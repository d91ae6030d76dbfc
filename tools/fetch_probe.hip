// FETCH_SIZE calibration for gathers vs streams (is the gfx950
// x2 correction of MI355X_MICROARCH.md valid for the path kernel's 16-B node
// gathers?).  Three kernels over a 2 GiB buffer much larger than L2 + MALL:
//   stream  — lane i reads float4 i (coalesced 16 B per lane), every byte once;
//   gather7 — lane i reads 7 consecutive float4 of 128-B line perm[i] (a BVH4
//             node fetch: 112 of the line's 128 B), every line once;
//   gather1 — lane i reads ONE float4 of line perm[i] (a 16-B gather).
// Each writes one float per lane.  Run under rocprofv3 --pmc FETCH_SIZE and
// compare with the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>
#include <numeric>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void stream_k(const float4* __restrict__ a, float* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = a[i];
  out[i & 0xFFFFFu] = v.x + v.y + v.z + v.w;
}
__global__ void gather7_k(const float4* __restrict__ a, const uint32_t* __restrict__ perm, float* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* p = a + (size_t)perm[i] * 8;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 7; ++k) { const float4 v = p[k]; s += v.x + v.y + v.z + v.w; }
  out[i] = s;
}
__global__ void gather1_k(const float4* __restrict__ a, const uint32_t* __restrict__ perm, float* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = a[(size_t)perm[i] * 8];
  out[i] = v.x + v.y + v.z + v.w;
}

int main() {
  const size_t bytes = (size_t)2 << 30, lines = bytes / 128, n16 = bytes / 16;
  float4* a; uint32_t* perm; float* out;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipMalloc(&perm, lines * 4));
  CHECK(hipMalloc(&out, lines * 4));
  std::vector<uint32_t> h(lines);
  std::iota(h.begin(), h.end(), 0u);
  std::shuffle(h.begin(), h.end(), std::mt19937(7));
  CHECK(hipMemcpy(perm, h.data(), lines * 4, hipMemcpyHostToDevice));
  CHECK(hipDeviceSynchronize());
  const int B = 256;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream_k, dim3((n16 + B - 1) / B), dim3(B), 0, 0, a, out, n16);
    hipLaunchKernelGGL(gather7_k, dim3((lines + B - 1) / B), dim3(B), 0, 0, a, perm, out, lines);
    hipLaunchKernelGGL(gather1_k, dim3((lines + B - 1) / B), dim3(B), 0, 0, a, perm, out, lines);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("{\"stream_bytes\": %zu, \"gather7_line_bytes\": %zu, \"gather7_used_bytes\": %zu, "
              "\"gather1_line_bytes\": %zu, \"perm_bytes\": %zu, \"out_bytes_gather\": %zu}\n",
              bytes, lines * 128, lines * 112, lines * 128, lines * 4, lines * 4);
  return 0;
}
