// noise.h — per-frame noise tables (renderer/Renderer.mm:102-129, :486-496).
//
// The reference seeds std::mt19937_64 from the clock; here the clock is a
// fixed 64-bit seed S:
//   initial table (copied to all 3 slots): seed_seq{lo, hi}
//   frame f (written to slot f%3)        : seed_seq{lo ^ (f+1), hi ^ (f+3)}
// 16,384 draws of uniform_real_distribution<float>(0,1), cell-major, xyzw.
// Serialized slot semantics: iteration i of frame f reads slot (f+i)%3, which
// holds T_f (i%3==0), T_{f-2} (i%3==1) or T_{f-1} (i%3==2); T_{<0} = initial.
#pragma once
#include <cstdint>
#include <random>

#include "mrt_layout.h"

namespace mrt {

inline void make_noise_table(uint64_t seed, int64_t frame, float* out) {
  uint32_t lo = (uint32_t)(seed & 0xffffffffu);
  uint32_t hi = (uint32_t)(seed >> 32);
  if (frame >= 0) {
    lo ^= (uint32_t)(frame + 1);
    hi ^= (uint32_t)(frame + 3);
  }
  std::seed_seq ss{lo, hi};
  std::mt19937_64 rng;
  rng.seed(ss);
  std::uniform_real_distribution<float> dist(0.0f, 1.0f);
  for (unsigned i = 0; i < kNoiseFloats; ++i) out[i] = dist(rng);
}

// Which table (frame id, -1 = initial) iteration i of frame f reads.
inline int64_t noise_frame_for_iteration(int64_t f, uint32_t i) {
  switch (i % 3) {
    case 0: return f;
    case 1: return f >= 2 ? f - 2 : -1;
    default: return f >= 1 ? f - 1 : -1;
  }
}

}  // namespace mrt
