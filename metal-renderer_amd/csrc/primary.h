// primary.h — camera-ray candidate lists (host build).
//
// The reference's camera is fixed (rayGenerator, renderer/Shaders.metal:75-103:
// origin (0, 1, 2.35), image plane z = -1 in front of it), and bounce 0 sends
// one ray per pixel through it.  Every camera ray of an 8x8 pixel block —
// one 64-lane wave of bounce 0 (kernels.hip slot_pixel) — points into a small
// rectangle of the image plane, so the only triangles such a ray can hit are
// those whose perspective projection overlaps that rectangle.  For each block
// we list them (leaf-order indices into DeviceScene::tris); bounce 0 then
// tests the block's list as wave-uniform LDS / scalar reads instead of walking
// the BVH.  The nearest hit is the lexicographic minimum of (t, primitive)
// over the triangles a ray hits, so any superset of those triangles gives the
// same answer as the traversal, bit for bit.
//
// Layout (uint32): [blocks_x * blocks_y] headers, then the lists.  A header is
// (offset << 8) | count, offset in words from the start of the buffer;
// count == kPrimaryFallback: the block traverses the BVH (list too long).
#pragma once
#include <cstdint>
#include <vector>

#include "mrt_layout.h"   // kPrimaryFallback, kPrimaryBlock (pixels per block edge: one wave of bounce 0)

namespace mrt {

struct PrimaryLists {
  std::vector<uint32_t> words;              // empty: not built (too few blocks listable)
  uint32_t blocks_x = 0, blocks_y = 0;
  uint32_t listed_blocks = 0;               // blocks with a list (the rest fall back)
  double mean_count = 0.0;                  // mean list length over listed blocks
};

// tris: 12 floats per leaf-ordered triangle {v0, bits(prim), e1, 0, e2, 0};
// lists longer than `cap` fall back to the traversal.  Returns false (and an
// empty result) when the scene is too dense for lists to pay off.
bool build_primary_lists(const float* tris, uint32_t num_tris, uint32_t width, uint32_t height, uint32_t cap,
                         PrimaryLists& out);

}  // namespace mrt
