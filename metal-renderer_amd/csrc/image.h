// image.h — golden-image I/O of the host side (see image.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mrt {

// Decode a scanline OpenEXR file into RGBA32F, row 0 = BOTTOM (the renderer's
// image orientation; loadReferenceImage flips the same way,
// renderer/Renderer.mm:233-235).  A missing A channel reads as 1.
bool load_exr(const std::string& path, std::vector<float>& rgba, uint32_t& width, uint32_t& height, std::string& err);

}  // namespace mrt
