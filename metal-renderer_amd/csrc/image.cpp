// image.cpp — OpenEXR scanline reader for golden images, the replacement for
// loadReferenceImage (renderer/Renderer.mm:162-253), which reads
// Media/reference/<scene>-<MAX_PATH_LENGTH>.exr through OpenEXR's RgbaInputFile
// and flips it vertically into the RGBA32F comparison texture.
//
// Own decoder (the vendored OpenEXR 2.2 is not built here): single-part
// scanline files, compression NONE / ZIPS (1 line per block) / ZIP (16 lines),
// HALF / FLOAT / UINT channels; R, G, B (and A, else 1) by name, everything
// else ignored.  ZIP blocks are zlib streams of the predictor-coded,
// byte-interleaved scanline data (OpenEXR's ImfZip: a delta predictor over the
// bytes, then the even and odd bytes split into two halves).
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "image.h"

namespace mrt {
namespace {

float half_to_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h >> 15) << 31;
  const uint32_t exp = (h >> 10) & 0x1Fu, man = h & 0x3FFu;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else {   // subnormal half: renormalise
      int e = -1;
      uint32_t m = man;
      do { ++e; m <<= 1; } while (!(m & 0x400u));
      bits = sign | ((uint32_t)(127 - 15 - e) << 23) | ((m & 0x3FFu) << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (man << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

struct Channel { std::string name; int32_t type; };   // 0 UINT, 1 HALF, 2 FLOAT

template <class T>
bool rd(const std::vector<uint8_t>& b, size_t pos, T& v) {
  if (pos + sizeof(T) > b.size()) return false;
  std::memcpy(&v, b.data() + pos, sizeof(T));
  return true;
}

}  // namespace

bool load_exr(const std::string& path, std::vector<float>& rgba, uint32_t& width, uint32_t& height, std::string& err) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) { err = "cannot open " + path; return false; }
  std::vector<uint8_t> b;
  uint8_t chunk[1 << 16];
  size_t n;
  while ((n = std::fread(chunk, 1, sizeof(chunk), f)) > 0) b.insert(b.end(), chunk, chunk + n);
  std::fclose(f);
  uint32_t magic = 0, version = 0;
  if (!rd(b, 0, magic) || magic != 20000630u || !rd(b, 4, version)) { err = "not an OpenEXR file"; return false; }
  if (version & 0x1200u) { err = "tiled / multi-part EXR not supported"; return false; }
  // header attributes: name\0 type\0 int32 size, value
  size_t pos = 8;
  std::vector<Channel> chans;
  int comp = -1;
  int32_t win[4] = {0, 0, -1, -1};
  bool have_window = false;
  for (;;) {
    const size_t e1 = std::find(b.begin() + (long)pos, b.end(), 0) - b.begin();
    if (e1 >= b.size()) { err = "truncated EXR header"; return false; }
    const std::string name((const char*)b.data() + pos, e1 - pos);
    pos = e1 + 1;
    if (name.empty()) break;
    const size_t e2 = std::find(b.begin() + (long)pos, b.end(), 0) - b.begin();
    if (e2 >= b.size()) { err = "truncated EXR header"; return false; }
    const std::string type((const char*)b.data() + pos, e2 - pos);
    pos = e2 + 1;
    int32_t size = 0;
    if (!rd(b, pos, size) || size < 0 || pos + 4 + (size_t)size > b.size()) { err = "bad EXR attribute"; return false; }
    pos += 4;
    if (name == "channels") {
      size_t p = pos;
      while (p < pos + (size_t)size && b[p] != 0) {
        const size_t e = std::find(b.begin() + (long)p, b.begin() + (long)(pos + size), 0) - b.begin();
        Channel c{std::string((const char*)b.data() + p, e - p), 0};
        p = e + 1;
        if (!rd(b, p, c.type)) { err = "bad channel list"; return false; }
        p += 16;   // type, pLinear + 3 reserved, xSampling, ySampling
        chans.push_back(c);
      }
    } else if (name == "compression") {
      comp = b[pos];
    } else if (name == "dataWindow") {
      for (int k = 0; k < 4; ++k) rd(b, pos + 4 * k, win[k]);
      have_window = true;
    }
    pos += (size_t)size;
  }
  if (chans.empty() || !have_window) { err = "EXR without channels or dataWindow"; return false; }
  const int lines_per_block = comp == 0 || comp == 2 ? 1 : comp == 3 ? 16 : 0;
  if (!lines_per_block) { err = "unsupported EXR compression " + std::to_string(comp); return false; }
  const int64_t W = (int64_t)win[2] - win[0] + 1, H = (int64_t)win[3] - win[1] + 1;
  if (W <= 0 || H <= 0 || W * H > (1ll << 28)) { err = "bad EXR data window"; return false; }
  width = (uint32_t)W;
  height = (uint32_t)H;
  size_t pixel_bytes = 0;
  int slot[4] = {-1, -1, -1, -1};   // R, G, B, A -> channel index
  for (size_t c = 0; c < chans.size(); ++c) {
    if (chans[c].type < 0 || chans[c].type > 2) { err = "bad EXR channel type"; return false; }
    pixel_bytes += chans[c].type == 1 ? 2 : 4;
    const std::string& nm = chans[c].name;
    if (nm == "R") slot[0] = (int)c;
    else if (nm == "G") slot[1] = (int)c;
    else if (nm == "B") slot[2] = (int)c;
    else if (nm == "A") slot[3] = (int)c;
  }
  rgba.assign((size_t)W * H * 4, 0.0f);
  for (size_t i = 0; i < (size_t)W * H; ++i) rgba[4 * i + 3] = 1.0f;
  const int64_t blocks = (H + lines_per_block - 1) / lines_per_block;
  std::vector<uint8_t> raw, tmp;
  for (int64_t k = 0; k < blocks; ++k) {
    uint64_t off = 0;
    if (!rd(b, pos + 8 * (size_t)k, off)) { err = "truncated EXR offset table"; return false; }
    int32_t y = 0, size = 0;
    if (!rd(b, off, y) || !rd(b, off + 4, size) || size < 0 || off + 8 + (uint64_t)size > b.size()) {
      err = "bad EXR block";
      return false;
    }
    const int64_t nlines = std::min<int64_t>(lines_per_block, (int64_t)win[3] - y + 1);
    const size_t raw_size = pixel_bytes * (size_t)W * (size_t)nlines;
    const uint8_t* data = b.data() + off + 8;
    if (comp != 0 && (size_t)size < raw_size) {
      tmp.resize(raw_size);
      uLongf out_len = (uLongf)raw_size;
      if (uncompress(tmp.data(), &out_len, data, (uLong)size) != Z_OK || out_len != raw_size) {
        err = "EXR zlib block failed to inflate";
        return false;
      }
      for (size_t i = 1; i < raw_size; ++i) tmp[i] = (uint8_t)(tmp[i - 1] + tmp[i] - 128);   // predictor
      raw.resize(raw_size);
      const size_t half = (raw_size + 1) / 2;
      for (size_t i = 0; i < raw_size; ++i) raw[i] = (i & 1) ? tmp[half + i / 2] : tmp[i / 2];   // interleave
      data = raw.data();
    } else if ((size_t)size < raw_size) {
      err = "short uncompressed EXR block";
      return false;
    }
    size_t p = 0;
    for (int64_t ly = 0; ly < nlines; ++ly) {
      const int64_t row = y - win[1] + ly;   // EXR row 0 = top
      if (row < 0 || row >= H) { err = "EXR block outside the data window"; return false; }
      const int64_t out_row = H - 1 - row;   // ours: row 0 = bottom (Renderer.mm:233-235 flips too)
      for (size_t c = 0; c < chans.size(); ++c) {
        int comp_idx = -1;
        for (int s = 0; s < 4; ++s) if (slot[s] == (int)c) comp_idx = s;
        const int bytes = chans[c].type == 1 ? 2 : 4;
        if (comp_idx >= 0) {
          float* dst = &rgba[4 * (size_t)(out_row * W)];
          for (int64_t x = 0; x < W; ++x) {
            const uint8_t* q = data + p + (size_t)x * bytes;
            float v;
            if (chans[c].type == 1) { uint16_t hv; std::memcpy(&hv, q, 2); v = half_to_float(hv); }
            else if (chans[c].type == 2) { std::memcpy(&v, q, 4); }
            else { uint32_t u; std::memcpy(&u, q, 4); v = (float)u; }
            dst[4 * x + comp_idx] = v;
          }
        }
        p += (size_t)bytes * (size_t)W;
      }
    }
  }
  return true;
}

}  // namespace mrt
