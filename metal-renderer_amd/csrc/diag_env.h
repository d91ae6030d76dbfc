// diag_env.h — the library's diagnostic environment variables (DESIGN.md
// §5.1: kernel / batch / stream / BVH-builder overrides used by the A/B
// measurements) are read only when MRT_DIAG=1 is set, so a host that
// integrates libmrt never inherits a stray MRT_* variable: without MRT_DIAG
// every default is the product configuration.
#pragma once
#include <cstdlib>

namespace mrt {

inline const char* diag_env(const char* name) {
  const char* d = std::getenv("MRT_DIAG");
  return (d && d[0] == '1' && d[1] == '\0') ? std::getenv(name) : nullptr;
}

}  // namespace mrt
