// Host-side helpers shared by the launchers: error reporting, grid sizing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/pdivgnn.h"

namespace pdg {

void set_error(const char* fmt, ...);
int device_cus();

constexpr int MAX_BLOCKS = 2048;

#define PDG_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::pdg::set_error(__VA_ARGS__);        \
      return PDG_ERR_ARG;                   \
    }                                       \
  } while (0)

#define PDG_CHECK_LAUNCH(name)                                                    \
  do {                                                                            \
    hipError_t _e = hipGetLastError();                                            \
    if (_e != hipSuccess) {                                                       \
      ::pdg::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));     \
      return PDG_ERR_HIP;                                                         \
    }                                                                             \
  } while (0)

#define PDG_ALIGNED(p) ((((uintptr_t)(p)) & 15u) == 0)

// Wave tiles of 16 rows (pdg_common.hpp).
__host__ __device__ inline int tiles_of(long rows) { return (int)((rows + 15) / 16); }

// Persistent grid: enough blocks to cover the tiles, at most `per_cu` blocks per CU.
inline int persistent_grid(long rows, int waves_per_block, int per_cu) {
  long tiles = tiles_of(rows);
  long want = (tiles + waves_per_block - 1) / waves_per_block;
  long cap = (long)device_cus() * per_cu;
  if (cap > MAX_BLOCKS) cap = MAX_BLOCKS;
  long g = want < cap ? want : cap;
  return g < 1 ? 1 : (int)g;
}

}  // namespace pdg
