// Shared helpers for the TransMVSNet MI355X (gfx950) kernels.
//
// Numerics policy: every translation unit is compiled with -ffp-contract=off so
// that a*b+c is two roundings unless a kernel writes fmaf() explicitly. The
// explicit fmaf() calls reproduce the FMA contractions the reference's PyTorch-CPU
// kernels perform (grid_sample bilinear, batch_norm, bilinear upsampling, bmm),
// measured in DESIGN.md "Numerics".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/transmvs.h"

#define TMVS_CHECK_LAUNCH()                                   \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return TMVS_ERR_HIP;                \
  } while (0)

namespace tmvs {

constexpr int kWave = 64;

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// Bijective XCD-aware block remap (cdna_hip_programming.md T1): blocks b and b+8 share
// an XCD, so give each XCD a contiguous chunk of the tile space.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7;
  const int q = nblk >> 3, r = nblk & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace tmvs
