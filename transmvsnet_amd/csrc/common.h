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
// Weight-gradient grids of (pixel-range block, tap) pairs as a 1-D grid of xcd_range_tap_grid(ntaps, nblk)
// blocks, dealt out so the ntaps blocks of one range share blockIdx % 8 -- one XCD, one L2: the taps
// gather overlapping input neighbourhoods and the same output-gradient rows. false for padding blocks.
#ifndef TMVS_WGRAD_XCD
#define TMVS_WGRAD_XCD 1
#endif
__device__ __forceinline__ bool xcd_range_tap(int ntaps, int nblk, int& rb, int& k) {
#if TMVS_WGRAD_XCD
  const int per = 8 * ntaps;
  const int grp = blockIdx.x / per, within = blockIdx.x % per;
  k = within / 8;
  rb = grp * 8 + within % 8;
  return rb < nblk;
#else
  (void)ntaps;
  (void)nblk;
  k = blockIdx.y;
  rb = blockIdx.x;
  return true;
#endif
}
static inline dim3 xcd_range_tap_grid(int ntaps, int nblk) {
  return TMVS_WGRAD_XCD ? dim3((unsigned)((nblk + 7) / 8 * 8 * ntaps)) : dim3((unsigned)nblk, (unsigned)ntaps);
}

// (b, y, x) of row v of a [B][H][W] pixel grid, for a loader whose wave's rows all lie in the 64-row chunk
// starting at v & ~63 (the weight-gradient reductions stage 64-row chunks from 64-aligned block starts):
// the chunk start's coordinates by one scalar (wave-uniform) division, the row's by carrying from it --
// instead of two divisions per lane and row
#ifndef TMVS_CHUNK_COORDS
#define TMVS_CHUNK_COORDS 1
#endif
__device__ __forceinline__ void chunk_row_coords(long v, int H, int W, int& b, int& y, int& x) {
  if (!TMVS_CHUNK_COORDS) {
    const long t = v / W;
    x = (int)(v - t * W);
    y = (int)(t % H);
    b = (int)(t / H);
    return;
  }
  const long vl = v & ~63L;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)vl);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long)vl >> 32));
  const long vb = (long)(((unsigned long)hi << 32) | lo);
  const long t = vb / W;
  x = (int)(vb - t * W) + (int)(v - vb);
  y = (int)(t % H);
  b = (int)(t / H);
  while (x >= W) {
    x -= W;
    if (++y == H) {
      y = 0;
      ++b;
    }
  }
}

// the same for row v of a [B][D][H][W] voxel grid: (b, z, y, x)
__device__ __forceinline__ void chunk_row_coords3(long v, int D, int H, int W, int& b, int& z, int& y, int& x) {
  if (!TMVS_CHUNK_COORDS) {
    long t = v / W;
    x = (int)(v - t * W);
    y = (int)(t % H);
    t /= H;
    z = (int)(t % D);
    b = (int)(t / D);
    return;
  }
  const long vl = v & ~63L;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)vl);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long)vl >> 32));
  const long vb = (long)(((unsigned long)hi << 32) | lo);
  long t = vb / W;
  x = (int)(vb - t * W) + (int)(v - vb);
  y = (int)(t % H);
  t /= H;
  z = (int)(t % D);
  b = (int)(t / D);
  while (x >= W) {
    x -= W;
    if (++y == H) {
      y = 0;
      if (++z == D) {
        z = 0;
        ++b;
      }
    }
  }
}

// The fp64 wave sum of the xor butterfly x += __shfl_xor(x, off), off = 32, 16, ..., 1 (the same pairs and
// operand order, so the same bits), with the partner moved by DPP row permutes for 1, 2, 4 (half mirror
// then quad reverse) and 8 (row mirror then half mirror), ds_swizzle (bit mode) for 16 and ds_bpermute for
// 32: 4 instead of 12 LDS-unit operations per value
template <int OFF>
__device__ __forceinline__ int xor_lane_dpp(int v) {
  if constexpr (OFF == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
  else if constexpr (OFF == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
  else if constexpr (OFF == 4)
    return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF, false);
  else if constexpr (OFF == 8)
    return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false), 0x141, 0xF, 0xF, false);
  else if constexpr (OFF == 16) return __builtin_amdgcn_ds_swizzle(v, 0x1F | (16 << 10));
  else return __shfl_xor(v, 32, 64);
}
template <int OFF>
__device__ __forceinline__ double xor_add_dpp(double x) {
  const int lo = xor_lane_dpp<OFF>(__double2loint(x)), hi = xor_lane_dpp<OFF>(__double2hiint(x));
  return x + __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_xor_sum_dpp(double x) {
  x = xor_add_dpp<32>(x);
  x = xor_add_dpp<16>(x);
  x = xor_add_dpp<8>(x);
  x = xor_add_dpp<4>(x);
  x = xor_add_dpp<2>(x);
  return xor_add_dpp<1>(x);
}

// s + p[j0 * stride] + p[(j0 + step) * stride] + ... (j < n), added in that order in fp64 -- the partial
// combines' fixed-order sums -- with 8 loads in flight ahead of their adds (a plain loop waits on each
// load before its dependent add)
#ifndef TMVS_SUM_BATCH
#define TMVS_SUM_BATCH 8
#endif
template <typename T>
__device__ __forceinline__ double strided_sum(const T* __restrict__ p, long j0, long n, long step, size_t stride,
                                              double s) {
  long j = j0;
  for (; j + (TMVS_SUM_BATCH - 1) * step < n; j += TMVS_SUM_BATCH * step) {
    T t[TMVS_SUM_BATCH];
#pragma unroll
    for (int u = 0; u < TMVS_SUM_BATCH; ++u) t[u] = p[(size_t)(j + u * step) * stride];
#pragma unroll
    for (int u = 0; u < TMVS_SUM_BATCH; ++u) s += (double)t[u];
  }
  for (; j < n; j += step) s += (double)p[(size_t)j * stride];
  return s;
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7;
  const int q = nblk >> 3, r = nblk & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Raw (stride 0) buffer resource over [base, base + bytes): 32-bit byte offsets, and any
// offset at or past `bytes` reads as 0 -- used for zero padding without branches (an
// out-of-image tap gets an out-of-range offset). Word 3 as for gfx9 raw buffers.
constexpr int kRsrcWord3 = 0x00020000;
constexpr unsigned kOffOut = 0x80000000u;  // an offset that is always out of range (bytes < 2^31)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, kRsrcWord3);
}
__device__ __forceinline__ float buf_load_f32(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));  // returns the raw bits
}
typedef float floatx4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ floatx4_t buf_load_f32x4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(floatx4_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// One pixel's softmax over D logits and winner-take-all (models/TransMVSNet.py:97-103,217-218):
// prob = exp((x - max) - log(sum exp(x - max))) stored through put_prob(d, p); returns the first
// maximum's index and its probability in best. Shared by softmax_wta_kernel (glue.hip) and the
// fused prob_wta_kernel (costreg.hip) so both produce the same bits.
template <int D, typename PutProb>
__device__ __forceinline__ int softmax_first_max(const float (&x)[D], PutProb put_prob, float& best) {
  float m = x[0];
#pragma unroll
  for (int d = 1; d < D; ++d) m = fmaxf(m, x[d]);
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) s = s + expf(x[d] - m);
  const float lse = logf(s);
  best = -1.f;
  int bi = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float pr = expf((x[d] - m) - lse);
    put_prob(d, pr);
    if (pr > best) {
      best = pr;
      bi = d;
    }
  }
  return bi;
}

}  // namespace tmvs

// fmt.hip: tmvs_fmt_apply with an explicit tiling (internal, used by tmvs_fmt_forward_split; the C-ABI entry point
// sizes the tiling from the kernel's occupancy)
int tmvs_fmt_apply_tiled(float* x, int nv, int l_tokens, const float* kv, long kv_view_stride, const float* enc_w,
                         int tiles_per_wave, void* stream);
