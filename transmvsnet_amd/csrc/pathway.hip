// FMT_with_pathway lateral step (models/FMT.py:195-228), fused:
//   out = smooth(bilinear_up2(reduce(coarse)) + lateral)
// reduce = 1x1 conv (no bias), bilinear align_corners=False (F.interpolate default, :209),
// smooth = 3x3 conv pad 1 (no bias). Weights arrive re-laid-out ([ci][co] and [ci][tap][co]) so
// every input value meets CF consecutive weights (one scalar load). A workgroup owns a 16x16 output tile: it reduces the
// 10x10 coarse pixels the tile's 18x18 halo interpolates from into LDS, builds the up-sampled
// + lateral halo in LDS, then each thread convolves one output pixel for all channels and
// writes it channels-last -- the layout the cost-volume kernel gathers from.
#include "common.h"

namespace tmvs {

constexpr int kTile = 16;
constexpr int kHalo = kTile + 2;
constexpr int kCoarse = kTile / 2 + 2;

struct Axis {
  int i0, i1;
  float l0, l1;
};

// The lateral halo values (NCHW, the FeatureNet output) do not depend on the coarse reduction:
// every thread requests its <= 2 halo pixels' CF channels before phase 1, so their HBM latency
// overlaps the reduction instead of sitting after the first barrier. Out-of-image pixels read 0.
#ifndef TMVS_PATHWAY_PREFETCH
#define TMVS_PATHWAY_PREFETCH 1
#endif
constexpr int kHaloIters = (kHalo * kHalo + 255) / 256;

// Tiles are dealt out XCD-contiguously over a 1-D grid (x fastest, then y, then view): consecutive
// block ids go to different XCDs, so with the plain 3-D grid a tile's x/y neighbours -- which read
// the same 128-B lines of the halo rows (an 18-float NCHW row spans 2-3 lines) -- sat behind
// different L2s and each re-fetched them.
#ifndef TMVS_PATHWAY_XCD
#define TMVS_PATHWAY_XCD 1
#endif
__device__ __forceinline__ void pathway_tile(int W, int H, int& v, int& y0, int& x0) {
#if TMVS_PATHWAY_XCD
  const int nbx = (W + kTile - 1) / kTile, nby = (H + kTile - 1) / kTile;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  x0 = (lb % nbx) * kTile;
  lb /= nbx;
  y0 = (lb % nby) * kTile;
  v = lb / nby;
#else
  v = blockIdx.z;
  y0 = blockIdx.y * kTile;
  x0 = blockIdx.x * kTile;
#endif
}

template <int CF>
__device__ __forceinline__ void load_lateral(const float* __restrict__ lv, int y0, int x0, int H, int W,
                                             float (&lat)[kHaloIters][CF]) {
#pragma unroll
  for (int it = 0; it < kHaloIters; ++it) {
    const int idx = threadIdx.x + 256 * it;
    const int r = idx / kHalo, c = idx - r * kHalo;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    const bool ok = idx < kHalo * kHalo && y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
    for (int o = 0; o < CF; ++o) lat[it][o] = ok ? lv[((size_t)o * H + y) * W + x] : 0.f;
  }
}

__device__ __forceinline__ Axis up_axis(int dst, int in_size, int out_size) {
  const float scale = (float)in_size / (float)out_size;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  Axis a;
  a.i0 = min((int)floorf(src), in_size - 1);
  a.i1 = a.i0 + (a.i0 < in_size - 1 ? 1 : 0);
  const float l = fminf(fmaxf(src - (float)a.i0, 0.f), 1.f);
  a.l1 = l;
  a.l0 = 1.f - l;
  return a;
}

template <int CC, int CF>
__global__ __launch_bounds__(256) void pathway_kernel(const float* __restrict__ coarse,
                                                      const float* __restrict__ lateral, long lat_stride,
                                                      const float* __restrict__ wred,
                                                      const float* __restrict__ wsm, int h, int w,
                                                      float* __restrict__ out) {
  __shared__ float red[CF][kCoarse][kCoarse + 1];
  __shared__ float inb[CF][kHalo][kHalo + 1];
  const int H = 2 * h, W = 2 * w;
  int v, y0, x0;
  pathway_tile(W, H, v, y0, x0);
  const int cy0 = y0 / 2 - 1, cx0 = x0 / 2 - 1;
  const float* cv = coarse + (size_t)v * h * w * CC;
  const float* lv = lateral + (size_t)v * lat_stride;
#if TMVS_PATHWAY_PREFETCH
  float lat[kHaloIters][CF];
  load_lateral<CF>(lv, y0, x0, H, W, lat);
#endif
  // 1) 1x1 reduction of the coarse patch
  for (int idx = threadIdx.x; idx < kCoarse * kCoarse; idx += blockDim.x) {
    const int r = idx / kCoarse, c = idx - r * kCoarse;
    const int cy = cy0 + r, cx = cx0 + c;
    if (cy < 0 || cy >= h || cx < 0 || cx >= w) continue;
    float xin[CC];
    const float* p = cv + ((size_t)cy * w + cx) * CC;
#pragma unroll
    for (int i4 = 0; i4 < CC / 4; ++i4) {
      const float4 t = *reinterpret_cast<const float4*>(p + 4 * i4);
      xin[4 * i4] = t.x;
      xin[4 * i4 + 1] = t.y;
      xin[4 * i4 + 2] = t.z;
      xin[4 * i4 + 3] = t.w;
    }
    float acc[CF];
#pragma unroll
    for (int o = 0; o < CF; ++o) acc[o] = 0.f;
#pragma unroll 2
    for (int i = 0; i < CC; ++i)
#pragma unroll
      for (int o = 0; o < CF; ++o) acc[o] = fmaf(wred[i * CF + o], xin[i], acc[o]);
#pragma unroll
    for (int o = 0; o < CF; ++o) red[o][r][c] = acc[o];
  }
  __syncthreads();
  // 2) bilinear x2 up-sampling + lateral over the 18x18 halo (zero outside the image)
#pragma unroll
  for (int it = 0; it < kHaloIters; ++it) {
    const int idx = threadIdx.x + 256 * it;
    if (idx >= kHalo * kHalo) break;
    const int r = idx / kHalo, c = idx - r * kHalo;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    if (y < 0 || y >= H || x < 0 || x >= W) {
#pragma unroll
      for (int o = 0; o < CF; ++o) inb[o][r][c] = 0.f;
      continue;
    }
    const Axis ay = up_axis(y, h, H), ax = up_axis(x, w, W);
    const int r0 = ay.i0 - cy0, r1 = ay.i1 - cy0, c0 = ax.i0 - cx0, c1 = ax.i1 - cx0;
#pragma unroll
    for (int o = 0; o < CF; ++o) {
      const float t0 = fmaf(red[o][r0][c0], ax.l0, red[o][r0][c1] * ax.l1);
      const float t1 = fmaf(red[o][r1][c0], ax.l0, red[o][r1][c1] * ax.l1);
      const float up = fmaf(t0, ay.l0, t1 * ay.l1);
#if TMVS_PATHWAY_PREFETCH
      inb[o][r][c] = up + lat[it][o];
#else
      inb[o][r][c] = up + lv[((size_t)o * H + y) * W + x];
#endif
    }
  }
  __syncthreads();
  // 3) 3x3 smoothing conv, one output pixel per thread
  const int ty = threadIdx.x / kTile, tx = threadIdx.x - ty * kTile;
  const int y = y0 + ty, x = x0 + tx;
  if (y >= H || x >= W) return;
  float acc[CF];
#pragma unroll
  for (int o = 0; o < CF; ++o) acc[o] = 0.f;
#pragma unroll 1
  for (int i = 0; i < CF; ++i) {
#pragma unroll 3
    for (int k = 0; k < 9; ++k) {
      const float xv = inb[i][ty + k / 3][tx + k % 3];
      const float* __restrict__ wk = wsm + (i * 9 + k) * CF;  // 16 consecutive weights: one s_load
#pragma unroll
      for (int o = 0; o < CF; ++o) acc[o] = fmaf(wk[o], xv, acc[o]);
    }
  }
  float4* op = reinterpret_cast<float4*>(out + (((size_t)v * H + y) * W + x) * CF);
#pragma unroll
  for (int o4 = 0; o4 < CF / 4; ++o4) op[o4] = make_float4(acc[4 * o4], acc[4 * o4 + 1], acc[4 * o4 + 2], acc[4 * o4 + 3]);
}

// Stage-3 form with R output rows per thread: a workgroup owns a 16 x 16R tile, so the two
// barriers, the coarse/halo staging and every scalar weight load are shared by R pixels. Tap
// (i, k) feeds the R accumulator sets back to back; each output's chain keeps pathway_kernel's
// (i, k, o) order, so the results are bitwise those of pathway_kernel.
#ifndef TMVS_PW_R
#define TMVS_PW_R 2
#endif
template <int CC, int CF, int R>
__global__ __launch_bounds__(256) void pathway_rows_kernel(const float* __restrict__ coarse,
                                                           const float* __restrict__ lateral, long lat_stride,
                                                           const float* __restrict__ wred,
                                                           const float* __restrict__ wsm, int h, int w,
                                                           float* __restrict__ out) {
  constexpr int TH = kTile * R, HH = TH + 2, CH = TH / 2 + 2;
  constexpr int NIT = (HH * kHalo + 255) / 256;
  __shared__ float red[CF][CH][kCoarse + 1];
  __shared__ float inb[CF][HH][kHalo + 1];
  const int H = 2 * h, W = 2 * w;
  const int nbx = (W + kTile - 1) / kTile, nby = (H + TH - 1) / TH;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int x0 = (lb % nbx) * kTile;
  lb /= nbx;
  const int y0 = (lb % nby) * TH;
  const int v = lb / nby;
  const int cy0 = y0 / 2 - 1, cx0 = x0 / 2 - 1;
  const float* cv = coarse + (size_t)v * h * w * CC;
  const float* lv = lateral + (size_t)v * lat_stride;
  float lat[NIT][CF];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = threadIdx.x + 256 * it;
    const int r = idx / kHalo, c = idx - r * kHalo;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    const bool ok = idx < HH * kHalo && y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
    for (int o = 0; o < CF; ++o) lat[it][o] = ok ? lv[((size_t)o * H + y) * W + x] : 0.f;
  }
  // 1) 1x1 reduction of the coarse patch
  for (int idx = threadIdx.x; idx < CH * kCoarse; idx += 256) {
    const int r = idx / kCoarse, c = idx - r * kCoarse;
    const int cy = cy0 + r, cx = cx0 + c;
    if (cy < 0 || cy >= h || cx < 0 || cx >= w) continue;
    float xin[CC];
    const float* p = cv + ((size_t)cy * w + cx) * CC;
#pragma unroll
    for (int i4 = 0; i4 < CC / 4; ++i4) {
      const float4 t = *reinterpret_cast<const float4*>(p + 4 * i4);
      xin[4 * i4] = t.x;
      xin[4 * i4 + 1] = t.y;
      xin[4 * i4 + 2] = t.z;
      xin[4 * i4 + 3] = t.w;
    }
    float acc[CF];
#pragma unroll
    for (int o = 0; o < CF; ++o) acc[o] = 0.f;
#pragma unroll 2
    for (int i = 0; i < CC; ++i)
#pragma unroll
      for (int o = 0; o < CF; ++o) acc[o] = fmaf(wred[i * CF + o], xin[i], acc[o]);
#pragma unroll
    for (int o = 0; o < CF; ++o) red[o][r][c] = acc[o];
  }
  __syncthreads();
  // 2) bilinear x2 up-sampling + lateral over the (16R+2) x 18 halo (zero outside the image)
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = threadIdx.x + 256 * it;
    if (idx >= HH * kHalo) break;
    const int r = idx / kHalo, c = idx - r * kHalo;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    if (y < 0 || y >= H || x < 0 || x >= W) {
#pragma unroll
      for (int o = 0; o < CF; ++o) inb[o][r][c] = 0.f;
      continue;
    }
    const Axis ay = up_axis(y, h, H), ax = up_axis(x, w, W);
    const int r0 = ay.i0 - cy0, r1 = ay.i1 - cy0, c0 = ax.i0 - cx0, c1 = ax.i1 - cx0;
#pragma unroll
    for (int o = 0; o < CF; ++o) {
      const float t0 = fmaf(red[o][r0][c0], ax.l0, red[o][r0][c1] * ax.l1);
      const float t1 = fmaf(red[o][r1][c0], ax.l0, red[o][r1][c1] * ax.l1);
      const float up = fmaf(t0, ay.l0, t1 * ay.l1);
      inb[o][r][c] = up + lat[it][o];
    }
  }
  __syncthreads();
  // 3) 3x3 smoothing conv, R vertically adjacent output pixels per thread (rows R*ty .. R*ty+R-1)
  const int ty = threadIdx.x / kTile, tx = threadIdx.x - ty * kTile;
  const int x = x0 + tx;
  if (x >= W || y0 + R * ty >= H) return;
  float acc[R][CF];
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int o = 0; o < CF; ++o) acc[q][o] = 0.f;
#pragma unroll 1
  for (int i = 0; i < CF; ++i) {
#pragma unroll 3
    for (int k = 0; k < 9; ++k) {
      const float* __restrict__ wk = wsm + (i * 9 + k) * CF;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const float xv = inb[i][R * ty + q + k / 3][tx + k % 3];
#pragma unroll
        for (int o = 0; o < CF; ++o) acc[q][o] = fmaf(wk[o], xv, acc[q][o]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int y = y0 + R * ty + q;
    if (y >= H) break;
    float4* op = reinterpret_cast<float4*>(out + (((size_t)v * H + y) * W + x) * CF);
#pragma unroll
    for (int o4 = 0; o4 < CF / 4; ++o4)
      op[o4] = make_float4(acc[q][4 * o4], acc[q][4 * o4 + 1], acc[q][4 * o4 + 2], acc[q][4 * o4 + 3]);
  }
}

// 16-channel variant (stage-2 pathway, the larger one): the 3x3 smoothing conv runs on fp32
// MFMA as an implicit GEMM -- M = 16 output channels, N = 16 pixels of a tile row,
// K = 16 channels x 9 taps -- with B fragments from the LDS halo and A fragments (weights) in
// VGPRs. The halo is stored [pixel][16 ch] with channels interleaved so a lane's 4 k-values
// (channels kgrp, 4+kgrp, 8+kgrp, 12+kgrp) are one ds_read_b128, quad-swizzled by pixel
// (bank-conflict free for 16 consecutive pixels, as in costreg.hip).
typedef float floatx4_p __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int halo16_index(int vox, int o) {
  const int q = (o & 3) ^ ((vox >> 1) & 3);
  return vox * 16 + q * 4 + (o >> 2);
}

template <int CC>
__global__ __launch_bounds__(256) void pathway16_mfma_kernel(const float* __restrict__ coarse,
                                                             const float* __restrict__ lateral, long lat_stride,
                                                             const float* __restrict__ wred,
                                                             const float* __restrict__ wsm, int h, int w,
                                                             float* __restrict__ out) {
  constexpr int CF = 16;
  __shared__ float red[CF][kCoarse][kCoarse + 1];
  __shared__ __attribute__((aligned(16))) float inb[kHalo * kHalo * CF];
  const int H = 2 * h, W = 2 * w;
  int v, y0, x0;
  pathway_tile(W, H, v, y0, x0);
  const int cy0 = y0 / 2 - 1, cx0 = x0 / 2 - 1;
  const float* cv = coarse + (size_t)v * h * w * CC;
  const float* lv = lateral + (size_t)v * lat_stride;
#if TMVS_PATHWAY_PREFETCH
  float lat[kHaloIters][CF];
  load_lateral<CF>(lv, y0, x0, H, W, lat);
#endif
  // 1) 1x1 reduction of the coarse patch (as pathway_kernel)
  for (int idx = threadIdx.x; idx < kCoarse * kCoarse; idx += blockDim.x) {
    const int r = idx / kCoarse, c = idx - r * kCoarse;
    const int cy = cy0 + r, cx = cx0 + c;
    if (cy < 0 || cy >= h || cx < 0 || cx >= w) continue;
    float xin[CC];
    const float* p = cv + ((size_t)cy * w + cx) * CC;
#pragma unroll
    for (int i4 = 0; i4 < CC / 4; ++i4) {
      const float4 t = *reinterpret_cast<const float4*>(p + 4 * i4);
      xin[4 * i4] = t.x;
      xin[4 * i4 + 1] = t.y;
      xin[4 * i4 + 2] = t.z;
      xin[4 * i4 + 3] = t.w;
    }
    float acc[CF];
#pragma unroll
    for (int o = 0; o < CF; ++o) acc[o] = 0.f;
#pragma unroll 2
    for (int i = 0; i < CC; ++i)
#pragma unroll
      for (int o = 0; o < CF; ++o) acc[o] = fmaf(wred[i * CF + o], xin[i], acc[o]);
#pragma unroll
    for (int o = 0; o < CF; ++o) red[o][r][c] = acc[o];
  }
  // A fragments meanwhile: lane (co = col, kgrp), tap t, k-step j -> W[co][ci = 4j + kgrp][t]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  float wa[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[t][j] = wsm[((4 * j + kgrp) * 9 + t) * CF + col];
  __syncthreads();
  // 2) bilinear x2 up-sampling + lateral over the 18x18 halo (zero outside the image)
#pragma unroll
  for (int it = 0; it < kHaloIters; ++it) {
    const int idx = threadIdx.x + 256 * it;
    if (idx >= kHalo * kHalo) break;
    const int r = idx / kHalo, c = idx - r * kHalo;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    if (y < 0 || y >= H || x < 0 || x >= W) {
#pragma unroll
      for (int o = 0; o < CF; ++o) inb[halo16_index(idx, o)] = 0.f;
      continue;
    }
    const Axis ay = up_axis(y, h, H), ax = up_axis(x, w, W);
    const int r0 = ay.i0 - cy0, r1 = ay.i1 - cy0, c0 = ax.i0 - cx0, c1 = ax.i1 - cx0;
#pragma unroll
    for (int o = 0; o < CF; ++o) {
      const float t0 = fmaf(red[o][r0][c0], ax.l0, red[o][r0][c1] * ax.l1);
      const float t1 = fmaf(red[o][r1][c0], ax.l0, red[o][r1][c1] * ax.l1);
      const float up = fmaf(t0, ay.l0, t1 * ay.l1);
#if TMVS_PATHWAY_PREFETCH
      inb[halo16_index(idx, o)] = up + lat[it][o];
#else
      inb[halo16_index(idx, o)] = up + lv[((size_t)o * H + y) * W + x];
#endif
    }
  }
  __syncthreads();
  // 3) 3x3 conv on MFMA: wave wv owns tile rows 4wv .. 4wv+3
  floatx4_p acc[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) acc[rr] = floatx4_p{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int kh = t / 3, kw = t % 3;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int vox = (4 * wv + rr + kh) * kHalo + col + kw;
      const float4 b = *reinterpret_cast<const float4*>(inb + vox * 16 + 4 * (kgrp ^ ((vox >> 1) & 3)));
      acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][0], b.x, acc[rr], 0, 0, 0);
      acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][1], b.y, acc[rr], 0, 0, 0);
      acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][2], b.z, acc[rr], 0, 0, 0);
      acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][3], b.w, acc[rr], 0, 0, 0);
    }
  }
  // D: lane (col, kgrp) holds output channels 4kgrp .. 4kgrp+3 of pixel (row, col)
  const int x = x0 + col;
  if (x >= W) return;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int y = y0 + 4 * wv + rr;
    if (y >= H) continue;
    *reinterpret_cast<float4*>(out + (((size_t)v * H + y) * W + x) * CF + 4 * kgrp) =
        make_float4(acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]);
  }
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_fmt_pathway(const float* coarse, const float* lateral, long lat_view_stride,
                                const float* w_reduce, const float* w_smooth, int nv, int cc, int cf, int h, int w,
                                float* out, void* stream) {
  if (!coarse || !lateral || !w_reduce || !w_smooth || !out || nv <= 0 || h <= 0 || w <= 0) return TMVS_ERR_ARG;
#if TMVS_PATHWAY_XCD
  const long nblk = (long)((2 * w + kTile - 1) / kTile) * ((2 * h + kTile - 1) / kTile) * nv;
  if (nblk > 0x7fffffffL) return TMVS_ERR_SHAPE;
  const dim3 grid((unsigned)nblk);
#else
  const dim3 grid((2 * w + kTile - 1) / kTile, (2 * h + kTile - 1) / kTile, nv);
#endif
  hipStream_t st = (hipStream_t)stream;
  if (cc == 32 && cf == 16)
    hipLaunchKernelGGL((pathway16_mfma_kernel<32>), grid, dim3(256), 0, st, coarse, lateral, lat_view_stride,
                       w_reduce, w_smooth, h, w, out);
  else if (cc == 16 && cf == 8) {
#if TMVS_PW_R > 1
    const long nrb = (long)((2 * w + kTile - 1) / kTile) * ((2 * h + kTile * TMVS_PW_R - 1) / (kTile * TMVS_PW_R)) * nv;
    hipLaunchKernelGGL((pathway_rows_kernel<16, 8, TMVS_PW_R>), dim3((unsigned)nrb), dim3(256), 0, st, coarse, lateral,
                       lat_view_stride, w_reduce, w_smooth, h, w, out);
#else
    hipLaunchKernelGGL((pathway_kernel<16, 8>), grid, dim3(256), 0, st, coarse, lateral, lat_view_stride, w_reduce,
                       w_smooth, h, w, out);
#endif
  }
  else
    return TMVS_ERR_SHAPE;
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
