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

#ifndef TMVS_PW_ABL
#define TMVS_PW_ABL 0  // timing ablations of pathway16_mfma_kernel only (wrong results): 1 no coarse reduction,
#endif                 // 2 no lateral loads, 4 no MFMA conv, 8 no halo build
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
  if (TMVS_PW_ABL & 2) {
#pragma unroll
    for (int it = 0; it < kHaloIters; ++it)
#pragma unroll
      for (int o = 0; o < CF; ++o) lat[it][o] = (float)(it + o);
  } else {
    load_lateral<CF>(lv, y0, x0, H, W, lat);
  }
#endif
  // 1) 1x1 reduction of the coarse patch (as pathway_kernel)
  for (int idx = threadIdx.x; idx < kCoarse * kCoarse && !(TMVS_PW_ABL & 1); idx += blockDim.x) {
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
  for (int it = 0; it < kHaloIters && !(TMVS_PW_ABL & 8); ++it) {
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
  for (int t = 0; t < 9 && !(TMVS_PW_ABL & 4); ++t) {
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

// The same stage-2 pathway, software-pipelined over a run of tiles (round 6). pathway16_mfma_kernel
// runs its three phases back to back between two barriers, so per workgroup the coarse loads, the
// reduction, the halo build and the 144 MFMAs per wave follow one another and the MFMA pipe idles
// while a tile is staged. Here a 512-thread workgroup walks `tiles` consecutive tiles (rows fastest
// within a column, so consecutive tiles share halo rows) with two roles:
//   waves 0-3 (producers): per step s, the halo of tile s+1 (from red[(s+1)&1] and the lateral values
//     requested one step earlier) into inb[(s+1)&1], the coarse reduction of tile s+2 (coarse pixels
//     requested one step earlier) into red[s&1], then the next step's requests;
//   waves 4-7 (consumers): the 3x3 MFMA convolution of tile s from inb[s&1] and its store,
// and one barrier per step. Every value is computed by the same instructions in the same order as
// pathway16_mfma_kernel (bitwise identical). 55.5 KB of LDS: 2 workgroups (16 waves) per CU.
constexpr int kPipeThreads = 512;
#ifndef TMVS_PW_PIPE
#define TMVS_PW_PIPE 0
#endif
#ifndef TMVS_PW_PIPE_WGS
#define TMVS_PW_PIPE_WGS 512
#endif
#ifndef TMVS_PW_PIPE_SB
#define TMVS_PW_PIPE_SB 1
#endif
#ifndef TMVS_PW_PIPE_SG
#define TMVS_PW_PIPE_SG 0
#endif
#ifndef TMVS_PW_PIPE_ABL
#define TMVS_PW_PIPE_ABL 0  // timing ablations (wrong results): 1 consumers skip the MFMAs, 2 producers skip halo + reduction
#endif

template <int CC>
__global__ __launch_bounds__(kPipeThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void pathway16_pipe_kernel(const float* __restrict__ coarse,
                                                                     const float* __restrict__ lateral,
                                                                     long lat_stride,
                                                                     const float* __restrict__ wred,
                                                                     const float* __restrict__ wsm, int h, int w,
                                                                     int nv, int tiles, float* __restrict__ out) {
  constexpr int CF = 16;
  __shared__ float red[2][CF][kCoarse][kCoarse + 1];
  __shared__ __attribute__((aligned(16))) float inb[2][kHalo * kHalo * CF];
  const int H = 2 * h, W = 2 * w;
  const int nrow = (H + kTile - 1) / kTile, ncol = (W + kTile - 1) / kTile, per_view = nrow * ncol;
  // consecutive logical workgroups (neighbouring tile runs) on one XCD
  const int first = xcd_remap(blockIdx.x, gridDim.x) * tiles;
  const int nt = min(tiles, nv * per_view - first);  // uniform over the workgroup; >= 1 by the grid
  auto tile_of = [&](int k, int& v, int& y0, int& x0) {
    int l = first + k;
    v = l / per_view;
    l -= v * per_view;
    x0 = (l / nrow) * kTile;
    y0 = (l - (l / nrow) * nrow) * kTile;
  };
  const int tid = threadIdx.x;
  if (tid < 256) {
    // ---------------- producers ----------------
    // reduction: wave pw handles coarse pixels 64 (pw >> 1) + lane, output channels 8 (pw & 1) .. +7
    // (wave-uniform halves: the weights stay scalar loads); each output's FMA chain is pathway16_mfma_kernel's
    const int pw = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, so the weights are scalar loads
    const int lane = tid & 63, half = pw & 1, cp = (pw >> 1) * 64 + lane;
    const int cr = cp / kCoarse, cc = cp - cr * kCoarse;
    float lat[kHaloIters][CF];
    float xin[CC];
    bool xin_ok = false;
    auto load_coarse = [&](int k) {
      int v, y0, x0;
      tile_of(k, v, y0, x0);
      const int cy = y0 / 2 - 1 + cr, cx = x0 / 2 - 1 + cc;
      xin_ok = cp < kCoarse * kCoarse && cy >= 0 && cy < h && cx >= 0 && cx < w;
      if (xin_ok) {
        const float* p = coarse + (size_t)v * h * w * CC + ((size_t)cy * w + cx) * CC;
#pragma unroll
        for (int i4 = 0; i4 < CC / 4; ++i4) {
          const float4 t = *reinterpret_cast<const float4*>(p + 4 * i4);
          xin[4 * i4] = t.x;
          xin[4 * i4 + 1] = t.y;
          xin[4 * i4 + 2] = t.z;
          xin[4 * i4 + 3] = t.w;
        }
      }
    };
    // lateral halo values as load_lateral, through a buffer resource: one pixel offset per thread and a
    // scalar channel offset (no 64-bit address per channel); out-of-image pixels read 0 (out of range)
    auto load_lat = [&](int k) {
      int v, y0, x0;
      tile_of(k, v, y0, x0);
      const __amdgpu_buffer_rsrc_t rl = raw_rsrc(lateral + (size_t)v * lat_stride, (unsigned)(CF * H * W * 4));
#pragma unroll
      for (int it = 0; it < kHaloIters; ++it) {
        const int idx = tid + 256 * it;
        const int r = idx / kHalo, c = idx - r * kHalo;
        const int y = y0 - 1 + r, x = x0 - 1 + c;
        const bool ok = idx < kHalo * kHalo && y >= 0 && y < H && x >= 0 && x < W;
        const unsigned off = ok ? (unsigned)(y * W + x) * 4u : kOffOut;
#pragma unroll
        for (int o = 0; o < CF; ++o)
          lat[it][o] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rl, (int)off, o * H * W * 4, 0));
      }
    };
    // step s: halo of tile s+1 (lateral requested at step s-1), reduction of tile s+2 (coarse requested
    // at step s-1), then the requests for tiles s+2 (lateral) and s+3 (coarse)
    load_coarse(0);
    for (int s = -2; s < nt; ++s) {
      const int kh = s + 1;
      if (kh >= 0 && kh < nt && !(TMVS_PW_PIPE_ABL & 2)) {
        int v, y0, x0;
        tile_of(kh, v, y0, x0);
        const int cy0 = y0 / 2 - 1, cx0 = x0 / 2 - 1;
        const float(*rb)[kCoarse][kCoarse + 1] = red[kh & 1];
        float* ib = inb[kh & 1];
#pragma unroll
        for (int it = 0; it < kHaloIters; ++it) {
          const int idx = tid + 256 * it;
          if (idx >= kHalo * kHalo) break;
          const int r = idx / kHalo, c = idx - r * kHalo;
          const int y = y0 - 1 + r, x = x0 - 1 + c;
          const int sw = (idx >> 1) & 3;
          const bool in = y >= 0 && y < H && x >= 0 && x < W;
          // out-of-image halo pixels: computed at the nearest image pixel (inside the window), stored as 0
          const Axis ay = up_axis(min(max(y, 0), H - 1), h, H), ax = up_axis(min(max(x, 0), W - 1), w, W);
          const int r0 = ay.i0 - cy0, r1 = ay.i1 - cy0, c0 = ax.i0 - cx0, c1 = ax.i1 - cx0;
          // halo16_index layout: channels g + 4j (j = 0..3) are the float4 quad g ^ sw of the pixel
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float q[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int o = g + 4 * j;
              const float t0 = fmaf(rb[o][r0][c0], ax.l0, rb[o][r0][c1] * ax.l1);
              const float t1 = fmaf(rb[o][r1][c0], ax.l0, rb[o][r1][c1] * ax.l1);
              q[j] = in ? fmaf(t0, ay.l0, t1 * ay.l1) + lat[it][o] : 0.f;
            }
            *reinterpret_cast<float4*>(ib + idx * 16 + 4 * (g ^ sw)) = make_float4(q[0], q[1], q[2], q[3]);
#if TMVS_PW_PIPE_SB
            __builtin_amdgcn_sched_barrier(0);  // one channel group's LDS reads at a time (VGPR budget)
#endif
          }
        }
      }
      const int kr = s + 2;
      if (kr < nt && xin_ok && !(TMVS_PW_PIPE_ABL & 2)) {
        float acc[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) acc[o] = 0.f;
        const float* wr = wred + 8 * half;
#pragma unroll
        for (int i = 0; i < CC; ++i)
#pragma unroll
          for (int o = 0; o < 8; ++o) acc[o] = fmaf(wr[i * CF + o], xin[i], acc[o]);
#pragma unroll
        for (int o = 0; o < 8; ++o) red[kr & 1][8 * half + o][cr][cc] = acc[o];
      }
      if (s + 2 >= 0 && s + 2 < nt) load_lat(s + 2);
      if (s + 3 < nt) load_coarse(s + 3);
      __syncthreads();
    }
  } else {
    // ---------------- consumers ----------------
    const int lane = tid & 63, wv = (tid >> 6) - 4;
    const int col = lane & 15, kgrp = lane >> 4;
    float wa[9][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[t][j] = wsm[((4 * j + kgrp) * 9 + t) * CF + col];
    for (int s = -2; s < nt; ++s) {
      if (s >= 0) {
        const float* ib = inb[s & 1];
        floatx4_p acc[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = floatx4_p{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9 && !(TMVS_PW_PIPE_ABL & 1); ++t) {
          const int kh = t / 3, kw = t % 3;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int vox = (4 * wv + rr + kh) * kHalo + col + kw;
            const float4 b = *reinterpret_cast<const float4*>(ib + vox * 16 + 4 * (kgrp ^ ((vox >> 1) & 3)));
            acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][0], b.x, acc[rr], 0, 0, 0);
            acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][1], b.y, acc[rr], 0, 0, 0);
            acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][2], b.z, acc[rr], 0, 0, 0);
            acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][3], b.w, acc[rr], 0, 0, 0);
          }
        }
        int v, y0, x0;
        tile_of(s, v, y0, x0);
        const int x = x0 + col;
        if (x < W) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int y = y0 + 4 * wv + rr;
            if (y >= H) continue;
            *reinterpret_cast<float4*>(out + (((size_t)v * H + y) * W + x) * CF + 4 * kgrp) =
                make_float4(acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]);
          }
        }
      }
      __syncthreads();
    }
  }
}

// The pipeline without roles (TMVS_PW_PIPE=2): a 256-thread workgroup walks `tiles` tiles and in
// step s EVERY wave issues the 144 MFMAs of tile s (rows 4wv..4wv+3, from inb[s&1]), the halo of
// tile s+1 (into inb[(s+1)&1]), its share of the reduction of tile s+2 (into red[s&1]) and the
// requests for tiles s+2 (lateral) and s+3 (coarse) -- one basic block with no data dependence between
// the parts, so the scheduler can place the staging VALU / LDS work in the MFMAs' issue gaps (an MFMA
// holds vector issue for 8 of its 32 cycles). Branch-free staging: out-of-range pixels and coarse
// pixels load 0 through buffer resources and store 0 / duplicates; steps past the last tile recompute
// the last tile into buffers nobody reads. The reduction weights sit in LDS (broadcast reads), so no
// scalar load shares lgkmcnt with the LDS traffic. Same instructions per value as pathway16_mfma_kernel.
template <int CC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void pathway16_pipe2_kernel(
    const float* __restrict__ coarse, const float* __restrict__ lateral, long lat_stride,
    const float* __restrict__ wred, const float* __restrict__ wsm, int h, int w, int nv, int tiles,
    float* __restrict__ out) {
  constexpr int CF = 16;
  __shared__ float red[2][CF][kCoarse][kCoarse + 1];
  __shared__ __attribute__((aligned(16))) float inb[2][kHalo * kHalo * CF];
  __shared__ __attribute__((aligned(16))) float wl[CC * CF];
#if TMVS_PW_PIPE_SG == 2
  __shared__ __attribute__((aligned(16))) float wal[9 * 64 * 4];  // A fragments per (tap, lane): one ds_read_b128
#endif
  const int H = 2 * h, W = 2 * w;
  const int nrow = (H + kTile - 1) / kTile, ncol = (W + kTile - 1) / kTile, per_view = nrow * ncol;
  const int first = xcd_remap(blockIdx.x, gridDim.x) * tiles;
  const int nt = min(tiles, nv * per_view - first);
  auto tile_of = [&](int k, int& v, int& y0, int& x0) {
    int l = first + min(k, nt - 1);
    v = l / per_view;
    l -= v * per_view;
    x0 = (l / nrow) * kTile;
    y0 = (l - (l / nrow) * nrow) * kTile;
  };
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  for (int i = tid; i < CC * CF; i += 256) wl[i] = wred[i];
#if TMVS_PW_PIPE_SG == 2
  for (int i = tid; i < 9 * 64 * 4; i += 256) {
    const int t = i >> 8, l = (i >> 2) & 63, j = i & 3;
    wal[i] = wsm[((4 * j + (l >> 4)) * 9 + t) * CF + (l & 15)];
  }
#endif
  // MFMA role: lane (col, kgrp), A fragments = W[co = col][ci = 4j + kgrp][t]
  const int col = lane & 15, kgrp = lane >> 4;
#if TMVS_PW_PIPE_SG != 2
  float wa[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[t][j] = wsm[((4 * j + kgrp) * 9 + t) * CF + col];
#endif
  // reduction role: coarse pixel cp, output channels 8 half .. +7 (cp >= 100 lanes write the pad column)
  const int half = wv & 1, cp = (wv >> 1) * 64 + lane;
  const bool cp_ok = cp < kCoarse * kCoarse;
  const int cr = cp_ok ? cp / kCoarse : (cp - kCoarse * kCoarse) % kCoarse;
  const int cc = cp_ok ? cp - (cp / kCoarse) * kCoarse : kCoarse;
  float lat[kHaloIters][CF];
  float xin[CC];
  auto load_coarse = [&](int k) {
    int v, y0, x0;
    tile_of(k, v, y0, x0);
    const int cy = y0 / 2 - 1 + cr, cx = x0 / 2 - 1 + cc;
    const bool ok = cp_ok && cy >= 0 && cy < h && cx >= 0 && cx < w;
    const __amdgpu_buffer_rsrc_t rc = raw_rsrc(coarse + (size_t)v * h * w * CC, (unsigned)(h * w * CC * 4));
    const unsigned off = ok ? (unsigned)((cy * w + cx) * CC) * 4u : kOffOut;
#pragma unroll
    for (int i4 = 0; i4 < CC / 4; ++i4) {
      const floatx4_t t = buf_load_f32x4(rc, off + 16u * i4);
      xin[4 * i4] = t[0];
      xin[4 * i4 + 1] = t[1];
      xin[4 * i4 + 2] = t[2];
      xin[4 * i4 + 3] = t[3];
    }
  };
  auto load_lat = [&](int k) {
    int v, y0, x0;
    tile_of(k, v, y0, x0);
    const __amdgpu_buffer_rsrc_t rl = raw_rsrc(lateral + (size_t)v * lat_stride, (unsigned)(CF * H * W * 4));
#pragma unroll
    for (int it = 0; it < kHaloIters; ++it) {
      const int idx = min(tid + 256 * it, kHalo * kHalo - 1);
      const int r = idx / kHalo, c = idx - r * kHalo;
      const int y = y0 - 1 + r, x = x0 - 1 + c;
      const bool ok = y >= 0 && y < H && x >= 0 && x < W;
      const unsigned off = ok ? (unsigned)(y * W + x) * 4u : kOffOut;
#pragma unroll
      for (int o = 0; o < CF; ++o)
        lat[it][o] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rl, (int)off, o * H * W * 4, 0));
    }
  };
  auto halo = [&](int k) {
    int v, y0, x0;
    tile_of(k, v, y0, x0);
    const int cy0 = y0 / 2 - 1, cx0 = x0 / 2 - 1;
    const float(*rb)[kCoarse][kCoarse + 1] = red[k & 1];
    float* ib = inb[k & 1];
#pragma unroll
    for (int it = 0; it < kHaloIters; ++it) {
      const int idx = min(tid + 256 * it, kHalo * kHalo - 1);  // surplus lanes duplicate the last pixel
      const int r = idx / kHalo, c = idx - r * kHalo;
      const int y = y0 - 1 + r, x = x0 - 1 + c;
      const int sw = (idx >> 1) & 3;
      const bool in = y >= 0 && y < H && x >= 0 && x < W;
      const Axis ay = up_axis(min(max(y, 0), H - 1), h, H), ax = up_axis(min(max(x, 0), W - 1), w, W);
      const int r0 = ay.i0 - cy0, r1 = ay.i1 - cy0, c0 = ax.i0 - cx0, c1 = ax.i1 - cx0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int o = g + 4 * j;
          const float t0 = fmaf(rb[o][r0][c0], ax.l0, rb[o][r0][c1] * ax.l1);
          const float t1 = fmaf(rb[o][r1][c0], ax.l0, rb[o][r1][c1] * ax.l1);
          const float val = fmaf(t0, ay.l0, t1 * ay.l1) + lat[it][o];
          q[j] = in ? val : 0.f;
        }
        *reinterpret_cast<float4*>(ib + idx * 16 + 4 * (g ^ sw)) = make_float4(q[0], q[1], q[2], q[3]);
      }
    }
  };
  auto reduce = [&](int k) {
    float acc[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) acc[o] = 0.f;
    const float* wr = wl + 8 * half;
#pragma unroll
    for (int i = 0; i < CC; ++i) {
      const float4 wlo = *reinterpret_cast<const float4*>(wr + i * CF);
      const float4 whi = *reinterpret_cast<const float4*>(wr + i * CF + 4);
      acc[0] = fmaf(wlo.x, xin[i], acc[0]);
      acc[1] = fmaf(wlo.y, xin[i], acc[1]);
      acc[2] = fmaf(wlo.z, xin[i], acc[2]);
      acc[3] = fmaf(wlo.w, xin[i], acc[3]);
      acc[4] = fmaf(whi.x, xin[i], acc[4]);
      acc[5] = fmaf(whi.y, xin[i], acc[5]);
      acc[6] = fmaf(whi.z, xin[i], acc[6]);
      acc[7] = fmaf(whi.w, xin[i], acc[7]);
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) red[k & 1][8 * half + o][cr][cc] = acc[o];
  };
#if TMVS_PW_PIPE_SG != 2
  auto conv = [&](int k, floatx4_p (&acc)[4]) {
    const float* ib = inb[k & 1];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) acc[rr] = floatx4_p{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int vox = (4 * wv + rr + kh) * kHalo + col + kw;
        const float4 b = *reinterpret_cast<const float4*>(ib + vox * 16 + 4 * (kgrp ^ ((vox >> 1) & 3)));
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][0], b.x, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][1], b.y, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][2], b.z, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][3], b.w, acc[rr], 0, 0, 0);
      }
    }
  };
#endif
  auto store = [&](int k, const floatx4_p (&acc)[4]) {
    int v, y0, x0;
    tile_of(k, v, y0, x0);
    const int x = x0 + col;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int y = y0 + 4 * wv + rr;
      if (x < W && y < H)
        *reinterpret_cast<float4*>(out + (((size_t)v * H + y) * W + x) * CF + 4 * kgrp) =
            make_float4(acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]);
    }
  };
  // prologue: reduction of tiles 0, 1 and halo of tile 0
  load_coarse(0);
  __syncthreads();  // wl
  load_lat(0);
  reduce(0);
  load_coarse(1);
  __syncthreads();
  halo(0);
  reduce(1);
  load_lat(1);
  load_coarse(2);
  __syncthreads();
  // TMVS_PW_PIPE_SG == 2: the step interleaved by hand. Per tap t the next tap's B fragments are
  // requested, the 16 MFMAs of tap t issued, then one staging piece (halo pixel block it = t/4, channel
  // group t%4; reduction quarter q after taps 1, 3, 5, 7); a scheduling barrier per tap keeps the order.
  auto step_interleaved = [&](int s, floatx4_p (&acc)[4]) {
    const float* ib = inb[s & 1];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) acc[rr] = floatx4_p{0.f, 0.f, 0.f, 0.f};
    int v1, y1, x1;
    tile_of(s + 1, v1, y1, x1);
    const int hcy0 = y1 / 2 - 1, hcx0 = x1 / 2 - 1;
    const float(*rb)[kCoarse][kCoarse + 1] = red[(s + 1) & 1];
    float* hb = inb[(s + 1) & 1];
    int hidx = 0, hsw = 0, hr0 = 0, hr1 = 0, hc0 = 0, hc1 = 0;
    bool hin = false;
    float hy0 = 0.f, hy1 = 0.f, hx0 = 0.f, hx1 = 0.f;
    float racc[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) racc[o] = 0.f;
    const float* wr = wl + 8 * half;
    float4 bc[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int vox = (4 * wv + rr) * kHalo + col;
      bc[rr] = *reinterpret_cast<const float4*>(ib + vox * 16 + 4 * (kgrp ^ ((vox >> 1) & 3)));
    }
    float4 at = *reinterpret_cast<const float4*>(wal + 4 * lane);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(at.x, bc[rr].x, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(at.y, bc[rr].y, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(at.z, bc[rr].z, acc[rr], 0, 0, 0);
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(at.w, bc[rr].w, acc[rr], 0, 0, 0);
      }
      if (t < 8) at = *reinterpret_cast<const float4*>(wal + 256 * (t + 1) + 4 * lane);
      if (t < 8) {  // next tap's B fragments; their latency is covered by the staging piece
        const int kh = (t + 1) / 3, kw = (t + 1) % 3;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int vox = (4 * wv + rr + kh) * kHalo + col + kw;
          bc[rr] = *reinterpret_cast<const float4*>(ib + vox * 16 + 4 * (kgrp ^ ((vox >> 1) & 3)));
        }
      }
      if ((t & 3) == 0 && t < 8) {  // halo geometry of pixel block t / 4 of tile s+1
        const int it = t >> 2;
        const int idx = min(tid + 256 * it, kHalo * kHalo - 1);
        const int r = idx / kHalo, c = idx - r * kHalo;
        const int y = y1 - 1 + r, x = x1 - 1 + c;
        hidx = idx;
        hsw = (idx >> 1) & 3;
        hin = y >= 0 && y < H && x >= 0 && x < W;
        const Axis ay = up_axis(min(max(y, 0), H - 1), h, H), ax = up_axis(min(max(x, 0), W - 1), w, W);
        hr0 = ay.i0 - hcy0;
        hr1 = ay.i1 - hcy0;
        hc0 = ax.i0 - hcx0;
        hc1 = ax.i1 - hcx0;
        hy0 = ay.l0;
        hy1 = ay.l1;
        hx0 = ax.l0;
        hx1 = ax.l1;
      }
      if (t < 8) {  // halo piece: pixel block t / 4, channel group t % 4
        const int it = t >> 2, g = t & 3;
        float q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int o = g + 4 * j;
          const float t0 = fmaf(rb[o][hr0][hc0], hx0, rb[o][hr0][hc1] * hx1);
          const float t1 = fmaf(rb[o][hr1][hc0], hx0, rb[o][hr1][hc1] * hx1);
          const float val = fmaf(t0, hy0, t1 * hy1) + lat[it][o];
          q[j] = hin ? val : 0.f;
        }
        *reinterpret_cast<float4*>(hb + hidx * 16 + 4 * (g ^ hsw)) = make_float4(q[0], q[1], q[2], q[3]);
      }
      if (t & 1) {  // reduction quarter (t - 1) / 2 of tile s+2
        const int i0 = 8 * ((t - 1) >> 1);
#pragma unroll
        for (int i = i0; i < i0 + 8; ++i) {
          const float4 wlo = *reinterpret_cast<const float4*>(wr + i * CF);
          const float4 whi = *reinterpret_cast<const float4*>(wr + i * CF + 4);
          racc[0] = fmaf(wlo.x, xin[i], racc[0]);
          racc[1] = fmaf(wlo.y, xin[i], racc[1]);
          racc[2] = fmaf(wlo.z, xin[i], racc[2]);
          racc[3] = fmaf(wlo.w, xin[i], racc[3]);
          racc[4] = fmaf(whi.x, xin[i], racc[4]);
          racc[5] = fmaf(whi.y, xin[i], racc[5]);
          racc[6] = fmaf(whi.z, xin[i], racc[6]);
          racc[7] = fmaf(whi.w, xin[i], racc[7]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) red[s & 1][8 * half + o][cr][cc] = racc[o];
  };
  for (int s = 0; s < nt; ++s) {
    floatx4_p acc[4];
#if TMVS_PW_PIPE_SG == 2
    step_interleaved(s, acc);
#else
    conv(s, acc);
    halo(s + 1);
    reduce(s + 2);
#endif
#if TMVS_PW_PIPE_SG == 1
    // interleave the staging work into the MFMA stream: per MFMA up to 4 VALU, 1 LDS read, 2 SALU
#pragma unroll
    for (int i = 0; i < 144; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x004, 2, 0);
    }
#endif
    load_lat(s + 2);
    load_coarse(s + 3);
    store(s, acc);
    __syncthreads();
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
  if (cc == 32 && cf == 16) {
#if TMVS_PW_PIPE
    // runs of `tiles` tiles, about TMVS_PW_PIPE_WGS workgroups: one round at 2 per CU on 256 CUs
    const long total = (long)((2 * w + kTile - 1) / kTile) * ((2 * h + kTile - 1) / kTile) * nv;
    if (total > 0x7fffffffL) return TMVS_ERR_SHAPE;
    const long tiles = (total + TMVS_PW_PIPE_WGS - 1) / TMVS_PW_PIPE_WGS;
    const long nwg = (total + tiles - 1) / tiles;
#if TMVS_PW_PIPE == 2
    hipLaunchKernelGGL((pathway16_pipe2_kernel<32>), dim3((unsigned)nwg), dim3(256), 0, st, coarse, lateral,
                       lat_view_stride, w_reduce, w_smooth, h, w, nv, (int)tiles, out);
#else
    hipLaunchKernelGGL((pathway16_pipe_kernel<32>), dim3((unsigned)nwg), dim3(kPipeThreads), 0, st, coarse, lateral,
                       lat_view_stride, w_reduce, w_smooth, h, w, nv, (int)tiles, out);
#endif
#else
    hipLaunchKernelGGL((pathway16_mfma_kernel<32>), grid, dim3(256), 0, st, coarse, lateral, lat_view_stride,
                       w_reduce, w_smooth, h, w, out);
#endif
  } else if (cc == 16 && cf == 8) {
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
