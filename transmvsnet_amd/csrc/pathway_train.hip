// FMT_with_pathway lateral step for training: the pieces of
// out = smooth(up2(reduce(coarse)) + lateral) (models/FMT.py:201-209, 221-228) that autograd needs
// besides the convolutions (those run on tmvs_conv3d_generic / tmvs_conv3d_wgrad with a depth of 1).
//   tmvs_upsample2_add_nhwc      u = F.interpolate(r, 2x, bilinear, align_corners=False) + lateral
//   tmvs_upsample2_backward_nhwc dr = the adjoint of that interpolation (a gather over the <= 4x4
//                                fine pixels whose bilinear sample reads each coarse pixel)
// Source index math: area_pixel_compute_source_index (align_corners=False): src = 0.5*(dst+0.5)-0.5,
// clamped at 0; i0 = floor(src), i1 = i0 + (i0 < in-1), l1 = src - i0 (upsample_bilinear2d).
#include "common.h"

namespace tmvs {

struct Lin1 {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Lin1 lin_x2(int dst, int in_size) {
  float src = 0.5f * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  Lin1 a;
  a.i0 = (int)src;  // src >= 0: truncation == floor
  a.i0 = a.i0 < in_size - 1 ? a.i0 : in_size - 1;
  a.i1 = a.i0 + (a.i0 < in_size - 1 ? 1 : 0);
  a.l1 = src - (float)a.i0;
  a.l0 = 1.f - a.l1;
  return a;
}

// u[n][y][x][c] = (h0 * (w0 * r[y0][x0] + w1 * r[y0][x1]) + h1 * (w0 * r[y1][x0] + w1 * r[y1][x1])) + lateral[n][c][y][x]
template <int C>
__global__ __launch_bounds__(256) void upsample2_add_kernel(const float* __restrict__ r, const float* __restrict__ lat,
                                                            int N, int h, int w, float* __restrict__ u) {
  const int H = 2 * h, W = 2 * w;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * H * W) return;
  const int x = (int)(i % W);
  const int y = (int)((i / W) % H);
  const int n = (int)(i / ((long)W * H));
  const Lin1 ay = lin_x2(y, h), ax = lin_x2(x, w);
  const float* rb = r + (size_t)n * h * w * C;
  const float* p00 = rb + ((size_t)ay.i0 * w + ax.i0) * C;
  const float* p01 = rb + ((size_t)ay.i0 * w + ax.i1) * C;
  const float* p10 = rb + ((size_t)ay.i1 * w + ax.i0) * C;
  const float* p11 = rb + ((size_t)ay.i1 * w + ax.i1) * C;
  float* out = u + (size_t)i * C;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float t0 = ax.l0 * p00[c] + ax.l1 * p01[c];
    const float t1 = ax.l0 * p10[c] + ax.l1 * p11[c];
    out[c] = (ay.l0 * t0 + ay.l1 * t1) + lat[(((size_t)n * C + c) * H + y) * W + x];
  }
}

// dr[n][i][j][c] = sum over fine (y, x) reading coarse (i, j) of wy * wx * du[n][y][x][c]
template <int C>
__global__ __launch_bounds__(256) void upsample2_backward_kernel(const float* __restrict__ du, int N, int h, int w,
                                                                 float* __restrict__ dr) {
  const int H = 2 * h, W = 2 * w;
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)N * h * w) return;
  const int j = (int)(q % w);
  const int i = (int)((q / w) % h);
  const int n = (int)(q / ((long)w * h));
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  for (int y = 2 * i - 1; y <= 2 * i + 2; ++y) {
    if (y < 0 || y >= H) continue;
    const Lin1 ay = lin_x2(y, h);
    const float wy = (ay.i0 == i ? ay.l0 : 0.f) + (ay.i1 == i ? ay.l1 : 0.f);
    if (wy == 0.f) continue;
    for (int x = 2 * j - 1; x <= 2 * j + 2; ++x) {
      if (x < 0 || x >= W) continue;
      const Lin1 ax = lin_x2(x, w);
      const float wx = (ax.i0 == j ? ax.l0 : 0.f) + (ax.i1 == j ? ax.l1 : 0.f);
      if (wx == 0.f) continue;
      const float ww = wy * wx;
      const float* g = du + (((size_t)n * H + y) * W + x) * C;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = fmaf(ww, g[c], acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) dr[(size_t)q * C + c] = acc[c];
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_upsample2_add_nhwc(const float* r, const float* lateral, int n, int h, int w, int channels,
                                       float* u, void* stream) {
  if (!r || !lateral || !u || n <= 0 || h <= 0 || w <= 0) return TMVS_ERR_ARG;
  const long tot = (long)n * 4 * h * w;
  const dim3 grid((unsigned)((tot + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  switch (channels) {
    case 8: hipLaunchKernelGGL(upsample2_add_kernel<8>, grid, dim3(256), 0, st, r, lateral, n, h, w, u); break;
    case 16: hipLaunchKernelGGL(upsample2_add_kernel<16>, grid, dim3(256), 0, st, r, lateral, n, h, w, u); break;
    default: return TMVS_ERR_SHAPE;
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_upsample2_backward_nhwc(const float* du, int n, int h, int w, int channels, float* dr,
                                            void* stream) {
  if (!du || !dr || n <= 0 || h <= 0 || w <= 0) return TMVS_ERR_ARG;
  const long tot = (long)n * h * w;
  const dim3 grid((unsigned)((tot + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  switch (channels) {
    case 8: hipLaunchKernelGGL(upsample2_backward_kernel<8>, grid, dim3(256), 0, st, du, n, h, w, dr); break;
    case 16: hipLaunchKernelGGL(upsample2_backward_kernel<16>, grid, dim3(256), 0, st, du, n, h, w, dr); break;
    default: return TMVS_ERR_SHAPE;
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
