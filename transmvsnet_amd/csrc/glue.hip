// Stage glue (depth hypotheses) and softmax / winner-take-all regression.
//
// Hypotheses: models/TransMVSNet.py:147-149,174-204 + get_depth_samples models/module.py:606-634.
// The reference materialises the full-resolution [B,D,H,W] samples (127 MB at DTU stage 2)
// and trilinearly resamples them; here each stage-resolution output evaluates the 1 (stage 3)
// or 2x2 (stage 2) full-resolution samples it averages, in the reference's fp32 op order:
//   cur  = fmaf(fmaf(x00,w0, x01*w1), h0, fmaf(x10,w0, x11*w1)*h1)   bilinear x2/x4 up-sampling
//   hyp  = (cur - hr) + k * (((cur + hr) - (cur - hr)) / (nd - 1))
//   out  = fmaf(fmaf(a,.5,b*.5), .5, fmaf(c,.5,d*.5)*.5)              trilinear 2x down (stage 2)
// Regression: models/TransMVSNet.py:97-103,217-221, depth_wta models/module.py:474-482.
#include "common.h"

namespace tmvs {

struct LinAxis {
  int i0, i1;
  float l0, l1;
};

// area_pixel_compute_source_index + guard_index_and_lambda (align_corners=False, linear)
__device__ __forceinline__ LinAxis lin_axis(int dst, int in_size, int out_size) {
  const float scale = (float)in_size / (float)out_size;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  LinAxis a;
  a.i0 = min((int)floorf(src), in_size - 1);
  a.i1 = a.i0 + (a.i0 < in_size - 1 ? 1 : 0);
  float l = src - (float)a.i0;
  l = fminf(fmaxf(l, 0.f), 1.f);
  a.l1 = l;
  a.l0 = 1.f - l;
  return a;
}

__device__ __forceinline__ float upsample_at(const float* __restrict__ prev, int ph, int pw, int y, int x, int H,
                                             int W) {
  const LinAxis ay = lin_axis(y, ph, H);
  const LinAxis ax = lin_axis(x, pw, W);
  const float* r0 = prev + (size_t)ay.i0 * pw;
  const float* r1 = prev + (size_t)ay.i1 * pw;
  const float t0 = fmaf(r0[ax.i0], ax.l0, r0[ax.i1] * ax.l1);
  const float t1 = fmaf(r1[ax.i0], ax.l0, r1[ax.i1] * ax.l1);
  return fmaf(t0, ay.l0, t1 * ay.l1);
}

__global__ void hyp_stage1_kernel(const float* __restrict__ dv, int n_values, int nd, int HWs,
                                  float* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HWs) return;
  const float dmin = dv[(size_t)b * n_values], dmax = dv[(size_t)b * n_values + n_values - 1];
  const float interval = (dmax - dmin) / (float)(nd - 1);
  float* o = out + (size_t)b * nd * HWs + p;
  for (int k = 0; k < nd; ++k) o[(size_t)k * HWs] = dmin + (float)k * interval;
}

template <int SCALE>
__global__ void hyp_refine_kernel(const float* __restrict__ dv, int n_values, const float* __restrict__ prev, int ph,
                                  int pw, int nd, float ratio, int H, int W, float* __restrict__ out) {
  const int Hs = H / SCALE, Ws = W / SCALE;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= Hs * Ws) return;
  const int i = p / Ws, j = p - i * Ws;
  // depth_interval from batch 0 in double, as the Python scalars of TransMVSNet.py:147-149
  const double depth_min = (double)dv[0], depth_max = (double)dv[n_values - 1];
  const double depth_interval = (depth_max - depth_min) / (double)n_values;
  const float hr = (float)(((double)nd / 2.0) * ((double)ratio * depth_interval));
  const float* pb = prev + (size_t)b * ph * pw;
  float* o = out + (size_t)b * nd * Hs * Ws + p;
  const float den = (float)(nd - 1);
  if constexpr (SCALE == 1) {
    const float cur = upsample_at(pb, ph, pw, i, j, H, W);
    const float lo = cur - hr, hi = cur + hr;
    const float iv = (hi - lo) / den;
    for (int k = 0; k < nd; ++k) o[(size_t)k * Hs * Ws] = lo + (float)k * iv;
  } else {
    float lo[4], iv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float cur = upsample_at(pb, ph, pw, 2 * i + (q >> 1), 2 * j + (q & 1), H, W);
      lo[q] = cur - hr;
      iv[q] = ((cur + hr) - lo[q]) / den;
    }
    for (int k = 0; k < nd; ++k) {
      const float fk = (float)k;
      const float a = lo[0] + fk * iv[0], bb = lo[1] + fk * iv[1];
      const float c = lo[2] + fk * iv[2], d = lo[3] + fk * iv[3];
      o[(size_t)k * Hs * Ws] = fmaf(fmaf(a, 0.5f, bb * 0.5f), 0.5f, fmaf(c, 0.5f, d * 0.5f) * 0.5f);
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void softmax_wta_kernel(const float* __restrict__ logits,
                                                          const float* __restrict__ hyp, int HW, float lo, float hi,
                                                          float* __restrict__ prob, float* __restrict__ depth,
                                                          float* __restrict__ depth_raw, float* __restrict__ conf) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  const size_t base = (size_t)blockIdx.y * D * HW + p;
  float x[D];
#pragma unroll
  for (int d = 0; d < D; ++d) x[d] = logits[base + (size_t)d * HW];
  float best;
  const int bi = softmax_first_max<D>(x, [&](int d, float pr) { prob[base + (size_t)d * HW] = pr; }, best);
  const size_t o = (size_t)blockIdx.y * HW + p;
  const float dr = hyp[base + (size_t)bi * HW];
  depth_raw[o] = dr;
  depth[o] = fminf(fmaxf(dr, lo), hi);
  conf[o] = best;
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_stage_hypotheses(const float* depth_values, int n_values, const float* prev_depth, int prev_h,
                                     int prev_w, int batch, int ndepth, float ratio, int full_h, int full_w,
                                     int stage_scale, float* hyp_out, void* stream) {
  if (!depth_values || !hyp_out || n_values < 2 || batch <= 0 || ndepth < 2 || full_h <= 0 || full_w <= 0)
    return TMVS_ERR_ARG;
  if (stage_scale != 1 && stage_scale != 2 && stage_scale != 4) return TMVS_ERR_ARG;
  if (full_h % stage_scale || full_w % stage_scale) return TMVS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int HWs = (full_h / stage_scale) * (full_w / stage_scale);
  const dim3 grid((HWs + 255) / 256, batch);
  if (!prev_depth) {
    hipLaunchKernelGGL(hyp_stage1_kernel, grid, dim3(256), 0, st, depth_values, n_values, ndepth, HWs, hyp_out);
  } else {
    if (prev_h <= 0 || prev_w <= 0) return TMVS_ERR_ARG;
    if (stage_scale == 2)
      hipLaunchKernelGGL(hyp_refine_kernel<2>, grid, dim3(256), 0, st, depth_values, n_values, prev_depth, prev_h,
                         prev_w, ndepth, ratio, full_h, full_w, hyp_out);
    else if (stage_scale == 1)
      hipLaunchKernelGGL(hyp_refine_kernel<1>, grid, dim3(256), 0, st, depth_values, n_values, prev_depth, prev_h,
                         prev_w, ndepth, ratio, full_h, full_w, hyp_out);
    else
      return TMVS_ERR_SHAPE;  // the reference never refines at 1/4 resolution
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_softmax_wta(const float* logits, const float* hyp, int batch, int ndepth, int height, int width,
                                float clamp_lo, float clamp_hi, float* prob, float* depth, float* depth_raw,
                                float* conf, void* stream) {
  if (!logits || !hyp || !prob || !depth || !depth_raw || !conf || batch <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  const int HW = height * width;
  const dim3 grid((HW + 255) / 256, batch);
  hipStream_t st = (hipStream_t)stream;
#define TMVS_SM_CASE(DD)                                                                                       \
  case DD:                                                                                                     \
    hipLaunchKernelGGL(softmax_wta_kernel<DD>, grid, dim3(256), 0, st, logits, hyp, HW, clamp_lo, clamp_hi,    \
                       prob, depth, depth_raw, conf);                                                          \
    break;
  switch (ndepth) {
    TMVS_SM_CASE(4)
    TMVS_SM_CASE(8)
    TMVS_SM_CASE(16)
    TMVS_SM_CASE(24)
    TMVS_SM_CASE(32)
    TMVS_SM_CASE(48)
    TMVS_SM_CASE(64)
    default:
      return TMVS_ERR_SHAPE;
  }
#undef TMVS_SM_CASE
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
