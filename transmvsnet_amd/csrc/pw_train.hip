// DepthNet view aggregation and the stage-1 PixelwiseNet in train mode, forward and backward
// (SURVEY.md 8f rank 2, config C5): models/TransMVSNet.py:10-30 (PixelwiseNet: 1x1x1 Conv3d 1->16
// + BatchNorm3d + ReLU, 16->8 + BatchNorm3d + ReLU, 8->1 + bias, sigmoid, max over D) and :71-93
// (sim = sum_v w_v sim_v / (1e-5 + sum_v w_v), views in order).
//
// One sample; per-view similarity volumes sims [V][D][P] (P = H*W). PixelwiseNet runs per view
// with BatchNorm batch statistics over that view's D*P elements (the reference calls it per view).
// Parameters (device, fp32, "pwp"): w0[16] g0[16] b0[16] W1[8][16] g1[8] b1[8] w2[8] b2 (201).
// Per-view statistics ("st", fp32): mean0[16] var0[16] mean1[8] var1[8] (biased variances).
// Every reduction is fp64 block partials + a fixed-order combine (deterministic, no atomics);
// the backward recomputes the forward chain per element instead of storing 24 channels per voxel.
#include "common.h"

namespace tmvs {

constexpr int kPwBlock = 256;
constexpr int PW_W0 = 0, PW_G0 = 16, PW_B0 = 32, PW_W1 = 48, PW_G1 = 176, PW_B1 = 184, PW_W2 = 192, PW_B2 = 200;
constexpr int ST_M0 = 0, ST_V0 = 16, ST_M1 = 32, ST_V1 = 40;
constexpr float kPwEps = 1e-5f;

struct PwChain {  // one element's forward chain
  float y0[16], pre1[8], y1[8], xhat1[8];
  float o, sg;
};

__device__ __forceinline__ void bn_coef(float mean, float var, float g, float b, float& a, float& sh, float& rstd) {
  rstd = 1.f / sqrtf(var + kPwEps);
  a = rstd * g;
  sh = fmaf(-mean, a, b);
}

// z0 -> y0 (and, if pre0 given, the pre-ReLU values), z1 = W1 y0
__device__ __forceinline__ void pw_layer0(float s, const float* __restrict__ p, const float* __restrict__ st,
                                          float (&y0)[16], float (&z1)[8], float* pre0 = nullptr) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    float a, sh, rstd;
    bn_coef(st[ST_M0 + j], st[ST_V0 + j], p[PW_G0 + j], p[PW_B0 + j], a, sh, rstd);
    const float pre = fmaf(p[PW_W0 + j] * s, a, sh);
    if (pre0) pre0[j] = pre;
    y0[j] = relu(pre);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = fmaf(p[PW_W1 + k * 16 + j], y0[j], acc);
    z1[k] = acc;
  }
}

__device__ __forceinline__ void pw_chain(float s, const float* __restrict__ p, const float* __restrict__ st,
                                         PwChain& c) {
  float z1[8];
  pw_layer0(s, p, st, c.y0, z1);
  float o = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a, sh, rstd;
    bn_coef(st[ST_M1 + k], st[ST_V1 + k], p[PW_G1 + k], p[PW_B1 + k], a, sh, rstd);
    c.pre1[k] = fmaf(z1[k], a, sh);
    c.xhat1[k] = (z1[k] - st[ST_M1 + k]) * rstd;
    c.y1[k] = relu(c.pre1[k]);
    o = fmaf(p[PW_W2 + k], c.y1[k], o);
  }
  c.o = o + p[PW_B2];
  c.sg = 1.f / (1.f + expf(-c.o));
}

// (TMVS_PW_DPP: the pass-2 wave sums by common.h's DPP butterfly, r15a)
#ifndef TMVS_PW_DPP
#define TMVS_PW_DPP 1
#endif
// fp64 block reduction of NV values per thread into partial[blockIdx.x][NV]: a fixed xor butterfly
// inside each wave, then the 4 wave sums in a fixed order (deterministic). The DPP moves for the 160-value
// pass-2 and the 16-value pass-3 / z1 reductions: with 25 values (pass 1) they raised it to 178 VGPRs
template <typename T, int NV>
__device__ __forceinline__ void block_reduce_store(const T (&v)[NV], double* __restrict__ partial) {
  constexpr bool kDpp = TMVS_PW_DPP && (NV >= 64 || NV == 16);
  __shared__ double red[kPwBlock / 64][NV];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double x = (double)v[i];
    if constexpr (kDpp) {
      x = wave_xor_sum_dpp(x);
    } else {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    }
    if (lane == 0) red[wv][i] = x;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += kPwBlock)
    partial[(size_t)blockIdx.x * NV + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

__global__ __launch_bounds__(kPwBlock) void pw_sum_partials_kernel(const double* __restrict__ partial, int nblk, int K,
                                                                   double* __restrict__ out) {
  __shared__ double red[kPwBlock];
  double a = 0.0;
  a = strided_sum(partial + blockIdx.x, threadIdx.x, nblk, kPwBlock, (size_t)K, a);
  red[threadIdx.x] = a;
  __syncthreads();
  for (int st = kPwBlock / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------- forward
// stats of s (sum, sum^2) -> layer-0 statistics mean0 = w0*mean_s, var0 = w0^2 * var_s
__global__ __launch_bounds__(kPwBlock) void pw_s_partial_kernel(const float* __restrict__ s, long n, long vpb,
                                                                double* __restrict__ partial) {
  const long i0 = (long)blockIdx.x * vpb, i1 = i0 + vpb < n ? i0 + vpb : n;
  double v[2] = {0.0, 0.0};
  for (long i = i0 + threadIdx.x; i < i1; i += kPwBlock) {
    const double x = (double)s[i];
    v[0] += x;
    v[1] += x * x;
  }
  block_reduce_store(v, partial);
}

__global__ void pw_stats0_kernel(const double* __restrict__ sums, long n, const float* __restrict__ p,
                                 float* __restrict__ st) {
  const int j = threadIdx.x;
  if (j >= 16) return;
  const double m = sums[0] / (double)n;
  double var = sums[1] / (double)n - m * m;
  var = var > 0.0 ? var : 0.0;
  const double w = (double)p[PW_W0 + j];
  st[ST_M0 + j] = (float)(w * m);
  st[ST_V0 + j] = (float)(w * w * var);
}

__global__ __launch_bounds__(kPwBlock) void pw_z1_partial_kernel(const float* __restrict__ s, long n, long vpb,
                                                                 const float* __restrict__ p,
                                                                 const float* __restrict__ st,
                                                                 double* __restrict__ partial) {
  const long i0 = (long)blockIdx.x * vpb, i1 = i0 + vpb < n ? i0 + vpb : n;
  double v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = 0.0;
  for (long i = i0 + threadIdx.x; i < i1; i += kPwBlock) {
    float y0[16], z1[8];
    pw_layer0(s[i], p, st, y0, z1);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] += (double)z1[k];
      v[8 + k] += (double)z1[k] * (double)z1[k];
    }
  }
  block_reduce_store(v, partial);
}

__global__ void pw_stats1_kernel(const double* __restrict__ sums, long n, float* __restrict__ st) {
  const int k = threadIdx.x;
  if (k >= 8) return;
  const double m = sums[k] / (double)n;
  const double var = sums[8 + k] / (double)n - m * m;
  st[ST_M1 + k] = (float)m;
  st[ST_V1 + k] = (float)(var > 0.0 ? var : 0.0);
}

// view weight w[p] = max_d sigmoid(PixelwiseNet(s[d][p])) and its (first) argmax
__global__ __launch_bounds__(kPwBlock) void pw_weight_kernel(const float* __restrict__ s, int D, int P,
                                                             const float* __restrict__ p, const float* __restrict__ st,
                                                             float* __restrict__ w, int* __restrict__ dstar) {
  const int q = blockIdx.x * kPwBlock + threadIdx.x;
  if (q >= P) return;
  float best = 0.f;
  int bi = 0;
  for (int d = 0; d < D; ++d) {
    PwChain c;
    pw_chain(s[(size_t)d * P + q], p, st, c);
    if (d == 0 || c.sg > best) {
      best = c.sg;
      bi = d;
    }
  }
  w[q] = best;
  dstar[q] = bi;
}

// sim[d][p] = (sum_v sims[v][d][p] * w_v) / (1e-5 + sum_v w_v), views in order; w_v read at
// (y >> shift, x >> shift) of a [V][H>>shift][W>>shift] map (nearest x2^shift up-sampling)
__global__ __launch_bounds__(kPwBlock) void aggregate_train_kernel(const float* __restrict__ sims,
                                                                   const float* __restrict__ w, int V, int D, int H,
                                                                   int W, int shift, float* __restrict__ sim,
                                                                   float* __restrict__ wsum) {
  const int P = H * W;
  const int q = blockIdx.x * kPwBlock + threadIdx.x;
  if (q >= P) return;
  const int y = q / W, x = q - y * W;
  const int Ws = W >> shift, Ps = (H >> shift) * Ws;
  const int qs = (y >> shift) * Ws + (x >> shift);
  float ws = 1e-5f;
  for (int v = 0; v < V; ++v) ws = ws + w[(size_t)v * Ps + qs];
  wsum[q] = ws;
  for (int d = 0; d < D; ++d) {
    float acc = 0.f;
    for (int v = 0; v < V; ++v) acc = acc + sims[((size_t)v * D + d) * P + q] * w[(size_t)v * Ps + qs];
    sim[(size_t)d * P + q] = acc / ws;
  }
}

// ---------------------------------------------------------------- backward
// dsims[v][d][p] = dsim[d][p] / wsum[p] * w_v[p]; dw_v[p] = sum_d dsim/wsum * (sims_v - sim)  (dw optional)
__global__ __launch_bounds__(kPwBlock) void aggregate_backward_kernel(
    const float* __restrict__ dsim, const float* __restrict__ sims, const float* __restrict__ sim,
    const float* __restrict__ wsum, const float* __restrict__ w, int V, int D, int H, int W, int shift,
    float* __restrict__ dsims, float* __restrict__ dw) {
  const int P = H * W;
  const int q = blockIdx.x * kPwBlock + threadIdx.x;
  if (q >= P) return;
  const int y = q / W, x = q - y * W;
  const int Ws = W >> shift, Ps = (H >> shift) * Ws;
  const int qs = (y >> shift) * Ws + (x >> shift);
  const float ws = wsum[q];
  for (int v = 0; v < V; ++v) {
    const float wv = w[(size_t)v * Ps + qs];
    float acc = 0.f;
    for (int d = 0; d < D; ++d) {
      const float g = dsim[(size_t)d * P + q] / ws;
      const size_t e = ((size_t)v * D + d) * P + q;
      dsims[e] = g * wv;
      if (dw) acc = fmaf(g, sims[e] - sim[(size_t)d * P + q], acc);
    }
    if (dw) dw[(size_t)v * P + q] = acc;
  }
}

// pass 1 (per pixel, at the argmax plane): sums of g1 (8), g1*xhat1 (8), g_o*y1 (8), g_o (1)
__global__ __launch_bounds__(kPwBlock) void pw_bwd1_kernel(const float* __restrict__ s, int D, int P,
                                                           const float* __restrict__ p, const float* __restrict__ st,
                                                           const float* __restrict__ w, const int* __restrict__ dstar,
                                                           const float* __restrict__ dw, long ppb,
                                                           double* __restrict__ partial) {
  double v[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) v[i] = 0.0;
  const long q0 = (long)blockIdx.x * ppb, q1 = q0 + ppb < P ? q0 + ppb : P;
  for (long q = q0 + threadIdx.x; q < q1; q += kPwBlock) {
    PwChain c;
    pw_chain(s[(size_t)dstar[q] * P + q], p, st, c);
    const float sg = w[q];
    const float go = dw[q] * ((1.f - sg) * sg);  // sigmoid backward at the argmax
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float g1 = c.pre1[k] > 0.f ? go * p[PW_W2 + k] : 0.f;
      v[k] += (double)g1;
      v[8 + k] += (double)g1 * (double)c.xhat1[k];
      v[16 + k] += (double)go * (double)c.y1[k];
    }
    v[24] += (double)go;
  }
  block_reduce_store(v, partial);
}

// the layer-1 gradient of one element: dz1 = a1 (g1 - S1a/N - xhat1 S1b/N), g1 nonzero at the argmax only
__device__ __forceinline__ void pw_dz1(float s, int d, int ds, float go, const float* __restrict__ p,
                                       const float* __restrict__ st, const double* __restrict__ s1, double inv_n,
                                       float (&y0)[16], float (&pre0)[16], float (&dz1)[8]) {
  float z1[8];
  pw_layer0(s, p, st, y0, z1, pre0);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a, sh, rstd;
    bn_coef(st[ST_M1 + k], st[ST_V1 + k], p[PW_G1 + k], p[PW_B1 + k], a, sh, rstd);
    const float xhat = (z1[k] - st[ST_M1 + k]) * rstd;
    const float g1 = (d == ds && fmaf(z1[k], a, sh) > 0.f) ? go * p[PW_W2 + k] : 0.f;
    dz1[k] = a * ((g1 - (float)(s1[k] * inv_n)) - xhat * (float)(s1[8 + k] * inv_n));
  }
}

// pass 2 (per element): sums of g0 (16), g0*xhat0 (16), dz1_k * y0_j (128)
__global__ __launch_bounds__(kPwBlock) void pw_bwd2_kernel(const float* __restrict__ s, int D, int P,
                                                           const float* __restrict__ p, const float* __restrict__ st,
                                                           const float* __restrict__ w, const int* __restrict__ dstar,
                                                           const float* __restrict__ dw, const double* __restrict__ s1,
                                                           long epb, double* __restrict__ partial) {
  const long n = (long)D * P;
  const double inv_n = 1.0 / (double)n;
  float acc[160];  // g0 sums [0,16), g0*xhat0 sums [16,32), dW1 [32,160)
#pragma unroll
  for (int i = 0; i < 160; ++i) acc[i] = 0.f;
  const long e0 = (long)blockIdx.x * epb, e1 = e0 + epb < n ? e0 + epb : n;
  for (long e = e0 + threadIdx.x; e < e1; e += kPwBlock) {
    const int d = (int)(e / P), q = (int)(e - (long)d * P);
    const float sg = w[q];
    const float go = dw[q] * ((1.f - sg) * sg);
    float y0[16], pre0[16], dz1[8];
    const float sv = s[e];
    pw_dz1(sv, d, dstar[q], go, p, st, s1, inv_n, y0, pre0, dz1);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float dy0 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dy0 = fmaf(p[PW_W1 + k * 16 + j], dz1[k], dy0);
        acc[32 + k * 16 + j] = fmaf(dz1[k], y0[j], acc[32 + k * 16 + j]);
      }
      const float g0 = pre0[j] > 0.f ? dy0 : 0.f;
      float a, sh, rstd;
      bn_coef(st[ST_M0 + j], st[ST_V0 + j], p[PW_G0 + j], p[PW_B0 + j], a, sh, rstd);
      const float xhat0 = (p[PW_W0 + j] * sv - st[ST_M0 + j]) * rstd;
      acc[j] += g0;
      acc[16 + j] = fmaf(g0, xhat0, acc[16 + j]);
    }
  }
  block_reduce_store(acc, partial);
}

// pass 3 (per element): dz0 = a0 (g0 - S0a/N - xhat0 S0b/N); dsims += sum_j w0_j dz0_j; sums of dz0*s (16)
__global__ __launch_bounds__(kPwBlock) void pw_bwd3_kernel(const float* __restrict__ s, int D, int P,
                                                           const float* __restrict__ p, const float* __restrict__ st,
                                                           const float* __restrict__ w, const int* __restrict__ dstar,
                                                           const float* __restrict__ dw, const double* __restrict__ s1,
                                                           const double* __restrict__ s2, long epb,
                                                           float* __restrict__ dsims, double* __restrict__ partial) {
  const long n = (long)D * P;
  const double inv_n = 1.0 / (double)n;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = 0.0;
  const long e0 = (long)blockIdx.x * epb, e1 = e0 + epb < n ? e0 + epb : n;
  for (long e = e0 + threadIdx.x; e < e1; e += kPwBlock) {
    const int d = (int)(e / P), q = (int)(e - (long)d * P);
    const float sg = w[q];
    const float go = dw[q] * ((1.f - sg) * sg);
    float y0[16], pre0[16], dz1[8];
    const float sv = s[e];
    pw_dz1(sv, d, dstar[q], go, p, st, s1, inv_n, y0, pre0, dz1);
    float ds = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float dy0 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) dy0 = fmaf(p[PW_W1 + k * 16 + j], dz1[k], dy0);
      const float g0 = pre0[j] > 0.f ? dy0 : 0.f;
      float a, sh, rstd;
      bn_coef(st[ST_M0 + j], st[ST_V0 + j], p[PW_G0 + j], p[PW_B0 + j], a, sh, rstd);
      const float xhat0 = (p[PW_W0 + j] * sv - st[ST_M0 + j]) * rstd;
      const float dz0 = a * ((g0 - (float)(s2[j] * inv_n)) - xhat0 * (float)(s2[16 + j] * inv_n));
      ds = fmaf(p[PW_W0 + j], dz0, ds);
      v[j] += (double)dz0 * (double)sv;
    }
    dsims[e] = dsims[e] + ds;
  }
  block_reduce_store(v, partial);
}

// parameter gradients of this view, added to grad[201] (pwp layout)
__global__ void pw_grad_finalize_kernel(const double* __restrict__ s1, const double* __restrict__ s2,
                                        const double* __restrict__ s3, float* __restrict__ grad) {
  const int t = threadIdx.x;
  if (t < 16) {
    grad[PW_W0 + t] += (float)s3[t];
    grad[PW_G0 + t] += (float)s2[16 + t];
    grad[PW_B0 + t] += (float)s2[t];
  }
  if (t < 128) grad[PW_W1 + t] += (float)s2[32 + t];
  if (t < 8) {
    grad[PW_G1 + t] += (float)s1[8 + t];
    grad[PW_B1 + t] += (float)s1[t];
    grad[PW_W2 + t] += (float)s1[16 + t];
  }
  if (t == 0) grad[PW_B2] += (float)s1[24];
}

static long pw_chunk(long n, long maxblk) {
  long c = 1024;
  while ((n + c - 1) / c > maxblk) c *= 2;
  return c;
}

}  // namespace tmvs

using namespace tmvs;

// workspace: partials (<= 1024 blocks x 160 doubles) + sums (2 + 16 + 25 + 160 + 16 doubles)
extern "C" size_t tmvs_pixelwise_train_workspace(void) { return (1024 * 160 + 256) * sizeof(double) + 256; }

extern "C" int tmvs_pixelwise_train_forward(const float* sims, int n_views, int ndepth, int height, int width,
                                            const float* pwp, void* workspace, size_t workspace_bytes, float* stats,
                                            float* view_w, int* dstar, void* stream) {
  if (!sims || !pwp || !workspace || !stats || !view_w || !dstar || n_views <= 0 || ndepth <= 0 || height <= 0 ||
      width <= 0)
    return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_pixelwise_train_workspace()) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int P = height * width;
  const long n = (long)ndepth * P;
  double* part = (double*)workspace;
  double* sums = part + 1024 * 160;
  const long c = pw_chunk(n, 1024);
  const int nb = (int)((n + c - 1) / c);
  for (int v = 0; v < n_views; ++v) {
    const float* s = sims + (size_t)v * n;
    float* sv = stats + (size_t)v * 48;
    hipLaunchKernelGGL(pw_s_partial_kernel, dim3(nb), dim3(kPwBlock), 0, st, s, n, c, part);
    hipLaunchKernelGGL(pw_sum_partials_kernel, dim3(2), dim3(kPwBlock), 0, st, (const double*)part, nb, 2, sums);
    hipLaunchKernelGGL(pw_stats0_kernel, dim3(1), dim3(64), 0, st, (const double*)sums, n, pwp, sv);
    hipLaunchKernelGGL(pw_z1_partial_kernel, dim3(nb), dim3(kPwBlock), 0, st, s, n, c, pwp, (const float*)sv, part);
    hipLaunchKernelGGL(pw_sum_partials_kernel, dim3(16), dim3(kPwBlock), 0, st, (const double*)part, nb, 16, sums);
    hipLaunchKernelGGL(pw_stats1_kernel, dim3(1), dim3(64), 0, st, (const double*)sums, n, sv);
    hipLaunchKernelGGL(pw_weight_kernel, dim3((P + kPwBlock - 1) / kPwBlock), dim3(kPwBlock), 0, st, s, ndepth, P,
                       pwp, (const float*)sv, view_w + (size_t)v * P, dstar + (size_t)v * P);
    TMVS_CHECK_LAUNCH();
  }
  return TMVS_OK;
}

extern "C" int tmvs_aggregate_train(const float* sims, const float* view_w, int n_views, int ndepth, int height,
                                    int width, int vw_shift, float* sim, float* wsum, void* stream) {
  if (!sims || !view_w || !sim || !wsum || n_views <= 0 || ndepth <= 0 || height <= 0 || width <= 0 || vw_shift < 0)
    return TMVS_ERR_ARG;
  const int P = height * width;
  hipLaunchKernelGGL(aggregate_train_kernel, dim3((P + kPwBlock - 1) / kPwBlock), dim3(kPwBlock), 0,
                     (hipStream_t)stream, sims, view_w, n_views, ndepth, height, width, vw_shift, sim, wsum);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_aggregate_train_backward(const float* dsim, const float* sims, const float* sim, const float* wsum,
                                             const float* view_w, int n_views, int ndepth, int height, int width,
                                             int vw_shift, float* dsims, float* dview_w, void* stream) {
  if (!dsim || !sims || !sim || !wsum || !view_w || !dsims || n_views <= 0 || ndepth <= 0 || height <= 0 ||
      width <= 0 || vw_shift < 0)
    return TMVS_ERR_ARG;
  const int P = height * width;
  hipLaunchKernelGGL(aggregate_backward_kernel, dim3((P + kPwBlock - 1) / kPwBlock), dim3(kPwBlock), 0,
                     (hipStream_t)stream, dsim, sims, sim, wsum, view_w, n_views, ndepth, height, width, vw_shift,
                     dsims, dview_w);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_pixelwise_train_backward(const float* sims, int n_views, int ndepth, int height, int width,
                                             const float* pwp, const float* stats, const float* view_w,
                                             const int* dstar, const float* dview_w, void* workspace,
                                             size_t workspace_bytes, float* dsims, float* dpwp, void* stream) {
  if (!sims || !pwp || !stats || !view_w || !dstar || !dview_w || !workspace || !dsims || !dpwp || n_views <= 0 ||
      ndepth <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_pixelwise_train_workspace()) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int P = height * width;
  const long n = (long)ndepth * P;
  double* part = (double*)workspace;
  double* s1 = part + 1024 * 160;
  double* s2 = s1 + 32;
  double* s3 = s2 + 160;
  const long cp = pw_chunk(P, 1024), ce = pw_chunk(n, 1024);
  const int nbp = (int)((P + cp - 1) / cp), nbe = (int)((n + ce - 1) / ce);
  for (int v = 0; v < n_views; ++v) {
    const float* s = sims + (size_t)v * n;
    const float* sv = stats + (size_t)v * 48;
    const float* w = view_w + (size_t)v * P;
    const int* ds = dstar + (size_t)v * P;
    const float* dw = dview_w + (size_t)v * P;
    hipLaunchKernelGGL(pw_bwd1_kernel, dim3(nbp), dim3(kPwBlock), 0, st, s, ndepth, P, pwp, sv, w, ds, dw, cp, part);
    hipLaunchKernelGGL(pw_sum_partials_kernel, dim3(25), dim3(kPwBlock), 0, st, (const double*)part, nbp, 25, s1);
    hipLaunchKernelGGL(pw_bwd2_kernel, dim3(nbe), dim3(kPwBlock), 0, st, s, ndepth, P, pwp, sv, w, ds, dw,
                       (const double*)s1, ce, part);
    hipLaunchKernelGGL(pw_sum_partials_kernel, dim3(160), dim3(kPwBlock), 0, st, (const double*)part, nbe, 160, s2);
    hipLaunchKernelGGL(pw_bwd3_kernel, dim3(nbe), dim3(kPwBlock), 0, st, s, ndepth, P, pwp, sv, w, ds, dw,
                       (const double*)s1, (const double*)s2, ce, dsims + (size_t)v * n, part);
    hipLaunchKernelGGL(pw_sum_partials_kernel, dim3(16), dim3(kPwBlock), 0, st, (const double*)part, nbe, 16, s3);
    hipLaunchKernelGGL(pw_grad_finalize_kernel, dim3(1), dim3(128), 0, st, (const double*)s1, (const double*)s2,
                       (const double*)s3, dpwp);
    TMVS_CHECK_LAUNCH();
  }
  return TMVS_OK;
}
