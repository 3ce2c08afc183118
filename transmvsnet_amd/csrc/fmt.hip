// Feature Matching Transformer (models/FMT.py) linear attention on MI355X.
//
// d_model = 32, 8 heads x 4 dims, tokens [nv][L][32] (channels-last stage-1 map). One
// EncoderLayer (FMT.py:96-111) is two launches plus a tiny combine:
//   fmt_kv_partial  : per source token K = elu(Wk x + bk) + 1, V = Wv x + bv, accumulate
//                     KV[h][m][d] = Σ_s K[h,d] V[h,m] and Ksum[h][d] = Σ_s K[h,d]  (FMT.py:23-32)
//                     per workgroup -> partial slab [nv][nblk][160]
//   fmt_kv_combine  : sums the slabs in a fixed order (bitwise reproducible; no atomics)
//   fmt_apply       : per query token: Q = elu(Wq x + bq) + 1, Z = 1/(Q·Ksum + 1e-6),
//                     msg = (Q·KV) Z, x = LN1(x + Wo msg + bo), x = LN2(x + W2 relu(W1 x + b1) + b2)
// Cross layers read the reference view's (KV, Ksum) for every source view (kv stride 0):
// the reference recomputes the identical values per view (FMT.py:170-176).
// The 8.5 KMAC/token of weights are wave-uniform: the compiler streams them through the
// scalar cache (s_load) as SGPR operands of v_fma_f32, so the VALU runs at full rate.
#include "common.h"

namespace tmvs {

constexpr int kD = 32;
constexpr int kKV = TMVS_KV_NFLOATS;
constexpr int kKvBlock = 256;
constexpr int kKvTokensPerThread = 2;

__device__ __forceinline__ float elu1(float x) { return (x > 0.f ? x : expm1f(x)) + 1.f; }

__device__ __forceinline__ void load_token(const float* __restrict__ p, float (&x)[kD]) {
#pragma unroll
  for (int c4 = 0; c4 < kD / 4; ++c4) {
    const float4 t = *reinterpret_cast<const float4*>(p + c4 * 4);
    x[c4 * 4 + 0] = t.x;
    x[c4 * 4 + 1] = t.y;
    x[c4 * 4 + 2] = t.z;
    x[c4 * 4 + 3] = t.w;
  }
}

// F.linear (addmm): bias + x·W^T, the dot product as an FMA chain over the input index
template <int OUT, int IN>
__device__ __forceinline__ void linear(const float* __restrict__ W, const float* __restrict__ b, const float* x,
                                       float* y) {
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < IN; ++i) acc = fmaf(W[o * IN + i], x[i], acc);
    y[o] = acc + b[o];
  }
}

__device__ __forceinline__ void layer_norm(float (&x)[kD], const float* __restrict__ g, const float* __restrict__ b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kD; ++i) s += x[i];
  const float mean = s / (float)kD;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < kD; ++i) {
    const float d = x[i] - mean;
    v = fmaf(d, d, v);
  }
  const float rstd = 1.f / sqrtf(v / (float)kD + 1e-5f);
  const float bias = -rstd * mean;
#pragma unroll
  for (int i = 0; i < kD; ++i) x[i] = fmaf(fmaf(x[i], rstd, bias), g[i], b[i]);
}

__global__ __launch_bounds__(256) void fmt_embed_kernel(const float* __restrict__ feat, long view_stride,
                                                        const float* __restrict__ pe, int pe_h, int pe_w, int H, int W,
                                                        float* __restrict__ tokens) {
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  const int v = blockIdx.y;
  const int y = p / W, x = p - y * W;
  const float* f = feat + (size_t)v * view_stride + p;
  float t[kD];
#pragma unroll
  for (int c = 0; c < kD; ++c) t[c] = f[(size_t)c * HW] + pe[((size_t)c * pe_h + y) * pe_w + x];
  float4* o = reinterpret_cast<float4*>(tokens + ((size_t)v * HW + p) * kD);
#pragma unroll
  for (int c4 = 0; c4 < kD / 4; ++c4) o[c4] = make_float4(t[4 * c4], t[4 * c4 + 1], t[4 * c4 + 2], t[4 * c4 + 3]);
}

// One token per thread computes (K, V); the block then contracts its 256 tokens out of LDS,
// thread i < 160 owning one (h, m, d) entry of KV (or one Ksum entry), summing in token order.
__global__ __launch_bounds__(kKvBlock) void fmt_kv_partial_kernel(const float* __restrict__ src, int S,
                                                                   const float* __restrict__ w,
                                                                   float* __restrict__ partial) {
  __shared__ float sk[kD][kKvBlock + 1];
  __shared__ float sv[kD][kKvBlock + 1];
  const int v = blockIdx.y;
  const float* srcv = src + (size_t)v * S * kD;
  const int i = threadIdx.x;
  // entry owned by thread i: KV[h][m][d] for i < 128, Ksum[h][d] for 128 <= i < 160
  const int kidx = i < 128 ? (i >> 4) * 4 + (i & 3) : i - 128;
  const int vidx = i < 128 ? (i >> 4) * 4 + ((i >> 2) & 3) : 0;
  float acc = 0.f;
  const int base = blockIdx.x * kKvBlock * kKvTokensPerThread;
  for (int it = 0; it < kKvTokensPerThread; ++it) {
    const int t0 = base + it * kKvBlock;
    if (t0 >= S) break;  // block-uniform
    const int s = t0 + threadIdx.x;
    if (s < S) {
      float x[kD], k[kD], val[kD];
      load_token(srcv + (size_t)s * kD, x);
      linear<kD, kD>(w + TMVS_ENC_WK, w + TMVS_ENC_BK, x, k);
      linear<kD, kD>(w + TMVS_ENC_WV, w + TMVS_ENC_BV, x, val);
#pragma unroll
      for (int c = 0; c < kD; ++c) {
        sk[c][threadIdx.x] = elu1(k[c]);
        sv[c][threadIdx.x] = val[c];
      }
    }
    __syncthreads();
    const int nt = min(kKvBlock, S - t0);
    if (i < 128) {
      for (int t = 0; t < nt; ++t) acc = fmaf(sk[kidx][t], sv[vidx][t], acc);
    } else if (i < kKV) {
      for (int t = 0; t < nt; ++t) acc += sk[kidx][t];
    }
    __syncthreads();
  }
  if (i < kKV) partial[((size_t)v * gridDim.x + blockIdx.x) * kKV + i] = acc;
}

__global__ void fmt_kv_combine_kernel(const float* __restrict__ partial, int nblk, float* __restrict__ kv) {
  const int v = blockIdx.x;
  const int i = threadIdx.x;
  if (i >= kKV) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += partial[((size_t)v * nblk + b) * kKV + i];
  kv[(size_t)v * kKV + i] = s;
}

__global__ __launch_bounds__(256) void fmt_apply_kernel(float* __restrict__ x, int L, const float* __restrict__ kvg,
                                                        long kv_stride, const float* __restrict__ w) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= L) return;
  const int v = blockIdx.y;
  const float* kv = kvg + (size_t)v * kv_stride;
  float* xp = x + ((size_t)v * L + l) * kD;
  float xs[kD];
  load_token(xp, xs);
  float msg[kD];
  {
    float q[kD];
    linear<kD, kD>(w + TMVS_ENC_WQ, w + TMVS_ENC_BQ, xs, q);
#pragma unroll
    for (int i = 0; i < kD; ++i) q[i] = elu1(q[i]);
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      float den = 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) den = fmaf(q[h * 4 + d], kv[128 + h * 4 + d], den);
      const float z = 1.f / (den + 1e-6f);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float num = 0.f;
#pragma unroll
        for (int d = 0; d < 4; ++d) num = fmaf(q[h * 4 + d], kv[h * 16 + m * 4 + d], num);
        msg[h * 4 + m] = num * z;
      }
    }
  }
  {
    float a[kD];
    linear<kD, kD>(w + TMVS_ENC_WO, w + TMVS_ENC_BO, msg, a);
#pragma unroll
    for (int i = 0; i < kD; ++i) xs[i] = xs[i] + a[i];
  }
  layer_norm(xs, w + TMVS_ENC_LN1G, w + TMVS_ENC_LN1B);
  {
    float hdn[2 * kD];
    linear<2 * kD, kD>(w + TMVS_ENC_W1, w + TMVS_ENC_B1, xs, hdn);
#pragma unroll
    for (int i = 0; i < 2 * kD; ++i) hdn[i] = relu(hdn[i]);
    float f[kD];
    linear<kD, 2 * kD>(w + TMVS_ENC_W2, w + TMVS_ENC_B2, hdn, f);
#pragma unroll
    for (int i = 0; i < kD; ++i) xs[i] = xs[i] + f[i];
  }
  layer_norm(xs, w + TMVS_ENC_LN2G, w + TMVS_ENC_LN2B);
  float4* o = reinterpret_cast<float4*>(xp);
#pragma unroll
  for (int c4 = 0; c4 < kD / 4; ++c4) o[c4] = make_float4(xs[4 * c4], xs[4 * c4 + 1], xs[4 * c4 + 2], xs[4 * c4 + 3]);
}

static int kv_nblk(int S) { return (S + kKvBlock * kKvTokensPerThread - 1) / (kKvBlock * kKvTokensPerThread); }

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_fmt_embed(const float* feat, long feat_view_stride, const float* pe, int pe_h, int pe_w, int nv,
                              int channels, int height, int width, float* tokens, void* stream) {
  if (!feat || !pe || !tokens || nv <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (channels != kD || height > pe_h || width > pe_w) return TMVS_ERR_SHAPE;
  const int HW = height * width;
  hipLaunchKernelGGL(fmt_embed_kernel, dim3((HW + 255) / 256, nv), dim3(256), 0, (hipStream_t)stream, feat,
                     feat_view_stride, pe, pe_h, pe_w, height, width, tokens);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" size_t tmvs_fmt_kv_workspace(int nv, int s_tokens) {
  return (size_t)nv * kv_nblk(s_tokens) * kKV * sizeof(float);
}

extern "C" int tmvs_fmt_kv(const float* source, int nv, int s_tokens, const float* enc_w, void* workspace,
                           size_t workspace_bytes, float* kv, void* stream) {
  if (!source || !enc_w || !workspace || !kv || nv <= 0 || s_tokens <= 0) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_fmt_kv_workspace(nv, s_tokens)) return TMVS_ERR_ARG;
  const int nblk = kv_nblk(s_tokens);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fmt_kv_partial_kernel, dim3(nblk, nv), dim3(kKvBlock), 0, st, source, s_tokens, enc_w,
                     (float*)workspace);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(fmt_kv_combine_kernel, dim3(nv), dim3(kKV), 0, st, (const float*)workspace, nblk, kv);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_fmt_apply(float* x, int nv, int l_tokens, const float* kv, long kv_view_stride,
                              const float* enc_w, void* stream) {
  if (!x || !kv || !enc_w || nv <= 0 || l_tokens <= 0 || kv_view_stride < 0) return TMVS_ERR_ARG;
  hipLaunchKernelGGL(fmt_apply_kernel, dim3((l_tokens + 255) / 256, nv), dim3(256), 0, (hipStream_t)stream, x,
                     l_tokens, kv, kv_view_stride, enc_w);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
