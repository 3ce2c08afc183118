// FMT backward for training: the pieces of EncoderLayer.forward
// (models/FMT.py:96-111; AttentionLayer :56-75; LinearAttention :22-37) that autograd needs, as
// token-wise kernels over [T][C] token matrices (C = 32, hidden 64, 8 heads x 4):
//   tmvs_token_linear      y = x W^T (+ b) or y = x W (the data gradient), optionally accumulated (fp32 MFMA)
//   tmvs_token_wgrad       dW = dy^T x and db = column sums of dy (fp64 block partials, fixed combine)
//   tmvs_layer_norm_fwd    LayerNorm(32) forward (the backward recomputes its statistics)
//   tmvs_layer_norm_bwd    dx, and dgamma / dbeta (deterministic reductions)
//   tmvs_linattn_fwd       msg = (Q KV) / (Q Ksum + 1e-6) per head, Q = elu(q) + 1
//   tmvs_linattn_bwd_q     dq (through the elu), and dKV / dKsum reduced over the queries of each
//                          K/V group (per view for self layers, all views for cross layers)
//   tmvs_linattn_bwd_kv    dk (through the elu), dv of the source tokens
// KV layout as the forward (csrc/fmt.hip): kv[h*16 + m*4 + d] = sum_s K[s,h,d] V[s,h,m], Ksum at
// 128 + h*4 + d. fp32 per token, fp64 in every cross-token reduction, no atomics.
#include "common.h"

namespace tmvs {

constexpr int kTB = 256;
constexpr float kLnEps = 1e-5f;
constexpr float kAttnEps = 1e-6f;

__device__ __forceinline__ float elu1f(float x) { return (x > 0.f ? x : expm1f(x)) + 1.f; }
__device__ __forceinline__ float elu1_grad(float x) { return x > 0.f ? 1.f : expf(x); }

// y[t][o] = sum_i W[o][i] x[t][i] + b[o] for a torch Linear weight W [OUT][IN]; TRANS: y[t][o] = sum_i W[i][o] x[t][i]
// for W [IN][OUT] (the data gradient dx = dy W of a Linear with weight W); relu_of masks y where relu_of <= 0;
// accumulate adds into y. On fp32 MFMA (v_mfma_f32_16x16x4f32): a wave computes 16 tokens x 16 outputs
// per block of OUT: A (16 x 4) = weights (lane l: output l & 15, k-group l >> 4), B (4 x 16) = tokens (lane l:
// token l & 15, k-group l >> 4), D lane l = outputs 4 (l >> 4) .. +3 of token l & 15 (one float4 store).
// The contraction runs over k = 16 i + 4 kg + e: a lane loads float4 chunk (i, kg) of its token's row, and
// MFMA (i, e) takes element e of it in B and W[., 16 i + 4 kg + e] in A -- the same permutation of k in
// both operands. A fragments stay in VGPRs for the wave's tiles; bias / ReLU mask / accumulate in the epilogue.
constexpr int kLinTiles = 4;  // 16-token tiles per wave
template <int IN, int OUT, bool TRANS>
__global__ __launch_bounds__(256) void token_linear_mfma_kernel(const float* __restrict__ x, long T,
                                                                const float* __restrict__ W,
                                                                const float* __restrict__ b,
                                                                const float* __restrict__ relu_of, int accumulate,
                                                                const float* __restrict__ res, float* __restrict__ y) {
  constexpr int NI = IN / 16, NB = OUT / 16;
  const int lane = threadIdx.x & 63, kg = lane >> 4, col = lane & 15;
  float afr[NB][NI][4];
#pragma unroll
  for (int ob = 0; ob < NB; ++ob)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = ob * 16 + col, k = 16 * i + 4 * kg + e;
        afr[ob][i][e] = TRANS ? W[k * OUT + o] : W[o * IN + k];
      }
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
#pragma unroll 1
  for (int it = 0; it < kLinTiles; ++it) {
    const long t0 = (wave * kLinTiles + it) * 16;
    if (t0 >= T) break;  // wave-uniform
    const long t = t0 + col;
    const long tc = t < T ? t : T - 1;
    float4 xb[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) xb[i] = *reinterpret_cast<const float4*>(x + tc * IN + 16 * i + 4 * kg);
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) {
      floatx4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[ob][i][0], xb[i].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[ob][i][1], xb[i].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[ob][i][2], xb[i].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[ob][i][3], xb[i].w, acc, 0, 0, 0);
      }
      // D: lane holds outputs ob*16 + 4 kg + r of token t0 + col
      const int o0 = ob * 16 + 4 * kg;
      float4 v = make_float4(acc[0], acc[1], acc[2], acc[3]);
      if (b) {
        v.x += b[o0];
        v.y += b[o0 + 1];
        v.z += b[o0 + 2];
        v.w += b[o0 + 3];
      }
      if (t < T) {
        if (relu_of) {
          const float4 m = *reinterpret_cast<const float4*>(relu_of + t * OUT + o0);
          v.x = m.x > 0.f ? v.x : 0.f;
          v.y = m.y > 0.f ? v.y : 0.f;
          v.z = m.z > 0.f ? v.z : 0.f;
          v.w = m.w > 0.f ? v.w : 0.f;
        }
        if (accumulate || res) {  // y += v, or y = res + v (the same addition without a copy of res into y)
          const float4 pr = *reinterpret_cast<const float4*>((res ? res : y) + t * OUT + o0);
          v.x = pr.x + v.x;
          v.y = pr.y + v.y;
          v.z = pr.z + v.z;
          v.w = pr.w + v.w;
        }
        *reinterpret_cast<float4*>(y + t * OUT + o0) = v;
      }
    }
  }
}

// partial[blk][a][b] = sum_t dy[t][a] x[t][b] over the block's token range; partial[blk][A*B + a] = sum_t dy[t][a].
// Chunks of 64 tokens are staged in LDS; wave w takes rows w, w+4, ...; each lane owns a TA x TB output tile
// ((A/TA)(B/TB) = 64), fp32 over a chunk's 16 rows then fp64; the 4 waves combine in a fixed order in LDS.
template <int A, int B, int TA, int TB>
__global__ __launch_bounds__(kTB) void token_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          long T, long tpb, double* __restrict__ partial) {
  static_assert((A / TA) * (B / TB) == 64, "one tile per lane");
  constexpr int CH = 64, NO = A * B + A;
  __shared__ __attribute__((aligned(16))) float sd[CH][A + 4];
  __shared__ __attribute__((aligned(16))) float sx[CH][B + 4];
  __shared__ double cmb[2][NO];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ci = lane % (B / TB), ai = lane / (B / TB);
  const long t0 = (long)blockIdx.x * tpb, t1 = t0 + tpb < T ? t0 + tpb : T;
  double acc[TA][TB], accb[TA];
#pragma unroll
  for (int i = 0; i < TA; ++i) {
    accb[i] = 0.0;
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = 0.0;
  }
  for (long tb = t0; tb < t1; tb += CH) {
    __syncthreads();
    for (int i = threadIdx.x; i < CH * A / 4; i += kTB) {
      const int r = i / (A / 4), c = (i % (A / 4)) * 4;
      const long t = tb + r;
      *reinterpret_cast<float4*>(&sd[r][c]) =
          t < t1 ? *reinterpret_cast<const float4*>(dy + t * A + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = threadIdx.x; i < CH * B / 4; i += kTB) {
      const int r = i / (B / 4), c = (i % (B / 4)) * 4;
      const long t = tb + r;
      *reinterpret_cast<float4*>(&sx[r][c]) =
          t < t1 ? *reinterpret_cast<const float4*>(x + t * B + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    float s[TA][TB], sb[TA];
#pragma unroll
    for (int i = 0; i < TA; ++i) {
      sb[i] = 0.f;
#pragma unroll
      for (int j = 0; j < TB; ++j) s[i][j] = 0.f;
    }
#pragma unroll 4
    for (int r = wv; r < CH; r += 4) {
      float av[TA], bv[TB];
#pragma unroll
      for (int i = 0; i < TA; i += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&sd[r][ai * TA + i]);
        av[i] = v.x;
        av[i + 1] = v.y;
        av[i + 2] = v.z;
        av[i + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < TB; j += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&sx[r][ci * TB + j]);
        bv[j] = v.x;
        bv[j + 1] = v.y;
        bv[j + 2] = v.z;
        bv[j + 3] = v.w;
      }
#pragma unroll
      for (int i = 0; i < TA; ++i) {
        sb[i] += av[i];
#pragma unroll
        for (int j = 0; j < TB; ++j) s[i][j] = fmaf(av[i], bv[j], s[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < TA; ++i) {
      accb[i] += (double)sb[i];
#pragma unroll
      for (int j = 0; j < TB; ++j) acc[i][j] += (double)s[i][j];
    }
  }
  // fixed-order wave combine: (w0 + w2) + (w1 + w3)
  auto put = [&](double* dst) {
#pragma unroll
    for (int i = 0; i < TA; ++i) {
#pragma unroll
      for (int j = 0; j < TB; ++j) dst[(ai * TA + i) * B + ci * TB + j] = acc[i][j];
      if (ci == 0) dst[A * B + ai * TA + i] = accb[i];
    }
  };
  auto add = [&](const double* src) {
#pragma unroll
    for (int i = 0; i < TA; ++i) {
#pragma unroll
      for (int j = 0; j < TB; ++j) acc[i][j] += src[(ai * TA + i) * B + ci * TB + j];
      if (ci == 0) accb[i] += src[A * B + ai * TA + i];
    }
  };
  __syncthreads();
  if (wv >= 2) put(cmb[wv - 2]);
  __syncthreads();
  if (wv < 2) add(cmb[wv]);
  __syncthreads();
  if (wv == 1) put(cmb[0]);
  __syncthreads();
  if (wv == 0) {
    add(cmb[0]);
    put(partial + (size_t)blockIdx.x * NO);
  }
}

// out0[i] (i < n0) / out1[i - n0] = sum over the block partials: 16 interleaved chains (block j in chain
// j % 16), then the 16 chain sums in order -- a fixed order, bitwise reproducible
__global__ __launch_bounds__(kTB) void fmt_sum_partials_kernel(const double* __restrict__ partial, int nblk, long n,
                                                               long n0, float* __restrict__ out0,
                                                               float* __restrict__ out1, int accumulate) {
  __shared__ double red[16][16];
  const int g = threadIdx.x >> 4, k = threadIdx.x & 15;
  const long i = (long)blockIdx.x * 16 + k;
  double s = 0.0;
  if (i < n)
    s = strided_sum(partial + i, g, nblk, 16, (size_t)n, s);
  red[g][k] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    double t = red[0][k];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][k];
    float* o = i < n0 ? out0 + i : out1 + (i - n0);
    *o = accumulate ? *o + (float)t : (float)t;
  }
}

// LayerNorm over 32 features, the reference CPU op order: mean, biased variance, (x - mean) * rstd * g + b
__device__ __forceinline__ void ln_stats(const float (&x)[32], float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) s += x[i];
  mean = s / 32.f;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const float d = x[i] - mean;
    v = fmaf(d, d, v);
  }
  rstd = 1.f / sqrtf(v / 32.f + kLnEps);
}

__global__ __launch_bounds__(kTB) void layer_norm_fwd_kernel(const float* __restrict__ x, long T,
                                                             const float* __restrict__ g, const float* __restrict__ b,
                                                             float* __restrict__ y) {
  const long t = (long)blockIdx.x * kTB + threadIdx.x;
  if (t >= T) return;
  float v[32];
#pragma unroll
  for (int i = 0; i < 32; i += 4) {  // the token's row as 16-byte quads (the same values)
    const float4 a = *reinterpret_cast<const float4*>(x + t * 32 + i);
    v[i] = a.x;
    v[i + 1] = a.y;
    v[i + 2] = a.z;
    v[i + 3] = a.w;
  }
  float mean, rstd;
  ln_stats(v, mean, rstd);
  float o[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) o[i] = fmaf((v[i] - mean) * rstd, g[i], b[i]);
#pragma unroll
  for (int i = 0; i < 32; i += 4)
    *reinterpret_cast<float4*>(y + t * 32 + i) = make_float4(o[i], o[i + 1], o[i + 2], o[i + 3]);
}

// dx = rstd/32 * (32*gy - sum gy - xhat * sum gy*xhat), gy = dy * g; partial[blk] = {sum dy*xhat (32), sum dy (32)}
#ifndef TMVS_LN_DPP
#define TMVS_LN_DPP 1
#endif
__global__ __launch_bounds__(kTB) void layer_norm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                             long T, const float* __restrict__ g, long tpb,
                                                             float* __restrict__ dx, double* __restrict__ partial) {
  __shared__ double red[64][kTB / 64];
  const long t0 = (long)blockIdx.x * tpb, t1 = t0 + tpb < T ? t0 + tpb : T;
  float pg[32], pb[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) pg[i] = pb[i] = 0.f;
  for (long t = t0 + threadIdx.x; t < t1; t += kTB) {
    float v[32], d[32];
#pragma unroll
    for (int i = 0; i < 32; i += 4) {  // 16-byte loads of the token's rows (the same values)
      const float4 a = *reinterpret_cast<const float4*>(x + t * 32 + i);
      const float4 b = *reinterpret_cast<const float4*>(dy + t * 32 + i);
      v[i] = a.x;
      v[i + 1] = a.y;
      v[i + 2] = a.z;
      v[i + 3] = a.w;
      d[i] = b.x;
      d[i + 1] = b.y;
      d[i + 2] = b.z;
      d[i + 3] = b.w;
    }
    float mean, rstd;
    ln_stats(v, mean, rstd);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const float xh = (v[i] - mean) * rstd;
      const float gy = d[i] * g[i];
      s1 += gy;
      s2 = fmaf(gy, xh, s2);
      pg[i] = fmaf(d[i], xh, pg[i]);
      pb[i] += d[i];
    }
    float o[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const float xh = (v[i] - mean) * rstd;
      o[i] = (rstd / 32.f) * ((32.f * (d[i] * g[i]) - s1) - xh * s2);
    }
#pragma unroll
    for (int i = 0; i < 32; i += 4)
      *reinterpret_cast<float4*>(dx + t * 32 + i) = make_float4(o[i], o[i + 1], o[i + 2], o[i + 3]);
  }
  // fp64 block reduction of the 64 per-thread sums (fixed butterfly per wave, then the 4 waves in order)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    double val = (double)(i < 32 ? pg[i] : pb[i - 32]);
    if (TMVS_LN_DPP) {
      val = wave_xor_sum_dpp(val);  // the same butterfly (common.h)
    } else {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) val += __shfl_xor(val, off, 64);
    }
    if (lane == 0) red[i][wv] = val;
  }
  __syncthreads();
  if (threadIdx.x < 64)
    partial[(size_t)blockIdx.x * 64 + threadIdx.x] =
        (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// Thread layout of the three token kernels below: thread = (token slot, head) with head = threadIdx & 7, so
// a wave's 64 lanes cover 8 consecutive tokens x 8 heads and each 16-byte head quad load/store of the wave
// is one contiguous 1 KiB span (the former token-per-thread loop over heads read 128-B-strided quads).
constexpr int kTokPerBlock = kTB / 8;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// msg[t][h*4+m] = (sum_d Q[h,d] KV[h][m][d]) / (sum_d Q[h,d] Ks[h][d] + eps); tokens of group gi use kv[gi*kvs]
__global__ __launch_bounds__(kTB) void linattn_fwd_kernel(const float* __restrict__ q, long T, long tpg,
                                                          const float* __restrict__ kv, long kv_stride,
                                                          float* __restrict__ msg) {
  const int h = threadIdx.x & 7;
  const long t = (long)blockIdx.x * kTokPerBlock + (threadIdx.x >> 3);
  if (t >= T) return;
  const float* K = kv + (t / tpg) * kv_stride;
  const float4 q4 = ld4(q + t * 32 + h * 4);
  const float Q[4] = {elu1f(q4.x), elu1f(q4.y), elu1f(q4.z), elu1f(q4.w)};
  float den = 0.f;
#pragma unroll
  for (int d = 0; d < 4; ++d) den = fmaf(Q[d], K[128 + h * 4 + d], den);
  const float z = 1.f / (den + kAttnEps);
  float o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float num = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) num = fmaf(Q[d], K[h * 16 + m * 4 + d], num);
    o[m] = num * z;
  }
  *reinterpret_cast<float4*>(msg + t * 32 + h * 4) = make_float4(o[0], o[1], o[2], o[3]);
}

// query side: dq, and per block partial dKV (128) + dKs (32) -- blocks never straddle a K/V group.
// Thread (slot, head) walks the block's tokens slot, slot + 32, ... for its head (20 fp32 accumulators),
// then per head a fixed fp64 reduction: xor 8, 16, 32 within the wave, then the 4 waves in order.
__global__ __launch_bounds__(kTB) void linattn_bwd_q_kernel(const float* __restrict__ q, const float* __restrict__ dmsg,
                                                            long T, long tpg, long tpb, const float* __restrict__ kv,
                                                            long kv_stride, float* __restrict__ dq,
                                                            double* __restrict__ partial) {
  __shared__ double red[kTB / 64][160];
  const long t0 = (long)blockIdx.x * tpb, t1 = t0 + tpb < T ? t0 + tpb : T;
  const float* K = kv + (t0 / tpg) * kv_stride;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = threadIdx.x & 7;
  float kvh[16], ksh[4];
#pragma unroll
  for (int i = 0; i < 16; ++i) kvh[i] = K[h * 16 + i];
#pragma unroll
  for (int d = 0; d < 4; ++d) ksh[d] = K[128 + h * 4 + d];
  float acc[20];
#pragma unroll
  for (int i = 0; i < 20; ++i) acc[i] = 0.f;
  for (long t = t0 + (threadIdx.x >> 3); t < t1; t += kTokPerBlock) {
    const float4 q4 = ld4(q + t * 32 + h * 4), d4 = ld4(dmsg + t * 32 + h * 4);
    const float qr[4] = {q4.x, q4.y, q4.z, q4.w}, dm[4] = {d4.x, d4.y, d4.z, d4.w};
    float Q[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) Q[d] = elu1f(qr[d]);
    float den = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) den = fmaf(Q[d], ksh[d], den);
    const float z = 1.f / (den + kAttnEps);
    float dz = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float nm = 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) nm = fmaf(Q[d], kvh[m * 4 + d], nm);
      dz = fmaf(dm[m], nm, dz);
    }
    const float dden = -dz * z * z;
    float o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float dQ = dden * ksh[d];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float dn = dm[m] * z;
        dQ = fmaf(dn, kvh[m * 4 + d], dQ);
        acc[m * 4 + d] = fmaf(dn, Q[d], acc[m * 4 + d]);
      }
      acc[16 + d] = fmaf(dden, Q[d], acc[16 + d]);
      o[d] = dQ * elu1_grad(qr[d]);
    }
    *reinterpret_cast<float4*>(dq + t * 32 + h * 4) = make_float4(o[0], o[1], o[2], o[3]);
  }
#pragma unroll
  for (int i = 0; i < 20; ++i) {
    double val = (double)acc[i];
    val += __shfl_xor(val, 8, 64);
    val += __shfl_xor(val, 16, 64);
    val += __shfl_xor(val, 32, 64);
    if (lane < 8) red[wv][i < 16 ? h * 16 + i : 128 + h * 4 + (i - 16)] = val;
  }
  __syncthreads();
  if (threadIdx.x < 160) {
    const int i = threadIdx.x;
    partial[(size_t)blockIdx.x * 160 + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// dkv[g][i] = sum over the blocks of group g of partial[blk][i]: 4 interleaved chains (block j in chain
// j % 4) combined as (c0 + c1) + (c2 + c3) -- a fixed order
__global__ void linattn_group_combine_kernel(const double* __restrict__ partial, int blocks_per_group,
                                             float* __restrict__ dkv) {
  const int g = blockIdx.x, i = threadIdx.x;
  if (i >= 160) return;
  const double* p = partial + (size_t)g * blocks_per_group * 160 + i;
  double c[4] = {0.0, 0.0, 0.0, 0.0};
  int j = 0;
  for (; j + 4 <= blocks_per_group; j += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] += p[(size_t)(j + u) * 160];
  for (; j < blocks_per_group; ++j) c[j & 3] += p[(size_t)j * 160];
  dkv[(size_t)g * 160 + i] = (float)((c[0] + c[1]) + (c[2] + c[3]));
}

// source side: dK[s,h,d] = sum_m dKV[h][m][d] V[s,h,m] + dKs[h][d]; dV[s,h,m] = sum_d dKV[h][m][d] K[s,h,d]
__global__ __launch_bounds__(kTB) void linattn_bwd_kv_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                             long S, long spg, const float* __restrict__ dkv,
                                                             float* __restrict__ dk, float* __restrict__ dv) {
  const int h = threadIdx.x & 7;
  const long s = (long)blockIdx.x * kTokPerBlock + (threadIdx.x >> 3);
  if (s >= S) return;
  const float* G = dkv + (s / spg) * 160;
  const float4 k4 = ld4(k + s * 32 + h * 4), v4 = ld4(v + s * 32 + h * 4);
  const float kr[4] = {k4.x, k4.y, k4.z, k4.w}, V[4] = {v4.x, v4.y, v4.z, v4.w};
  float Kf[4], ok[4], ov[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) Kf[d] = elu1f(kr[d]);
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    float g = G[128 + h * 4 + d];
#pragma unroll
    for (int m = 0; m < 4; ++m) g = fmaf(G[h * 16 + m * 4 + d], V[m], g);
    ok[d] = g * elu1_grad(kr[d]);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float g = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) g = fmaf(G[h * 16 + m * 4 + d], Kf[d], g);
    ov[m] = g;
  }
  *reinterpret_cast<float4*>(dk + s * 32 + h * 4) = make_float4(ok[0], ok[1], ok[2], ok[3]);
  *reinterpret_cast<float4*>(dv + s * 32 + h * 4) = make_float4(ov[0], ov[1], ov[2], ov[3]);
}

static long tok_chunk(long T, long maxblk, long c = 1024) {
  while ((T + c - 1) / c > maxblk) c *= 2;
  return c;
}

}  // namespace tmvs

using namespace tmvs;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int token_linear_impl(const float* x, long tokens, int in_features, int out_features, const float* w,
                             const float* b, int transpose_w, const float* relu_of, int accumulate, const float* res,
                             float* y, void* stream) {
  if (!x || !w || !y || tokens <= 0) return TMVS_ERR_ARG;
  const dim3 grid((unsigned)((tokens + 16L * 4 * kLinTiles - 1) / (16L * 4 * kLinTiles)));
  hipStream_t st = (hipStream_t)stream;
#define TMVS_TL(I, O)                                                                                             \
  if (in_features == I && out_features == O) {                                                                    \
    if (transpose_w)                                                                                              \
      hipLaunchKernelGGL((token_linear_mfma_kernel<I, O, true>), grid, dim3(256), 0, st, x, tokens, w, b,         \
                         relu_of, accumulate, res, y);                                                            \
    else                                                                                                          \
      hipLaunchKernelGGL((token_linear_mfma_kernel<I, O, false>), grid, dim3(256), 0, st, x, tokens, w, b,        \
                         relu_of, accumulate, res, y);                                                            \
    TMVS_CHECK_LAUNCH();                                                                                          \
    return TMVS_OK;                                                                                               \
  }
  TMVS_TL(32, 32) TMVS_TL(32, 64) TMVS_TL(64, 32)
#undef TMVS_TL
  return TMVS_ERR_SHAPE;
}

extern "C" int tmvs_token_linear(const float* x, long tokens, int in_features, int out_features, const float* w,
                                 const float* b, int transpose_w, const float* relu_of, int accumulate, float* y,
                                 void* stream) {
  return token_linear_impl(x, tokens, in_features, out_features, w, b, transpose_w, relu_of, accumulate, nullptr, y,
                           stream);
}

extern "C" int tmvs_token_linear_res(const float* x, long tokens, int in_features, int out_features, const float* w,
                                     const float* b, int transpose_w, const float* relu_of, const float* residual,
                                     float* y, void* stream) {
  if (!residual || residual == y || !aligned16(residual) || !aligned16(y)) return TMVS_ERR_ARG;  // float4 rows
  return token_linear_impl(x, tokens, in_features, out_features, w, b, transpose_w, relu_of, 0, residual, y, stream);
}

extern "C" size_t tmvs_token_wgrad_workspace(long tokens, int a, int b) {
  const long c = tok_chunk(tokens, 512, 256);
  return (size_t)((tokens + c - 1) / c) * (a * b + a) * sizeof(double);
}

extern "C" int tmvs_token_wgrad(const float* dy, int a, const float* x, int b, long tokens, void* workspace,
                                size_t workspace_bytes, float* dw, float* db, int accumulate, void* stream) {
  if (!dy || !x || !workspace || !dw || !db || tokens <= 0) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_token_wgrad_workspace(tokens, a, b)) return TMVS_ERR_ARG;
  const long c = tok_chunk(tokens, 512, 256);
  const int nblk = (int)((tokens + c - 1) / c);
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
#define TMVS_TW(A, B, TA, TB)                                                                                   \
  if (a == A && b == B) {                                                                                       \
    hipLaunchKernelGGL((token_wgrad_kernel<A, B, TA, TB>), dim3(nblk), dim3(kTB), 0, st, dy, x, tokens, c, part); \
    TMVS_CHECK_LAUNCH();                                                                                        \
    hipLaunchKernelGGL(fmt_sum_partials_kernel, dim3((A * B + A + 15) / 16), dim3(kTB), 0, st,                 \
                       (const double*)part, nblk, (long)(A * B + A), (long)(A * B), dw, db, accumulate);        \
    TMVS_CHECK_LAUNCH();                                                                                        \
    return TMVS_OK;                                                                                             \
  }
  TMVS_TW(32, 32, 4, 4) TMVS_TW(64, 32, 8, 4) TMVS_TW(32, 64, 4, 8)
#undef TMVS_TW
  return TMVS_ERR_SHAPE;
}


// The LayerNorm kernels move a token's 32 channels as 16-byte quads: x, y, dy and dx must be
// 16-byte aligned (any row of a contiguous [tokens][32] buffer is when its base is).
extern "C" int tmvs_layer_norm_fwd(const float* x, long tokens, const float* g, const float* b, float* y, void* stream) {
  if (!x || !g || !b || !y || tokens <= 0) return TMVS_ERR_ARG;
  if (!aligned16(x) || !aligned16(y)) return TMVS_ERR_ARG;
  hipLaunchKernelGGL(layer_norm_fwd_kernel, dim3((unsigned)((tokens + kTB - 1) / kTB)), dim3(kTB), 0,
                     (hipStream_t)stream, x, tokens, g, b, y);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" size_t tmvs_layer_norm_bwd_workspace(long tokens) {
  const long c = tok_chunk(tokens, 1024, 256);
  return (size_t)((tokens + c - 1) / c) * 64 * sizeof(double);
}

extern "C" int tmvs_layer_norm_bwd(const float* dy, const float* x, long tokens, const float* g, void* workspace,
                                   size_t workspace_bytes, float* dx, float* dgb, int accumulate, void* stream) {
  if (!dy || !x || !g || !workspace || !dx || !dgb || tokens <= 0) return TMVS_ERR_ARG;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dx)) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_layer_norm_bwd_workspace(tokens)) return TMVS_ERR_ARG;
  const long c = tok_chunk(tokens, 1024, 256);
  const int nblk = (int)((tokens + c - 1) / c);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(layer_norm_bwd_kernel, dim3(nblk), dim3(kTB), 0, st, dy, x, tokens, g, c, dx, (double*)workspace);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(fmt_sum_partials_kernel, dim3(4), dim3(kTB), 0, st, (const double*)workspace, nblk, 64L, 64L, dgb,
                     dgb, accumulate);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_linattn_fwd(const float* q, long tokens, long tokens_per_group, const float* kv, long kv_stride,
                                float* msg, void* stream) {
  if (!q || !kv || !msg || tokens <= 0 || tokens_per_group <= 0) return TMVS_ERR_ARG;
  hipLaunchKernelGGL(linattn_fwd_kernel, dim3((unsigned)((tokens + kTokPerBlock - 1) / kTokPerBlock)), dim3(kTB), 0,
                     (hipStream_t)stream, q, tokens, tokens_per_group, kv, kv_stride, msg);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// blocks of tpb tokens that never straddle a group: tpb divides tokens_per_group
static long group_chunk(long tpg) {
  long c = 128;  // 4 tokens per (slot, head) thread: ~3 blocks per CU at the C5 size
  while (c > 1 && tpg % c) c >>= 1;
  while (tpg / c > 512 && tpg % (2 * c) == 0) c *= 2;
  return c;
}

extern "C" size_t tmvs_linattn_bwd_workspace(long tokens, long tokens_per_group) {
  return (size_t)(tokens / group_chunk(tokens_per_group)) * 160 * sizeof(double);
}

extern "C" int tmvs_linattn_bwd_q(const float* q, const float* dmsg, long tokens, long tokens_per_group,
                                  const float* kv, long kv_stride, void* workspace, size_t workspace_bytes, float* dq,
                                  float* dkv, void* stream) {
  if (!q || !dmsg || !kv || !workspace || !dq || !dkv || tokens <= 0 || tokens_per_group <= 0) return TMVS_ERR_ARG;
  if (tokens % tokens_per_group) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_linattn_bwd_workspace(tokens, tokens_per_group)) return TMVS_ERR_ARG;
  const long c = group_chunk(tokens_per_group);
  const int nblk = (int)(tokens / c);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(linattn_bwd_q_kernel, dim3(nblk), dim3(kTB), 0, st, q, dmsg, tokens, tokens_per_group, c, kv,
                     kv_stride, dq, (double*)workspace);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(linattn_group_combine_kernel, dim3((unsigned)(tokens / tokens_per_group)), dim3(256), 0, st,
                     (const double*)workspace, (int)(tokens_per_group / c), dkv);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_linattn_bwd_kv(const float* k, const float* v, long tokens, long tokens_per_group,
                                   const float* dkv, float* dk, float* dv, void* stream) {
  if (!k || !v || !dkv || !dk || !dv || tokens <= 0 || tokens_per_group <= 0) return TMVS_ERR_ARG;
  hipLaunchKernelGGL(linattn_bwd_kv_kernel, dim3((unsigned)((tokens + kTokPerBlock - 1) / kTokPerBlock)), dim3(kTB), 0,
                     (hipStream_t)stream, k, v, tokens, tokens_per_group, dkv, dk, dv);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
