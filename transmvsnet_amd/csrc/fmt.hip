// Feature Matching Transformer (models/FMT.py) linear attention on MI355X.
//
// d_model = 32, 8 heads x 4 dims, tokens [nv][L][32] (channels-last stage-1 map). One
// EncoderLayer (FMT.py:96-111) is two launches plus a tiny combine:
//   fmt_kv_partial  : per source token K = elu(Wk x + bk) + 1, V = Wv x + bv, accumulate
//                     KV[h][m][d] = Σ_s K[h,d] V[h,m] and Ksum[h][d] = Σ_s K[h,d]  (FMT.py:23-32)
//                     per workgroup -> partial slab [nv][nblk][160]
//   fmt_kv_combine  : sums the slabs in a fixed order (bitwise reproducible; no atomics)
// (dense 32x32 linears of the FFN use W2 transposed, TMVS_ENC_W2T)
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

// F.linear (addmm) y = x·W^T + b with W stored transposed ([in][out]): for each input i the
// OUT consecutive weights of row i arrive as one scalar load (SGPR operands of v_fma_f32) and
// are accumulated into y[0..OUT) -- per output an FMA chain over the input index, in order.
template <int IN, int OUT>
__device__ __forceinline__ void linear_t(const float* __restrict__ WT, const float* __restrict__ b, const float* x,
                                         float* y) {
#pragma unroll
  for (int o = 0; o < OUT; ++o) y[o] = 0.f;
#pragma unroll 2
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int o = 0; o < OUT; ++o) y[o] = fmaf(WT[i * OUT + o], x[i], y[o]);
#pragma unroll
  for (int o = 0; o < OUT; ++o) y[o] = y[o] + b[o];
}

// Layer weights are staged once per workgroup into LDS (34 KB) and read back as wave-uniform
// (broadcast) LDS loads; streaming them through the scalar cache from every wave thrashes it.
__device__ __forceinline__ void stage_weights(float* __restrict__ lds, const float* __restrict__ w, int n) {
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4)
    *reinterpret_cast<float4*>(lds + i) = *reinterpret_cast<const float4*>(w + i);
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

// tokens[v][p][c] = feat[v][c][p] + pe[c][y][x]: a block transposes 64 pixels x 32 channels through
// LDS for every view (coalesced 256-B channel rows in, 8 KB of contiguous token rows out), reading
// its positional-encoding tile once for all views.
__global__ __launch_bounds__(256) void fmt_embed_kernel(const float* __restrict__ feat, long view_stride,
                                                        const float* __restrict__ pe, int pe_h, int pe_w, int H, int W,
                                                        int nv, float* __restrict__ tokens) {
  __shared__ float tile[64][kD + 1];
  const int HW = H * W;
  const int p0 = blockIdx.x * 64;
  const int px = threadIdx.x & 63, c0 = threadIdx.x >> 6;  // loads: pixel px, channels c0 + 4k
  const int p = p0 + px;
  const bool in = p < HW;
  const int y = in ? p / W : 0, x = in ? p - y * W : 0;
  float pv[kD / 4];
#pragma unroll
  for (int k = 0; k < kD / 4; ++k) pv[k] = in ? pe[((size_t)(c0 + 4 * k) * pe_h + y) * pe_w + x] : 0.f;
  const int tp = threadIdx.x >> 3, q = threadIdx.x & 7;  // stores: token tp (and tp + 32), channel quad q
  float t[kD / 4];
  auto load = [&](int v) {
    const float* f = feat + (size_t)v * view_stride;
#pragma unroll
    for (int k = 0; k < kD / 4; ++k) t[k] = in ? f[(size_t)(c0 + 4 * k) * HW + p] : 0.f;
  };
  load(0);
#pragma unroll 1
  for (int v = 0; v < nv; ++v) {
    __syncthreads();  // the previous view's tile has been stored
#pragma unroll
    for (int k = 0; k < kD / 4; ++k) tile[px][c0 + 4 * k] = t[k] + pv[k];
    __syncthreads();
    if (v + 1 < nv) load(v + 1);  // in flight during this view's stores
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = tp + 32 * h;
      if (p0 + r < HW)
        *reinterpret_cast<float4*>(tokens + ((size_t)v * HW + p0 + r) * kD + 4 * q) =
            make_float4(tile[r][4 * q], tile[r][4 * q + 1], tile[r][4 * q + 2], tile[r][4 * q + 3]);
    }
  }
}

// ============================================================================ MFMA formulation
// The token-wise linears are dense 32x32 / 32x64 / 64x32 GEMMs over tokens. They run on the
// exact-fp32 matrix cores (v_mfma_f32_16x16x4_f32: D = A.B + C as an fp32 FMA chain, the VALU
// fp32 rate) with the weights resident in VGPRs as A fragments, loaded once per wave:
//   D[o][t] = sum_k W[o][k] X[t][k]   A = W (16 outputs x 4 k),  B = X^T (4 k x 16 tokens)
// Lane l holds D[o = 16mb + 4(l>>4) + r][t = l&15]: a token's 32 features live in lanes
// t, t+16, t+32, t+48 (8 each), and head h = 4mb + (l>>4) is lane-local (4 consecutive features).
// K-step s of a linear takes, in lane group g = l>>4, input feature f(s,g) = 16(s>>2) + 4g + (s&3):
// exactly the register (mb = s>>2, r = s&3) that lane already holds from the previous linear's
// accumulator -- so the linears chain with no data movement. Within a chain the input features
// are summed in that permuted order (an exact fp32 FMA chain; the reference's BLAS order is
// unknown anyway). VALU version of this file's history: bound by weight delivery (PMC).
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned uint4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int kfeat(int s, int g) { return 16 * (s >> 2) + 4 * g + (s & 3); }

// A fragments of a [OUT][IN] linear: frag[mb][s] = W[16mb + (l&15)][kfeat(s, l>>4)].
// TRANS: the packed matrix is stored [IN][OUT].
template <int OUT, int IN, bool TRANS>
__device__ __forceinline__ void load_afrag(const float* __restrict__ W, float (&frag)[OUT / 16][IN / 4], int lane) {
#pragma unroll
  for (int mb = 0; mb < OUT / 16; ++mb)
#pragma unroll
    for (int s = 0; s < IN / 4; ++s) {
      const int o = 16 * mb + (lane & 15), i = kfeat(s, lane >> 4);
      frag[mb][s] = TRANS ? W[i * OUT + o] : W[o * IN + i];
    }
}

// acc[mb] = sum_s A[mb][s] * in[s>>2][s&3]  (in: the B operand registers, D-layout of the input)
template <int OUT, int IN>
__device__ __forceinline__ void mfma_linear(const float (&frag)[OUT / 16][IN / 4], const floatx4 (&in)[IN / 16],
                                            floatx4 (&acc)[OUT / 16]) {
#pragma unroll
  for (int mb = 0; mb < OUT / 16; ++mb) acc[mb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < IN / 4; ++s)
#pragma unroll
    for (int mb = 0; mb < OUT / 16; ++mb)
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(frag[mb][s], in[s >> 2][s & 3], acc[mb], 0, 0, 0);
}

// A fragments staged in LDS in read order [mb][s/4][lane][4]: one ds_read_b128 per lane
// serves 4 consecutive k-steps of an MFMA chain, and the 64 lanes read 1 KiB contiguous
// (conflict-free). Used by fmt_apply_kernel, whose 96 weight VGPRs otherwise capped it at
// 2 waves/SIMD.
template <int OUT, int IN, bool TRANS>
__device__ __forceinline__ void stage_afrag(const float* __restrict__ W, float* __restrict__ lds) {
  constexpr int N = OUT * IN;  // = (OUT/16) * (IN/16) * 64 lanes * 4
  for (int idx = threadIdx.x; idx < N; idx += blockDim.x) {
    const int j = idx & 3, l = (idx >> 2) & 63, rest = idx >> 8;
    const int s4 = rest % (IN / 16), mb = rest / (IN / 16);
    const int s = 4 * s4 + j;
    const int o = 16 * mb + (l & 15), i = kfeat(s, l >> 4);
    lds[idx] = TRANS ? W[i * OUT + o] : W[o * IN + i];
  }
}

template <int OUT, int IN, int NT>
__device__ __forceinline__ void mfma_linear_lds(const float* __restrict__ fl, const floatx4 (&in)[NT][IN / 16],
                                                floatx4 (&acc)[NT][OUT / 16], int lane) {
#pragma unroll
  for (int p = 0; p < NT; ++p)
#pragma unroll
    for (int mb = 0; mb < OUT / 16; ++mb) acc[p][mb] = floatx4{0.f, 0.f, 0.f, 0.f};
  // per s4: every output block's fragment first, then the MFMAs block-interleaved (each accumulator's
  // own order unchanged), so consecutive MFMAs feed different accumulators
#pragma unroll
  for (int s4 = 0; s4 < IN / 16; ++s4) {
    float4 a4[OUT / 16];
#pragma unroll
    for (int mb = 0; mb < OUT / 16; ++mb)
      a4[mb] = *reinterpret_cast<const float4*>(fl + ((mb * (IN / 16) + s4) * 64 + lane) * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mb = 0; mb < OUT / 16; ++mb)
#pragma unroll
        for (int p = 0; p < NT; ++p)
          acc[p][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(j == 0 ? a4[mb].x : j == 1 ? a4[mb].y : j == 2 ? a4[mb].z : a4[mb].w,
                                                            in[p][s4][j], acc[p][mb], 0, 0, 0);
  }
}

// NT independent tiles interleaved: NT x OUT/16 independent accumulation chains in flight
template <int OUT, int IN, int NT>
__device__ __forceinline__ void mfma_linear_n(const float (&frag)[OUT / 16][IN / 4], const floatx4 (&in)[NT][IN / 16],
                                              floatx4 (&acc)[NT][OUT / 16]) {
#pragma unroll
  for (int p = 0; p < NT; ++p)
#pragma unroll
    for (int mb = 0; mb < OUT / 16; ++mb) acc[p][mb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < IN / 4; ++s)
#pragma unroll
    for (int p = 0; p < NT; ++p)
#pragma unroll
      for (int mb = 0; mb < OUT / 16; ++mb)
        acc[p][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(frag[mb][s], in[p][s >> 2][s & 3], acc[p][mb], 0, 0, 0);
}

// a token's 32 features are spread over lanes t, t+16, t+32, t+48 (8 per lane)
__device__ __forceinline__ float token_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

__device__ __forceinline__ void layer_norm_frag(floatx4 (&x)[2], const float* __restrict__ g,
                                                const float* __restrict__ b, int lane) {
  float s = 0.f;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += x[mb][r];
  const float mean = token_sum(s) / (float)kD;
  float v = 0.f;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = x[mb][r] - mean;
      v = fmaf(d, d, v);
    }
  const float rstd = 1.f / sqrtf(token_sum(v) / (float)kD + 1e-5f);
  const float bias = -rstd * mean;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    // features 16 mb + 4 (lane >> 4) + r, r < 4: one 16-byte read each of gamma and beta (aligned)
    const float4 g4 = *reinterpret_cast<const float4*>(g + 16 * mb + 4 * (lane >> 4));
    const float4 b4 = *reinterpret_cast<const float4*>(b + 16 * mb + 4 * (lane >> 4));
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) x[mb][r] = fmaf(fmaf(x[mb][r], rstd, bias), gg[r], bb[r]);
  }
}

__device__ __forceinline__ void load_token_frag(const float* __restrict__ row, floatx4 (&x)[2], int lane) {
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const float4 t = *reinterpret_cast<const float4*>(row + 16 * mb + 4 * (lane >> 4));
    x[mb] = floatx4{t.x, t.y, t.z, t.w};
  }
}

constexpr int kKvTilesPerWave = 8;     // kv: at most this many tiles per wave (see kv_tiles_per_wave)

// x + x[lane ^ 1], then ^2, ^4, ^8: the butterfly sum over a 16-lane row. The partner values move by
// DPP (quad_perm for 1 and 2; row_half_mirror = ^7 and row_mirror = ^15 composed with a quad_perm /
// half mirror for 4 and 8), not by ds_bpermute through the LDS unit: the same values in the same
// additions, so the sums are bitwise those of __shfl_xor.
#ifndef TMVS_KV_DPP
#define TMVS_KV_DPP 1
#endif
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float xor_sum16(float x) {
#if TMVS_KV_DPP
  x += dppf<0xB1>(x);               // quad_perm [1,0,3,2]: lane ^ 1
  x += dppf<0x4E>(x);               // quad_perm [2,3,0,1]: lane ^ 2
  x += dppf<0x1B>(dppf<0x141>(x));  // half mirror (^7) then quad_perm [3,2,1,0] (^3): lane ^ 4
  x += dppf<0x141>(dppf<0x140>(x)); // row mirror (^15) then half mirror (^7): lane ^ 8
#else
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) x += __shfl_xor(x, off, 64);
#endif
  return x;
}

// (KV, Ksum) partial sums: per wave, tiles of 16 source tokens; K, V by MFMA; per lane the
// two heads it owns are accumulated over its tokens, then summed over the 16 token lanes.
__global__ __launch_bounds__(256) void fmt_kv_partial_kernel(const float* __restrict__ src, int S,
                                                              const float* __restrict__ w,
                                                              float* __restrict__ partial, int tpw) {
  __shared__ float red[4][kKV];
  __shared__ __attribute__((aligned(16))) float frag[2 * 32 * 32];  // Wk, Wv fragments (see stage_afrag)
  const int v = blockIdx.y;
  // wave index wave-uniform (readfirstlane): the tile loop is then scalar control flow, not a divergent
  // loop whose per-lane exits make the compiler wait vmcnt(0) (stores included) at its head
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  stage_afrag<32, 32, true>(w + TMVS_ENC_WK, frag);
  stage_afrag<32, 32, true>(w + TMVS_ENC_WV, frag + 1024);
  float bk[2][4], bv[2][4];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bk[mb][r] = w[TMVS_ENC_BK + 16 * mb + 4 * g + r];
      bv[mb][r] = w[TMVS_ENC_BV + 16 * mb + 4 * g + r];
    }
  float kv[2][16], ks[2][4];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) kv[mb][i] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) ks[mb][i] = 0.f;
  }
  __syncthreads();
  const float* sv = src + (size_t)v * S * kD;
  const int tile0 = (blockIdx.x * 4 + wv) * tpw;
  floatx4 xa[2], xb[2];  // this tile's tokens, the next tile's (loaded while this one computes)
  if (tile0 * 16 < S) {
    const int t = tile0 * 16 + (lane & 15);
    load_token_frag(sv + (size_t)(t < S ? t : S - 1) * kD, xa, lane);
  }
  auto tile = [&](int it, floatx4 (&cur)[2], floatx4 (&nxt)[2]) {
    int salt = 0;  // opaque offset: fragment reads stay in the loop (not hoisted back into VGPRs)
    asm volatile("" : "+s"(salt));  // an SGPR: a VGPR here could alias a pending load (vmcnt wait)
    const float* fr = frag + salt;
    bool okp[1];
    floatx4 xin[1][2], kk[1][2], vv[1][2];
    {
      const int t = (tile0 + it) * 16 + (lane & 15);
      okp[0] = t < S;
      xin[0][0] = cur[0];
      xin[0][1] = cur[1];
      // unconditional (clamped row; past the wave's range the value is never used): a branch here
      // made the compiler wait vmcnt(0) for this prefetch before the tile's first MFMA
      const int tn = t + 16;
      load_token_frag(sv + (size_t)(tn < S ? tn : S - 1) * kD, nxt, lane);
    }
    mfma_linear_lds<32, 32, 1>(fr, xin, kk, lane);
    mfma_linear_lds<32, 32, 1>(fr + 1024, xin, vv, lane);
#pragma unroll
    for (int p = 0; p < 1; ++p)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const bool ok = okp[p];
      float kh[4], vh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kh[r] = ok ? elu1(kk[p][mb][r] + bk[mb][r]) : 0.f;
        vh[r] = ok ? vv[p][mb][r] + bv[mb][r] : 0.f;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int d = 0; d < 4; ++d) kv[mb][m * 4 + d] = fmaf(kh[d], vh[m], kv[mb][m * 4 + d]);
#pragma unroll
      for (int d = 0; d < 4; ++d) ks[mb][d] += kh[d];
    }
  };
  // (unrolled by two like the apply it needed 144 VGPRs, 3 waves/SIMD: one buffer, copied per tile)
#pragma unroll 1
  for (int it = 0; it < tpw; ++it) {
    if ((tile0 + it) * 16 >= S) break;  // wave-uniform
    tile(it, xa, xb);
    xa[0] = xb[0];
    xa[1] = xb[1];
  }
  // sum over the 16 token lanes of each lane group (fixed butterfly)
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) kv[mb][i] = xor_sum16(kv[mb][i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) ks[mb][i] = xor_sum16(ks[mb][i]);
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int h = 4 * mb + g;
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wv][h * 16 + i] = kv[mb][i];
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wv][128 + h * 4 + i] = ks[mb][i];
    }
  }
  __syncthreads();
  if (threadIdx.x < kKV) {
    const int i = threadIdx.x;
    partial[((size_t)v * gridDim.x + blockIdx.x) * kKV + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// grid (nv, 5): 32 groups x 32 entries; group g sums partial blocks g, g+32, ... with all
// loads independent, then the 32 group sums are added in a fixed order (bitwise reproducible).
__global__ __launch_bounds__(1024) void fmt_kv_combine_kernel(const float* __restrict__ partial, int nblk,
                                                              float* __restrict__ kv) {
  __shared__ float red[32][32];
  const int v = blockIdx.x;
  const int e = blockIdx.y * 32 + (threadIdx.x & 31);
  const int g = threadIdx.x >> 5;
  float s = 0.f;
#pragma unroll 4
  for (int b = g; b < nblk; b += 32) s += partial[((size_t)v * nblk + b) * kKV + e];
  red[g][threadIdx.x & 31] = s;
  __syncthreads();
  if (g == 0) {
    float t = red[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < 32; ++k) t += red[k][threadIdx.x];
    kv[(size_t)v * kKV + e] = t;
  }
}

// The rest of EncoderLayer.forward for tiles of 16 query tokens, entirely in registers;
// kApplyNT tiles are processed together so their MFMA chains interleave.
#ifndef TMVS_APPLY_NT
#define TMVS_APPLY_NT 1
#endif
constexpr int kApplyNT = TMVS_APPLY_NT;
#ifndef TMVS_APPLY_BUFST
#define TMVS_APPLY_BUFST 0
#endif
// (amdgpu_waves_per_eu(5) fits it in 94 VGPRs without AGPRs, 5 waves/SIMD instead of 4: the 8 applies
// measured 456.6 vs 448.1 us per step, 6 waves (80 VGPRs + scratch) 472.0 -- profiles/r11n: not kept)
__global__ __launch_bounds__(256) void fmt_apply_kernel(float* __restrict__ x, int L, const float* __restrict__ kvg,
                                                        long kv_stride, const float* __restrict__ w, int tpw) {
  __shared__ __attribute__((aligned(16))) float kvs[kKV];
  // the per-feature vectors, read from LDS in the tile loop: a global load there is a full memory
  // latency, and its vmcnt(0) wait also drains the next tile's token prefetch
  // [0, 32) BQ  [32, 64) BO  [64, 128) B1  [128, 160) B2  [160, 288) LN1G LN1B LN2G LN2B
  constexpr int kVB2 = 128, kVLN = 160;
  __shared__ __attribute__((aligned(16))) float vec[288];
  const int v = blockIdx.y;
  // wave index wave-uniform (readfirstlane): the tile loop is then scalar control flow, not a divergent
  // loop whose per-lane exits make the compiler wait vmcnt(0) (stores included) at its head
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  if (threadIdx.x < kKV) kvs[threadIdx.x] = kvg[(size_t)v * kv_stride + threadIdx.x];
  for (int i = threadIdx.x; i < 288; i += blockDim.x)
    vec[i] = i < 32 ? w[TMVS_ENC_BQ + i] : i < 64 ? w[TMVS_ENC_BO + i - 32] : i < 128 ? w[TMVS_ENC_B1 + i - 64]
                                                                                      : w[TMVS_ENC_B2 + i - kVB2];
  __shared__ __attribute__((aligned(16))) float frag[32 * 32 * 2 + 64 * 32 * 2];  // Wq, Wo, W1, W2 fragments
  stage_afrag<32, 32, false>(w + TMVS_ENC_WQ, frag);
  stage_afrag<32, 32, false>(w + TMVS_ENC_WO, frag + 1024);
  stage_afrag<64, 32, false>(w + TMVS_ENC_W1, frag + 2048);
  stage_afrag<32, 64, true>(w + TMVS_ENC_W2T, frag + 4096);
  __syncthreads();
  float* xv = x + (size_t)v * L * kD;
  const auto xr = raw_rsrc(xv, (unsigned)L * kD * 4);
  const int tile0 = (blockIdx.x * 4 + wv) * tpw;
  constexpr int NT = kApplyNT;
  // two token buffers used alternately (the loop unrolled by two, so they swap by name: a
  // loop-carried copy made the compiler wait vmcnt(0) -- this tile's stores included -- at the latch)
  floatx4 xa[NT][2], xb[NT][2];
#pragma unroll
  for (int p = 0; p < NT; ++p) {
    const int t = (tile0 + p) * 16 + (lane & 15);
    if (p < tpw) load_token_frag(xv + (size_t)(t < L ? t : L - 1) * kD, xa[p], lane);
  }
  auto tile = [&](int it, floatx4 (&cur)[NT][2], floatx4 (&nxt)[NT][2]) {
    int salt = 0;  // opaque offset: fragment reads stay in the loop (not hoisted back into VGPRs)
    asm volatile("" : "+s"(salt));  // an SGPR: a VGPR here could alias a pending load (vmcnt wait)
    const float* fr = frag + salt;
    const float* vb = vec + salt;
    float* row[NT];
    bool ok[NT];
    unsigned soff[NT];  // byte offset of the lane's token row in the view, or out of range
    floatx4 xs[NT][2];
#pragma unroll
    for (int p = 0; p < NT; ++p) {
      const int t = (tile0 + it + p) * 16 + (lane & 15);
      ok[p] = t < L && it + p < tpw;
      soff[p] = ok[p] ? (unsigned)t * (kD * 4) : kOffOut;
      row[p] = xv + (size_t)(t < L ? t : L - 1) * kD;
      xs[p][0] = cur[p][0];
      xs[p][1] = cur[p][1];
      const int tn = t + 16 * NT;
      // unconditional (clamped row; a prefetch past the wave's range is never used): a branch here made
      // the compiler wait vmcnt(0) for this prefetch before the tile's first MFMA
      load_token_frag(xv + (size_t)(tn < L ? tn : L - 1) * kD, nxt[p], lane);
    }
    floatx4 q[NT][2], msg[NT][2];
    mfma_linear_lds<32, 32, NT>(fr, xs, q, lane);
#pragma unroll
    for (int p = 0; p < NT; ++p)
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const int h = 4 * mb + g;
        // head h's K/V summary, bias and Ksum as 16-byte LDS reads issued together
        const float4 bq = *reinterpret_cast<const float4*>(vb + 4 * h);
        const float4 ks4 = *reinterpret_cast<const float4*>(kvs + 128 + h * 4);
        float4 kv4[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) kv4[m] = *reinterpret_cast<const float4*>(kvs + h * 16 + m * 4);
        const float bqa[4] = {bq.x, bq.y, bq.z, bq.w}, ksa[4] = {ks4.x, ks4.y, ks4.z, ks4.w};
        float qe[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) qe[d] = elu1(q[p][mb][d] + bqa[d]);
        float den = 0.f;
#pragma unroll
        for (int d = 0; d < 4; ++d) den = fmaf(qe[d], ksa[d], den);
        const float z = 1.f / (den + 1e-6f);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float kva[4] = {kv4[m].x, kv4[m].y, kv4[m].z, kv4[m].w};
          float num = 0.f;
#pragma unroll
          for (int d = 0; d < 4; ++d) num = fmaf(qe[d], kva[d], num);
          msg[p][mb][m] = num * z;
        }
      }
    floatx4 a[NT][2];
    mfma_linear_lds<32, 32, NT>(fr + 1024, msg, a, lane);
#pragma unroll
    for (int p = 0; p < NT; ++p) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
      {
        const float4 b4 = *reinterpret_cast<const float4*>(vb + 32 + 16 * mb + 4 * g);
        const float bo[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) xs[p][mb][r] = xs[p][mb][r] + (a[p][mb][r] + bo[r]);
      }
      layer_norm_frag(xs[p], vb + kVLN, vb + kVLN + kD, lane);
    }
    floatx4 hdn[NT][4], ff[NT][2];
    mfma_linear_lds<64, 32, NT>(fr + 2048, xs, hdn, lane);
#pragma unroll
    for (int p = 0; p < NT; ++p)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
      {
        const float4 b4 = *reinterpret_cast<const float4*>(vb + 64 + 16 * mb + 4 * g);
        const float b1[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) hdn[p][mb][r] = relu(hdn[p][mb][r] + b1[r]);
      }
    mfma_linear_lds<32, 64, NT>(fr + 4096, hdn, ff, lane);
#pragma unroll
    for (int p = 0; p < NT; ++p) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
      {
        const float4 b4 = *reinterpret_cast<const float4*>(vb + kVB2 + 16 * mb + 4 * g);
        const float b2[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) xs[p][mb][r] = xs[p][mb][r] + (ff[p][mb][r] + b2[r]);
      }
      layer_norm_frag(xs[p], vb + kVLN + 2 * kD, vb + kVLN + 3 * kD, lane);
      if (TMVS_APPLY_BUFST) {
        // unconditional buffer stores, rows outside the wave's range at an out-of-range offset (dropped):
        // no branch around the stores, so the next tile's wait for its prefetched tokens does not merge
        // with a path where those loads were the last VMEM ops (which made it wait for these stores too)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, xs[p][mb]), xr,
                                                 soff[p] == kOffOut ? kOffOut : soff[p] + (16 * mb + 4 * g) * 4, 0, 0);
      } else if (ok[p]) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          *reinterpret_cast<float4*>(row[p] + 16 * mb + 4 * g) =
              make_float4(xs[p][mb][0], xs[p][mb][1], xs[p][mb][2], xs[p][mb][3]);
      }
    }
  };
#pragma unroll 1
  for (int it = 0; it < tpw; it += 2 * NT) {
    if ((tile0 + it) * 16 >= L) break;  // wave-uniform
    tile(it, xa, xb);
    if (it + NT >= tpw || (tile0 + it + NT) * 16 >= L) break;
    tile(it + NT, xb, xa);
  }
}

// Resident 4-wave blocks of `kernel` on the whole GPU (its occupancy at 256 threads: VGPRs, LDS)
template <typename K>
static long block_slots(K kernel) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess || per <= 0) per = 4;
  return (long)(cus > 0 ? cus : 256) * per;
}
static int wave_slots_apply() {
  static long slots = 0;
  if (!slots) slots = 4 * block_slots(fmt_apply_kernel);
  return (int)slots;
}

// Tiles per wave: as many as possible (small partial slabs, short combine) while the launch still
// has >= 2048 waves (2 per SIMD); the one-view cross-attention K/V otherwise runs at 0.1 waves/SIMD.
// (Sizing it from the occupancy like the apply measured 28.6 -> 26.4 us for the 5-view launch, but it
// changes the partial sums' grouping -- the K/V bits -- and with them a C2 near-tie at stage 2 whose
// flip then moves stage 3's hypotheses (tests/test_gpu_fullsize.py, r11g): kept as before.)
static int kv_tiles_per_wave(int nv, int S) {
  const int tiles = (S + 15) / 16;
  int tpw = kKvTilesPerWave;
  while (tpw > 2 && (long)nv * ((tiles + tpw - 1) / tpw) < 2048) tpw >>= 1;
  return tpw;
}
static int kv_nblk(int nv, int S) {
  const int per = 16 * 4 * kv_tiles_per_wave(nv, S);
  return (S + per - 1) / per;
}
// Tiles per wave for the apply: the whole launch in ONE round of resident waves (5 per SIMD at its
// 92 VGPRs since the bias vectors moved to LDS): with a fixed 4 tiles per wave the C2 grid (5 x 3888
// tiles = 4.75 waves per SIMD at 4/SIMD) ran as a full round plus a 3/4-empty second one (2.4
// waves/SIMD on average, r05f).
static int apply_tiles_per_wave(int nv, int L) {
  const long tiles = (long)nv * ((L + 15) / 16);
  const long tpw = std::max<long>(1, (tiles + wave_slots_apply() - 1) / wave_slots_apply());
  return (int)((tpw + kApplyNT - 1) / kApplyNT * kApplyNT);  // whole groups of kApplyNT tiles
}
static int apply_nblk(int L, int tpw) { return (L + 16 * 4 * tpw - 1) / (16 * 4 * tpw); }

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_fmt_embed(const float* feat, long feat_view_stride, const float* pe, int pe_h, int pe_w, int nv,
                              int channels, int height, int width, float* tokens, void* stream) {
  if (!feat || !pe || !tokens || nv <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (channels != kD || height > pe_h || width > pe_w) return TMVS_ERR_SHAPE;
  const int HW = height * width;
  hipLaunchKernelGGL(fmt_embed_kernel, dim3((HW + 63) / 64), dim3(256), 0, (hipStream_t)stream, feat,
                     feat_view_stride, pe, pe_h, pe_w, height, width, nv, tokens);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" size_t tmvs_fmt_kv_grouped_workspace(int nv, int group_nv, int s_tokens) {
  if (nv <= 0 || group_nv <= 0 || s_tokens <= 0) return 0;
  return (size_t)nv * kv_nblk(group_nv, s_tokens) * kKV * sizeof(float);
}

extern "C" size_t tmvs_fmt_kv_workspace(int nv, int s_tokens) { return tmvs_fmt_kv_grouped_workspace(nv, nv, s_tokens); }

// The tiling (tiles per wave, hence each view's partial-sum grouping) is the one a launch over group_nv
// views uses, so a view's K/V is bitwise the same whichever subset of views a launch carries.
extern "C" int tmvs_fmt_kv_grouped(const float* source, int nv, int group_nv, int s_tokens, const float* enc_w,
                                   void* workspace, size_t workspace_bytes, float* kv, void* stream) {
  if (!source || !enc_w || !workspace || !kv || nv <= 0 || group_nv <= 0 || s_tokens <= 0) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_fmt_kv_grouped_workspace(nv, group_nv, s_tokens)) return TMVS_ERR_ARG;
  const int nblk = kv_nblk(group_nv, s_tokens);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fmt_kv_partial_kernel, dim3(nblk, nv), dim3(kKvBlock), 0, st, source, s_tokens, enc_w,
                     (float*)workspace, kv_tiles_per_wave(group_nv, s_tokens));
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(fmt_kv_combine_kernel, dim3(nv, kKV / 32), dim3(1024), 0, st, (const float*)workspace, nblk, kv);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_fmt_kv(const float* source, int nv, int s_tokens, const float* enc_w, void* workspace,
                           size_t workspace_bytes, float* kv, void* stream) {
  return tmvs_fmt_kv_grouped(source, nv, nv, s_tokens, enc_w, workspace, workspace_bytes, kv, stream);
}

// tiles_per_wave > 0 overrides the occupancy-sized tiling (the per-token arithmetic, hence the output, is the same)
int tmvs_fmt_apply_tiled(float* x, int nv, int l_tokens, const float* kv, long kv_view_stride, const float* enc_w,
                         int tiles_per_wave, void* stream) {
  if (!x || !kv || !enc_w || nv <= 0 || l_tokens <= 0 || kv_view_stride < 0) return TMVS_ERR_ARG;
  const int tpw = tiles_per_wave > 0 ? (tiles_per_wave + kApplyNT - 1) / kApplyNT * kApplyNT
                                     : apply_tiles_per_wave(nv, l_tokens);
  hipLaunchKernelGGL(fmt_apply_kernel, dim3(apply_nblk(l_tokens, tpw), nv), dim3(256), 0, (hipStream_t)stream, x,
                     l_tokens, kv, kv_view_stride, enc_w, tpw);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_fmt_apply(float* x, int nv, int l_tokens, const float* kv, long kv_view_stride,
                              const float* enc_w, void* stream) {
  return tmvs_fmt_apply_tiled(x, nv, l_tokens, kv, kv_view_stride, enc_w, 0, stream);
}
