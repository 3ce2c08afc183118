// FeatureNet training: the pieces of the backward of
// models/module.py:343-422 (Conv2d blocks, FPN merges) and models/dcn.py:66-80 (DCNv2 ->
// torchvision.ops.deform_conv2d) that the inference kernels do not already cover, plus the softmax
// backward of prob_volume = exp(log_softmax(logits)) (models/TransMVSNet.py:99).
//
// Layout: NHWC fp32 activations (as featurenet.hip), the offset/mask tensor om [B][27][H][W] as
// the DCN kernels read it (channel 2k / 2k+1 = dy / dx of tap k = 3i + j, 18 + k = mask logit).
//
//   conv2d_generic   strided:    y[o][co] = b[co] + sum_{k,ci} W[k][co][ci] x[o*s - pad + k][ci]
//                    transposed: y[i][co] = b[co] + sum_{k,ci} W[k][co][ci] x[(i + pad - k)/s][ci]
//                    (the data gradient of a strided conv; taps with s not dividing are skipped)
//   conv2d_wgrad     dW[k][a][b] = sum_p direct[p][a] * gathered[p*s - pad + k][b]
//   dcn backward     with col_k[p][c] = m_k(p) * bilinear_c(x, pos_k(p)) the forward's column and
//                    dcol_k[p][c] = sum_o dy[p][o] W[o][c][k]:
//                      dW[k][o][c]  = sum_p dy[p][o] col_k[p][c]
//                      d mask logit = m (1 - m) sum_c dcol * bilinear_c
//                      d pos_y      = m sum_c dcol * (hx (v10 - v00) + lx (v11 - v01))   (x alike)
//                      dx           = the bilinear scatter of m * dcol (torchvision's col2im)
//                    with torchvision's conventions (a sample outside (-1, H) x (-1, W) is zero and
//                    carries no gradient; corners outside the image read 0 and receive nothing).
//
// Determinism: every reduction over pixels (weight / bias gradients) is block partials in fp64 plus
// a fixed-order combine. The DCN input gradient is a scatter with data-dependent targets; it is
// accumulated in LDS windows (per block tile + a halo of R px) of 64-bit fixed point -- integer LDS
// atomics are order-independent, and on gfx950 ds_add_u64 is ~20x the rate of ds_add_f32 (193
// cycles per wave-instruction per CU, scripts/micro/lds_atomic.hip) -- converted once and summed per
// texel in a fixed block order; only corners beyond the window (offsets over R px) go to global
// memory with fp32 atomics, as torchvision's deformable_col2im adds every contribution with atomicAdd.
#include "common.h"
#include "reduce_mfma.h"

namespace tmvs {
namespace {

constexpr int kBlk = 256;

// ---------------------------------------------------------------- generic 2-D conv (VALU)
template <int CIN, int COB>
__global__ __launch_bounds__(kBlk) void conv2d_generic_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ bias, int cout, int B, int Hi,
                                                             int Wi, int Ho, int Wo, int K, int stride, int pad,
                                                             int transposed, int accumulate, float* __restrict__ y) {
  const int cob = blockIdx.y;
  const long np = (long)B * Ho * Wo;
  const long p = (long)blockIdx.x * kBlk + threadIdx.x;
  if (p >= np) return;
  const int ow = (int)(p % Wo);
  const long t = p / Wo;
  const int oh = (int)(t % Ho), b = (int)(t / Ho);
  float acc[COB];
#pragma unroll
  for (int c = 0; c < COB; ++c) acc[c] = 0.f;
  const float* xb = x + (size_t)b * Hi * Wi * CIN;
#pragma unroll 1
  for (int kh = 0; kh < K; ++kh) {
    int ih;
    if (transposed) {
      const int th = oh + pad - kh;
      if (th < 0 || th % stride) continue;
      ih = th / stride;
    } else {
      ih = oh * stride - pad + kh;
    }
    if (ih < 0 || ih >= Hi) continue;
#pragma unroll 1
    for (int kw = 0; kw < K; ++kw) {
      int iw;
      if (transposed) {
        const int tw = ow + pad - kw;
        if (tw < 0 || tw % stride) continue;
        iw = tw / stride;
      } else {
        iw = ow * stride - pad + kw;
      }
      if (iw < 0 || iw >= Wi) continue;
      const float* xp = xb + ((size_t)ih * Wi + iw) * CIN;
      const float* wk = w + ((size_t)(kh * K + kw) * cout + cob * COB) * CIN;  // wave-uniform
      if constexpr (CIN % 4 == 0) {
#pragma unroll 4
        for (int c4 = 0; c4 < CIN / 4; ++c4) {
          const float4 xv = *reinterpret_cast<const float4*>(xp + 4 * c4);
#pragma unroll
          for (int co = 0; co < COB; ++co) {
            const float* wc = wk + co * CIN + 4 * c4;
            acc[co] = fmaf(wc[0], xv.x, acc[co]);
            acc[co] = fmaf(wc[1], xv.y, acc[co]);
            acc[co] = fmaf(wc[2], xv.z, acc[co]);
            acc[co] = fmaf(wc[3], xv.w, acc[co]);
          }
        }
      } else {
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const float xv = xp[ci];
#pragma unroll
          for (int co = 0; co < COB; ++co) acc[co] = fmaf(wk[co * CIN + ci], xv, acc[co]);
        }
      }
    }
  }
  float* yp = y + (size_t)p * cout + cob * COB;
#pragma unroll
  for (int c = 0; c < COB; ++c) {
    float v = acc[c];
    if (bias) v = v + bias[cob * COB + c];
    if (accumulate) v = yp[c] + v;
    yp[c] = v;
  }
}

// ---------------------------------------------------------------- pixel-reduction helpers
// A register-tiled reduction sum_p a[p][i] * b[p][j] over a block's pixel range [v0, v1): chunks of
// 64 rows are staged in LDS by the callers' row loaders (float4 quads, zero rows where the gathered
// tap is outside); lane (ai, ci) of each wave owns a TA x TB block, fp32 per chunk, fp64 across
// chunks; the 4 waves combine in the fixed order ((w0 + w1) + w2) + w3. A = rows of `a` (padded to
// a multiple of 8 by the loader), BC = columns of `b` (multiple of 8).
template <int A, int BC, typename LoadA, typename LoadB>
__device__ __forceinline__ void tile_reduce(long v0, long v1, LoadA load_a, LoadB load_b, double* __restrict__ out) {
  constexpr int CH = 64, TA = A / 8, TB = BC / 8, SA = A + 4, SB = BC + 4;
  static_assert(A % 8 == 0 && BC % 8 == 0, "tile");
  static_assert(CH * (SA + SB) * 4 >= A * BC * 8, "combine buffer fits the staging LDS");
  __shared__ __attribute__((aligned(16))) float lds[CH * (SA + SB)];
  float* sa = lds;
  float* sb = lds + CH * SA;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ci = lane & 7, ai = lane >> 3;
  double acc[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = 0.0;
#pragma unroll 1
  for (long vb = v0; vb < v1; vb += CH) {
    __syncthreads();
    for (int i = threadIdx.x; i < CH * A / 4; i += kBlk) {
      const int r = i / (A / 4), q = i % (A / 4);
      const long v = vb + r;
      *reinterpret_cast<float4*>(sa + r * SA + 4 * q) = v < v1 ? load_a(v, q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = threadIdx.x; i < CH * BC / 4; i += kBlk) {
      const int r = i / (BC / 4), q = i % (BC / 4);
      const long v = vb + r;
      *reinterpret_cast<float4*>(sb + r * SB + 4 * q) = v < v1 ? load_b(v, q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    float s[TA][TB];
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) s[i][j] = 0.f;
#pragma unroll 4
    for (int r = wv; r < CH; r += 4) {
      float av[TA], bv[TB];
#pragma unroll
      for (int i = 0; i < TA; ++i) av[i] = sa[r * SA + ai * TA + i];
#pragma unroll
      for (int j = 0; j < TB; ++j) bv[j] = sb[r * SB + ci * TB + j];
#pragma unroll
      for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j) s[i][j] = fmaf(av[i], bv[j], s[i][j]);
    }
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) acc[i][j] += (double)s[i][j];
  }
  double* cmb = reinterpret_cast<double*>(lds);
#pragma unroll 1
  for (int w = 1; w < 4; ++w) {
    __syncthreads();
    if (wv == w)
#pragma unroll
      for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j) cmb[(ai * TA + i) * BC + ci * TB + j] = acc[i][j];
    __syncthreads();
    if (wv == 0)
#pragma unroll
      for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j) acc[i][j] += cmb[(ai * TA + i) * BC + ci * TB + j];
  }
  if (wv == 0)
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) out[(ai * TA + i) * BC + ci * TB + j] = acc[i][j];
}

// the matrix-core form (reduce_mfma.h) wherever both sides have >= 8 channels
template <int A, int BC, bool BROW = false, typename LoadA, typename LoadB>
__device__ __forceinline__ void tile_reduce_any(long v0, long v1, LoadA load_a, LoadB load_b, double* __restrict__ out) {
  if constexpr (A % 8 == 0 && BC % 8 == 0)
    tile_reduce_mfma<A, BC, BROW>(v0, v1, load_a, load_b, out);
  else
    tile_reduce<A, BC>(v0, v1, load_a, load_b, out);
}

__device__ __forceinline__ float4 load_row4(const float* __restrict__ base, long v, int ch, int q) {
  // 4 channels 4q..4q+3 of row v of a [.][ch] tensor, zero past ch (ch = 27 rows are not 16-B aligned)
  const float* r = base + (size_t)v * ch;
  const int c = 4 * q;
  if (ch % 4 == 0) return *reinterpret_cast<const float4*>(r + c);
  return make_float4(c < ch ? r[c] : 0.f, c + 1 < ch ? r[c + 1] : 0.f, c + 2 < ch ? r[c + 2] : 0.f,
                     c + 3 < ch ? r[c + 3] : 0.f);
}

// dW[k][a][b] (a padded to AP rows, b = BC): grid (nblk, K*K)
template <int AP, int BC>
__global__ __launch_bounds__(kBlk) void conv2d_wgrad_kernel(const float* __restrict__ direct, int a_ch,
                                                           const float* __restrict__ gath, int B, int Ph, int Pw,
                                                           int Gh, int Gw, int K, int stride, int pad, long ppb,
                                                           int nblk, double* __restrict__ partial) {
  int rb, k;
  if (!xcd_range_tap(K * K, nblk, rb, k)) return;
  const int kh = k / K, kw = k % K;
  const long np = (long)B * Ph * Pw;
  const long v0 = (long)rb * ppb, v1 = v0 + ppb < np ? v0 + ppb : np;
  auto la = [&](long v, int q) { return load_row4(direct, v, a_ch, q); };
  auto lb = [&](long v, int q) {
    int b, ph, pw;
    chunk_row_coords(v, Ph, Pw, b, ph, pw);  // rows of 64-aligned chunks (ppb_for: multiples of 1024)
    const int gh = ph * stride - pad + kh, gw = pw * stride - pad + kw;
    if (gh < 0 || gw < 0 || gh >= Gh || gw >= Gw) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(gath + (((size_t)b * Gh + gh) * Gw + gw) * BC + 4 * q);
  };
  tile_reduce_any<AP, BC>(v0, v1, la, lb, partial + ((size_t)rb * K * K + k) * AP * BC);
}

#ifndef TMVS_SMALL_DPP
#define TMVS_SMALL_DPP 1
#endif
// few channels on the gathered side (the image: 3): thread t owns pairs t, t+256, .. of a x b,
// straight from global memory (L1 hits), fp32 over a block's pixels in 8 interleaved chains, fp64 after
template <int A, int BC>
__global__ __launch_bounds__(kBlk) void conv2d_wgrad_small_kernel(const float* __restrict__ direct,
                                                                 const float* __restrict__ gath, int B, int Ph, int Pw,
                                                                 int Gh, int Gw, int K, int stride, int pad, long ppb,
                                                                 int nblk, double* __restrict__ partial) {
  constexpr int NPR = A * BC;
  __shared__ double red[NPR][kBlk / 64];
  int rb, k;
  if (!xcd_range_tap(K * K, nblk, rb, k)) return;
  const int kh = k / K, kw = k % K;
  const long np = (long)B * Ph * Pw;
  const long v0 = (long)rb * ppb, v1 = v0 + ppb < np ? v0 + ppb : np;
  float acc[NPR];
#pragma unroll
  for (int q = 0; q < NPR; ++q) acc[q] = 0.f;
  for (long v = v0 + threadIdx.x; v < v1; v += kBlk) {
    const int pw = (int)(v % Pw);
    const long t = v / Pw;
    const int ph = (int)(t % Ph), b = (int)(t / Ph);
    const int gh = ph * stride - pad + kh, gw = pw * stride - pad + kw;
    if (gh < 0 || gw < 0 || gh >= Gh || gw >= Gw) continue;
    const float* gp = gath + (((size_t)b * Gh + gh) * Gw + gw) * BC;
    float gv[BC];
#pragma unroll
    for (int c = 0; c < BC; ++c) gv[c] = gp[c];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float d = direct[v * A + a];
#pragma unroll
      for (int c = 0; c < BC; ++c) acc[a * BC + c] = fmaf(d, gv[c], acc[a * BC + c]);
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    double x = (double)acc[q];
    if (TMVS_SMALL_DPP) {
      x = wave_xor_sum_dpp(x);  // the same butterfly (common.h)
    } else {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    }
    if (lane == 0) red[q][wv] = x;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NPR; i += kBlk)
    partial[((size_t)rb * K * K + k) * NPR + i] = (red[i][0] + red[i][1]) + (red[i][2] + red[i][3]);
}

// out[i] = sum_j partial[j][i] in a fixed order (8 interleaved chains, then the chains in order)
__global__ __launch_bounds__(kBlk) void sum_partials_f32_kernel(const double* __restrict__ partial, int nblk, long n,
                                                                float* __restrict__ out) {
  __shared__ double red[8][32];
  const int g = threadIdx.x >> 5, q = threadIdx.x & 31;
  const long i = (long)blockIdx.x * 32 + q;
  double s = 0.0;
  if (i < n)
    s = strided_sum(partial + i, g, nblk, 8, (size_t)n, s);
  red[g][q] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    double t = red[0][q];
#pragma unroll
    for (int c = 1; c < 8; ++c) t += red[c][q];
    out[i] = (float)t;
  }
}

// the same with [nblk][taps][ap][b] partials (rows padded to ap) -> dw [taps][a][b]
__global__ __launch_bounds__(kBlk) void sum_partials_rows_kernel(const double* __restrict__ partial, int nblk, int ap,
                                                                 int a, int bc, long n, float* __restrict__ out) {
  __shared__ double red[8][32];
  const int g = threadIdx.x >> 5, q = threadIdx.x & 31;
  const long i = (long)blockIdx.x * 32 + q;
  const long per = (long)a * bc;
  const long src = i < n ? ((i / per) * ap + (i % per) / bc) * bc + i % bc : 0;
  const long np = n / per * ap * bc;
  double s = 0.0;
  if (i < n)
    s = strided_sum(partial + src, g, nblk, 8, (size_t)np, s);
  red[g][q] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    double t = red[0][q];
#pragma unroll
    for (int c = 1; c < 8; ++c) t += red[c][q];
    out[i] = (float)t;
  }
}

// per-block fp64 partial column sums of x [n][C] (C <= 32): thread (r, c) = (t / 32, t % 32)
__global__ __launch_bounds__(kBlk) void colsum_partial_kernel(const float* __restrict__ x, long n, int C, long ppb,
                                                              double* __restrict__ partial) {
  __shared__ double red[8][32];
  const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
  const long v0 = (long)blockIdx.x * ppb, v1 = v0 + ppb < n ? v0 + ppb : n;
  double s = 0.0;
  if (c < C) s = strided_sum(x + c, v0 + r0, v1, 8, (size_t)C, s);
  red[r0][c] = s;
  __syncthreads();
  if (r0 == 0 && c < C) {
    double t = red[0][c];
#pragma unroll
    for (int r = 1; r < 8; ++r) t += red[r][c];
    partial[(size_t)blockIdx.x * C + c] = t;
  }
}

// ---------------------------------------------------------------- DCN backward
// torchvision's sample geometry (models/dcn.py:71-80 -> deform_conv2d, stride 1, pad 1, dil 1) and
// the forward kernel's exact mask (featurenet.hip: fast sigmoid) and bilinear weights
struct DcnSample {
  bool inside;
  int y0, x0;
  float ly, lx, hy, hx, m;
};
__device__ __forceinline__ DcnSample dcn_sample(const float* __restrict__ omp, size_t HW, int y, int x, int k, int H,
                                                int W) {
  DcnSample s;
  const int ki = k / 3, kj = k - 3 * ki;
  const float py = (float)(y + ki - 1) + omp[(size_t)(2 * k) * HW];
  const float px = (float)(x + kj - 1) + omp[(size_t)(2 * k + 1) * HW];
  s.m = __frcp_rn(1.f + __expf(-omp[(size_t)(18 + k) * HW]));
  s.inside = py > -1.f && py < (float)H && px > -1.f && px < (float)W;
  const float y0 = floorf(py), x0 = floorf(px);
  s.ly = py - y0;
  s.lx = px - x0;
  s.hy = 1.f - s.ly;
  s.hx = 1.f - s.lx;
  s.y0 = s.inside ? (int)y0 : 0;
  s.x0 = s.inside ? (int)x0 : 0;
  return s;
}

namespace dbw {
constexpr int TY = 8, TX = 32;          // block tile of reference pixels (one thread each)
constexpr int R = 2;                    // offsets up to R px keep every corner in the LDS window
constexpr int CC = 8;                   // channels per pass
constexpr int WR = TY + 2 * R + 3, WC = TX + 2 * R + 3;
// one cell of one pass receives at most TY*TX pixels x 9 taps contributions
constexpr long kMaxAdds = (long)TY * TX * 9;
}  // namespace dbw

// max |x| over n floats of two tensors -> atomicMax on the bit patterns (non-negative floats order as
// unsigned): mx[0] over a (n_a), mx[1] over b (n_b). One atomic per block (a per-wave atomic on one
// word from ~30K waves serialised to 0.6 ms).
// The maxima are taken on the bit patterns of |x| as unsigned integers: for non-negative floats that
// order is the float order, and a NaN (bits above +inf's) wins -- fmaxf would drop it, and a NaN dy
// would then pass as finite into the fixed-point scatter (garbage integers instead of kFixBad).
__device__ __forceinline__ unsigned abits(float v) { return __float_as_uint(v) & 0x7fffffffu; }
__device__ __forceinline__ unsigned amax4(float4 u) {
  return max(max(abits(u.x), abits(u.y)), max(abits(u.z), abits(u.w)));
}
__global__ __launch_bounds__(kBlk) void absmax2_kernel(const float* __restrict__ a, long n_a,
                                                       const float* __restrict__ b, long n_b,
                                                       unsigned* __restrict__ mx) {
  __shared__ unsigned red[kBlk / 64];
  const float4* x = reinterpret_cast<const float4*>(blockIdx.y ? b : a);
  const long n4 = (blockIdx.y ? n_b : n_a) / 4;  // a multiple of 4 floats (16-byte aligned tensors)
  const long stride = (long)gridDim.x * kBlk;
  unsigned m0 = 0u, m1 = 0u;
  long i = (long)blockIdx.x * kBlk + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {  // two independent loads in flight per thread
    const float4 u = x[i], v = x[i + stride];
    m0 = max(m0, amax4(u));
    m1 = max(m1, amax4(v));
  }
  if (i < n4) m0 = max(m0, amax4(x[i]));
  unsigned m = max(m0, m1);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = red[0];
    for (int w = 1; w < kBlk / 64; ++w) t = max(t, red[w]);
    atomicMax(mx + blockIdx.y, t);
  }
}

// the window's fixed-point exponent: a contribution m * w_bilinear * dcol_c has magnitude at most
// CO max|dy| max|W| (m, w_bilinear <= 1), a cell at most kMaxAdds of them: with 2^e above that
// bound, units of 2^-(62 - e) keep every cell's int64 sum in range, at a resolution 2^-40 or finer
// relative to the largest possible contribution. A non-finite max|dy| or max|W| (an inf/NaN
// upstream gradient) returns kFixBad: every block's window is then written as NaN, so the WHOLE dx
// becomes NaN (torch's deform_conv2d backward would poison only the texels the bad values reach);
// this is deliberate -- a poisoned step must not pass as finite, and the training overflow check sees
// it -- instead of converting inf/NaN to garbage integers.
constexpr int kFixBad = -100000;
__device__ __forceinline__ int dcn_fix_shift(const unsigned* __restrict__ mx, int CO) {
  const double bound = (double)__uint_as_float(mx[0]) * (double)__uint_as_float(mx[1]) * CO * (double)dbw::kMaxAdds;
  if (!(bound < 1e300)) return kFixBad;  // inf or NaN (finite floats bound it far below 1e300)
  if (!(bound > 0.0)) return 0;          // every contribution is 0
  int e;
  frexp(bound, &e);
  return 62 - e;
}

// dcol, d om (NHWC [B][H][W][32], channels 27..31 zero) and the scatter of m * dcol into dx (accumulated)
// The block's LDS window of each 8-channel pass (int64 fixed point, see the header) is converted and
// written whole to scratch [block][cell][32] (plain, coalesced stores); dcn_gather_windows_kernel then
// sums, for every texel, the <= 4 windows covering it in a fixed block order (no global atomics).
// Corners beyond the window (offsets over R px) are added to dx with fp32 atomics before that pass.
// dcol on the matrix cores (TMVS_DCNB_MFMA, the 32-output-channel instance): per pass and tap pair,
// each wave computes the 16 x 64 tile D[(tap, channel)][pixel] = sum_o W[o][channel][tap] dy[pixel][o]
// as v_mfma_f32_16x16x4f32 chains over o (the same fmaf chain, bitwise, as the VALU form's
// dc[c] = fmaf(g[o], w[o][c], dc[c]), o ascending), parks it in a wave-private LDS tile, and every lane
// reads its pixel's 8 channels back, so the 9216 dcol MACs per pixel run beside the VALU's sampling,
// offset gradients and scatter (r14w: 2163 -> 2066 / 622 -> 559 / 200 -> 158 us at 4 x 576x768 /
// 288x384 / 144x192; the 8- and 16-channel instances measured slower that way and keep the VALU form).
#ifndef TMVS_DCNB_MFMA
#define TMVS_DCNB_MFMA 1
#endif
// The scatter's fixed-point conversion in fp32 (TMVS_DCNB_FIX32): ldexpf(f * dcol, k) is exact (a power-of-two
// scale of an fp32 value, no overflow below 2^62, and a result in the denormal range rounds to 0 either
// way) and llrintf rounds it to nearest-even as __double2ll_rn does the fp64 value: the same integers
// (bitwise, r14x). Faster for the VALU-dcol instances (32 -> 8: 1725 -> 1599 us), slower for the MFMA one
// (2109 -> 2228 us, 2 VGPRs spilled; with the dy^T operands re-read per tap pair to make room, 3480 us,
// r14z), so only there.
#ifndef TMVS_DCNB_FIX32
#define TMVS_DCNB_FIX32 1
#endif
template <int CO>
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(CO == 8 ? 4 : 3,
                                                                     CO == 8 ? 4 : 3)))
void dcn_bwd_data_kernel(const float* __restrict__ x, const float* __restrict__ om, const float* __restrict__ wt,
                         const float* __restrict__ dy, int B, int H, int W, const unsigned* __restrict__ absmax,
                         float* __restrict__ dx, float* __restrict__ dom, float* __restrict__ scratch) {
  using namespace dbw;
  constexpr bool kMf = TMVS_DCNB_MFMA && CO == 32;
  __shared__ unsigned long long win[WR * WC * CC];
  const int kfix = dcn_fix_shift(absmax, CO);
  const int tid = threadIdx.x;
  const int ntx = (W + TX - 1) / TX, nty = (H + TY - 1) / TY;
  int blk = blockIdx.x;
  const int bx = blk % ntx;
  blk /= ntx;
  const int by = blk % nty, b = blk / nty;
  const int y = by * TY + tid / TX, xq = bx * TX + tid % TX;
  const bool live = y < H && xq < W;
  const size_t HW = (size_t)H * W;
  const int wy0 = by * TY - R - 1, wx0 = bx * TX - R - 1;
  const size_t pix = (size_t)b * HW + (size_t)(live ? y : 0) * W + (live ? xq : 0);
  static_assert(CC == 8 && kBlk == 256 && CO % 4 == 0, "dcol tile: 2 taps x 8 channels, 4 waves");
  // wave-private [64 pixels][16] dcol tiles; quad q of pixel p at quad q ^ ((p >> 1) & 3) (conflict-free
  // b128 writes of a lane group's 16 pixels and b128 reads of 8 consecutive pixels)
  __shared__ __attribute__((aligned(16))) float dcl[kMf ? kBlk * 16 : 4];
  const int lane = tid & 63, l15 = lane & 15, lg = lane >> 4;
  float* dw = dcl + (kMf ? (tid & ~63) * 16 : 0);
  float g[CO];        // VALU form: this pixel's dy row
  float dyt[4][CO / 4];  // MFMA form, B operand dy^T: lane (g, n) of pixel block i holds dy[pixel 16 i + n][4 s + g]
  if constexpr (kMf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t2 = (tid & ~63) + 16 * i + l15;
      const int y2 = by * TY + t2 / TX, x2 = bx * TX + t2 % TX;
      const bool ok2 = y2 < H && x2 < W;
      const float* dp = dy + ((size_t)b * HW + (size_t)(ok2 ? y2 : 0) * W + (ok2 ? x2 : 0)) * CO + lg;
#pragma unroll
      for (int s = 0; s < CO / 4; ++s) dyt[i][s] = ok2 ? dp[4 * s] : 0.f;
    }
  } else {
#pragma unroll
    for (int o4 = 0; o4 < CO / 4; ++o4) {
      const float4 t = live ? *reinterpret_cast<const float4*>(dy + pix * CO + 4 * o4) : make_float4(0.f, 0.f, 0.f, 0.f);
      g[4 * o4] = t.x;
      g[4 * o4 + 1] = t.y;
      g[4 * o4 + 2] = t.z;
      g[4 * o4 + 3] = t.w;
    }
  }
  // A operand: W^T, lane (g, n) holds W[4 s + g][channel n & 7][tap 2 j + (n >> 3)] (0 past tap 8)
  auto load_wa = [&](int j, int cc, float (&wa)[CO / 4]) {
    const int kk = 2 * j + (l15 >> 3);
    const float* wp = wt + ((size_t)(kk < 9 ? kk : 0) * CO + lg) * 32 + cc * CC + (l15 & 7);
#pragma unroll
    for (int s = 0; s < CO / 4; ++s) wa[s] = kk < 9 ? wp[(size_t)(4 * s) * 32] : 0.f;
  };
  // taps 2j, 2j+1 of the pass: D rows 4g + r = (tap 2j + (g >> 1), channel 4 (g & 1) + r), column n
  auto dcol_pair = [&](const float (&wa)[CO / 4]) {
    floatx4_t d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = floatx4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < CO / 4; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[s], dyt[i][s], d[i], 0, 0, 0);
    asm volatile("" ::: "memory");  // the previous pair's reads of the tile precede these writes
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = 16 * i + l15;
      *reinterpret_cast<floatx4_t*>(dw + p * 16 + 4 * (lg ^ ((p >> 1) & 3))) = d[i];
    }
    asm volatile("" ::: "memory");  // one wave's LDS operations complete in order
  };
  const float* xb = x + (size_t)b * HW * 32;
  // corners beyond the window go to dx: the caller's dx (accumulate form) or the zeroed far buffer
  // (overwrite form, tmvs_dcn_backward_set); either way they raise the flag word after absmax[0..1]
  float* dxb = dx + (size_t)b * HW * 32;
  const float* omp = om + (size_t)b * 27 * HW + (size_t)(live ? y : 0) * W + (live ? xq : 0);
  float aY[9], aX[9], aM[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) aY[k] = aX[k] = aM[k] = 0.f;
#pragma unroll 1
  for (int cc = 0; cc < 32 / CC; ++cc) {
    for (int i = tid; i < WR * WC * CC; i += kBlk) win[i] = 0ull;
    __syncthreads();
    float wa[CO / 4];
    if constexpr (kMf) load_wa(0, cc, wa);
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
      if constexpr (kMf)
        if ((k & 1) == 0) {  // wave-uniform: the pair's tile, then the next pair's weights in flight
          dcol_pair(wa);
          if (k < 8) load_wa((k >> 1) + 1, cc, wa);
        }
      if (live) {
        const DcnSample s = dcn_sample(omp, HW, y, xq, k, H, W);
        if (!s.inside) continue;  // the column is 0 and carries no gradient (torchvision)
        float dc[CC];
        if constexpr (kMf) {
          const int q0 = 2 * (k & 1);
          const floatx4_t d0 = *reinterpret_cast<const floatx4_t*>(dw + lane * 16 + 4 * (q0 ^ ((lane >> 1) & 3)));
          const floatx4_t d1 = *reinterpret_cast<const floatx4_t*>(dw + lane * 16 + 4 * ((q0 + 1) ^ ((lane >> 1) & 3)));
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            dc[c] = d0[c];
            dc[4 + c] = d1[c];
          }
        } else {
          // dcol: the tap's weights are block-uniform -- scalar loads, SGPR operands of the FMAs
          const float* wk = wt + (size_t)k * CO * 32 + cc * CC;
#pragma unroll
          for (int c = 0; c < CC; ++c) dc[c] = 0.f;
#pragma unroll
          for (int o = 0; o < CO; ++o)
#pragma unroll
            for (int c = 0; c < CC; ++c) dc[c] = fmaf(g[o], wk[o * 32 + c], dc[c]);
        }
        const float wq[4] = {s.hy * s.hx, s.hy * s.lx, s.ly * s.hx, s.ly * s.lx};
        float v[4][CC];
        bool ok[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cy = s.y0 + (q >> 1), cx = s.x0 + (q & 1);
          ok[q] = (unsigned)cy < (unsigned)H && (unsigned)cx < (unsigned)W;
          const float* p = xb + ((size_t)(ok[q] ? cy : 0) * W + (ok[q] ? cx : 0)) * 32 + cc * CC;
          const float4 u0 = *reinterpret_cast<const float4*>(p), u1 = *reinterpret_cast<const float4*>(p + 4);
          const float t[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
          for (int c = 0; c < CC; ++c) v[q][c] = ok[q] ? t[c] : 0.f;
        }
        float sm = 0.f, sy = 0.f, sx = 0.f;
#pragma unroll
        for (int c = 0; c < CC; ++c) {
          float val = wq[0] * v[0][c];
          val = val + wq[1] * v[1][c];
          val = val + wq[2] * v[2][c];
          val = val + wq[3] * v[3][c];
          sm = fmaf(dc[c], val, sm);
          sy = fmaf(dc[c], s.hx * (v[2][c] - v[0][c]) + s.lx * (v[3][c] - v[1][c]), sy);
          sx = fmaf(dc[c], s.hy * (v[1][c] - v[0][c]) + s.ly * (v[3][c] - v[2][c]), sx);
        }
        aM[k] += sm;
        aY[k] += sy;
        aX[k] += sx;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (!ok[q]) continue;
          const int cy = s.y0 + (q >> 1), cx = s.x0 + (q & 1);
          const int ry = cy - wy0, rx = cx - wx0;
          const float f = s.m * wq[q];
          if (f == 0.f) continue;  // a zero bilinear weight (integer sample positions: 3 of 4 corners)
          if ((unsigned)ry < (unsigned)WR && (unsigned)rx < (unsigned)WC) {
            // channel-major window: neighbouring pixels' corners are neighbouring words
            unsigned long long* wp = win + ry * WC + rx;
#pragma unroll
            for (int c = 0; c < CC; ++c)
              atomicAdd(wp + c * (WR * WC),
                        (unsigned long long)(kfix == kFixBad ? 0ll
                                             : TMVS_DCNB_FIX32 && !kMf ? (long long)llrintf(ldexpf(f * dc[c], kfix))
                                                               : __double2ll_rn(ldexp((double)(f * dc[c]), kfix))));
          } else {  // an offset beyond the window: straight to global memory
            float* gp = dxb + ((size_t)cy * W + cx) * 32 + cc * CC;
            // the gather pass must read `far` (every writer stores the same 1; the word follows the two maxima)
            const_cast<unsigned*>(absmax)[2] = 1u;
#pragma unroll
            for (int c = 0; c < CC; ++c) unsafeAtomicAdd(gp + c, f * dc[c]);
          }
        }
      }
    }
    __syncthreads();
    float* sb = scratch + (size_t)blockIdx.x * (WR * WC) * 32 + cc * CC;
    for (int i = tid; i < WR * WC * CC; i += kBlk) {
      const int cell = i / CC, c = i - cell * CC;  // 8 lanes = one cell's 32-byte channel chunk
      sb[(size_t)cell * 32 + c] =
          kfix == kFixBad ? __builtin_nanf("") : (float)ldexp((double)(long long)win[c * (WR * WC) + cell], -kfix);
    }
    __syncthreads();
  }
  if (live) {  // one 128-byte row per pixel: 27 gradients + 5 zeros (16-byte aligned for the consumers)
    float r[32];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float m = __frcp_rn(1.f + __expf(-omp[(size_t)(18 + k) * HW]));
      r[2 * k] = m * aY[k];
      r[2 * k + 1] = m * aX[k];
      r[18 + k] = aM[k] * (m * (1.f - m));
    }
#pragma unroll
    for (int c = 27; c < 32; ++c) r[c] = 0.f;
    float4* dp = reinterpret_cast<float4*>(dom + pix * 32);
#pragma unroll
    for (int q = 0; q < 8; ++q) dp[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
  }
}

// dx[q][c] += sum over the blocks whose windows cover texel q (block rows / columns ascending) of their
// window value: one thread per (texel, channel); grid (ceil(32 W / 256), H, B), so a thread's texel comes
// from its block coordinates (a flat index had cost two 64-bit divisions per element)
// Overwrite form (far != nullptr): dx[q][c] = far[q][c] + (the window sum), where far holds the corners
// beyond the windows when the data kernel raised far_flag (else 0), and far is cleared again for the next call.
__global__ __launch_bounds__(kBlk) void dcn_gather_windows_kernel(const float* __restrict__ scratch, int B, int H,
                                                                 int W, float* __restrict__ dx,
                                                                 float* __restrict__ far,
                                                                 const unsigned* __restrict__ far_flag) {
  using namespace dbw;
  const int j = blockIdx.x * kBlk + threadIdx.x;
  if (j >= W * 32) return;
  const int c = j & 31, xq = j >> 5, y = blockIdx.y, b = blockIdx.z;
  const size_t i = ((size_t)b * H + y) * W * 32 + j;
  const int ntx = (W + TX - 1) / TX, nty = (H + TY - 1) / TY;
  // block row by covers window rows [by*TY - R - 1, by*TY - R - 1 + WR)
  const int by0 = max(0, (y + R + 1 - WR + 1 + TY - 1) / TY), by1 = min(nty - 1, (y + R + 1) / TY);
  const int bx0 = max(0, (xq + R + 1 - WC + 1 + TX - 1) / TX), bx1 = min(ntx - 1, (xq + R + 1) / TX);
  // at most 2 x 2 windows (WR < 2 TY, WC < 2 TX): all their loads issued before the adds, which run in
  // the loop order (block rows, then columns, ascending) from 0
  static_assert(WR < 2 * TY && WC < 2 * TX, "a texel is covered by at most 2 x 2 windows");
  float v[2][2];
  bool ok[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int by = by0 + r, bx = bx0 + q;
      ok[r][q] = by <= by1 && bx <= bx1;
      const int cell = (y - (by * TY - R - 1)) * WC + (xq - (bx * TX - R - 1));
      const size_t blk = ((size_t)b * nty + by) * ntx + bx;
      v[r][q] = ok[r][q] ? scratch[(blk * (WR * WC) + cell) * 32 + c] : 0.f;
    }
  const bool fr = far && *far_flag;
  const float d0 = far ? (fr ? far[i] : 0.f) : dx[i];
  if (fr) far[i] = 0.f;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (ok[r][q]) s += v[r][q];
  dx[i] = d0 + s;
}

// dW[k][o][c] = sum_p dy[p][o] col_k[p][c]: grid (nblk, 9), block partials [nblk][9][CO][32]. A thread
// stages two channel quads of one pixel (BROW), so the pixel's sample geometry (offsets, sigmoid mask,
// bilinear weights) is derived once for both instead of once per quad.
#ifndef TMVS_DCNW_BROW
#define TMVS_DCNW_BROW 1
#endif
template <int CO>
__global__ __launch_bounds__(kBlk) void dcn_bwd_weight_kernel(const float* __restrict__ x, const float* __restrict__ om,
                                                             const float* __restrict__ dy, int B, int H, int W, long ppb,
                                                             int nblk, double* __restrict__ partial) {
  // the 9 taps of a pixel range on one XCD (common.h: they gather the same input neighbourhood, r14l)
  int rb, k;
  if (!xcd_range_tap(9, nblk, rb, k)) return;
  const long HW = (long)H * W, np = (long)B * HW;
  const long v0 = (long)rb * ppb, v1 = v0 + ppb < np ? v0 + ppb : np;
  auto la = [&](long v, int q) { return *reinterpret_cast<const float4*>(dy + (size_t)v * CO + 4 * q); };
  // the column value of one channel quad at (pixel v, tap k), given the pixel's sample
  auto col_quad = [&](const DcnSample& s, int b, int q) {
    const float wq[4] = {s.hy * s.hx, s.hy * s.lx, s.ly * s.hx, s.ly * s.lx};
    const float* xb = x + (size_t)b * HW * 32 + 4 * q;
    float4 v4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int cy = s.y0 + (c >> 1), cx = s.x0 + (c & 1);
      const bool ok = (unsigned)cy < (unsigned)H && (unsigned)cx < (unsigned)W;
      v4[c] = ok ? *reinterpret_cast<const float4*>(xb + ((size_t)cy * W + cx) * 32) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto blend = [&](float a0, float a1, float a2, float a3) {
      float val = wq[0] * a0;
      val = val + wq[1] * a1;
      val = val + wq[2] * a2;
      val = val + wq[3] * a3;
      return s.m * val;  // the forward's column value (featurenet.hip: mk * val)
    };
    return make_float4(blend(v4[0].x, v4[1].x, v4[2].x, v4[3].x), blend(v4[0].y, v4[1].y, v4[2].y, v4[3].y),
                       blend(v4[0].z, v4[1].z, v4[2].z, v4[3].z), blend(v4[0].w, v4[1].w, v4[2].w, v4[3].w));
  };
  auto sample_at = [&](long v, int& b) {
    int yy, xx;
    chunk_row_coords(v, H, W, b, yy, xx);  // rows of 64-aligned chunks (ppb_for: multiples of 1024)
    const long p = (long)yy * W + xx;
    return dcn_sample(om + (size_t)b * 27 * HW + p, (size_t)HW, yy, xx, k, H, W);
  };
#if TMVS_DCNW_BROW
  auto lb = [&](long v, int q0, float4 (&o)[2]) {
    int b;
    const DcnSample s = sample_at(v, b);
    if (!s.inside) return;  // (o is zero)
    o[0] = col_quad(s, b, q0);
    o[1] = col_quad(s, b, q0 + 1);
  };
#else
  auto lb = [&](long v, int q) {
    int b;
    const DcnSample s = sample_at(v, b);
    if (!s.inside) return make_float4(0.f, 0.f, 0.f, 0.f);
    return col_quad(s, b, q);
  };
#endif
  tile_reduce_any<CO, 32, TMVS_DCNW_BROW>(v0, v1, la, lb, partial + ((size_t)rb * 9 + k) * CO * 32);
}

// ---------------------------------------------------------------- small backward pieces
// d prev [n][h][w][C] (+)= sum of the 2x2 block of d [n][2h][2w][C] (nearest x2 up-sampling's adjoint,
// models/module.py:413,417)
__global__ __launch_bounds__(kBlk) void nearest_up2_bwd_kernel(const float* __restrict__ d, int n, int h, int w, int C,
                                                              int accumulate, float* __restrict__ dprev) {
  const long i = (long)blockIdx.x * kBlk + threadIdx.x;
  const long tot = (long)n * h * w * C;
  if (i >= tot) return;
  const int c = (int)(i % C);
  long t = i / C;
  const int xx = (int)(t % w);
  t /= w;
  const int yy = (int)(t % h), b = (int)(t / h);
  const size_t row = (size_t)2 * w * C;
  const float* p = d + (((size_t)b * 2 * h + 2 * yy) * 2 * w + 2 * xx) * C + c;
  float s = (p[0] + p[C]) + (p[row] + p[row + C]);
  if (accumulate) s = dprev[i] + s;
  dprev[i] = s;
}

// d logits = p * (dp - sum_d p dp) per pixel (prob = exp(log_softmax(x)), models/TransMVSNet.py:99)
__global__ __launch_bounds__(kBlk) void softmax_bwd_kernel(const float* __restrict__ prob, const float* __restrict__ dprob,
                                                          int B, int D, long HW, float* __restrict__ dx) {
  const long i = (long)blockIdx.x * kBlk + threadIdx.x;
  if (i >= (long)B * HW) return;
  const long b = i / HW, p = i - b * HW;
  const float* pp = prob + (size_t)b * D * HW + p;
  const float* gp = dprob + (size_t)b * D * HW + p;
  float s = 0.f;
  for (int d = 0; d < D; ++d) s = fmaf(pp[(size_t)d * HW], gp[(size_t)d * HW], s);
  float* op = dx + (size_t)b * D * HW + p;
  for (int d = 0; d < D; ++d) op[(size_t)d * HW] = pp[(size_t)d * HW] * (gp[(size_t)d * HW] - s);
}

long ppb_for(long n, int max_blocks) {
  long ppb = 1024;
  while ((n + ppb - 1) / ppb > max_blocks) ppb *= 2;
  return ppb;
}

}  // namespace
}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_conv2d_generic(const float* x, int batch, int cin, int h_in, int w_in, const float* w,
                                   const float* bias, int cout, int h_out, int w_out, int k, int stride, int pad,
                                   int flags, float* y, void* stream) {
  if (!x || !w || !y || batch <= 0 || h_in <= 0 || w_in <= 0 || h_out <= 0 || w_out <= 0) return TMVS_ERR_ARG;
  if (k < 1 || k > 7 || (stride != 1 && stride != 2) || pad < 0) return TMVS_ERR_SHAPE;
  const int tr = (flags & TMVS_CONV_TRANSPOSED) ? 1 : 0, acc = (flags & TMVS_CONV_ACCUMULATE) ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  const long np = (long)batch * h_out * w_out;
  const unsigned gx = (unsigned)((np + kBlk - 1) / kBlk);
#define TMVS_C2G(CI, CB)                                                                                       \
  if (cin == CI && cout % CB == 0) {                                                                           \
    hipLaunchKernelGGL((conv2d_generic_kernel<CI, CB>), dim3(gx, cout / CB), dim3(kBlk), 0, st, x, w, bias,   \
                       cout, batch, h_in, w_in, h_out, w_out, k, stride, pad, tr, acc, y);                      \
    TMVS_CHECK_LAUNCH();                                                                                       \
    return TMVS_OK;                                                                                            \
  }
  if (cout % 8 == 0) {
    TMVS_C2G(3, 8) TMVS_C2G(8, 8) TMVS_C2G(16, 8) TMVS_C2G(27, 8) TMVS_C2G(32, 8)
  } else {
    TMVS_C2G(32, 9) TMVS_C2G(16, 9) TMVS_C2G(8, 9)
  }
#undef TMVS_C2G
  return TMVS_ERR_SHAPE;
}

static int wgrad_ap(int a) { return (a + 7) / 8 * 8; }

extern "C" size_t tmvs_conv2d_wgrad_workspace(int batch, int h, int w, int a_ch, int b_ch, int k) {
  const long np = (long)batch * h * w;
  const long ppb = ppb_for(np, 512);
  return (size_t)((np + ppb - 1) / ppb) * k * k * wgrad_ap(a_ch) * b_ch * sizeof(double);
}

// dw [k*k][a_ch][b_ch]
extern "C" int tmvs_conv2d_wgrad(const float* direct, int a_ch, int batch, int ph, int pw, const float* gathered,
                                 int b_ch, int gh, int gw, int k, int stride, int pad, void* workspace,
                                 size_t workspace_bytes, float* dw, void* stream) {
  if (!direct || !gathered || !workspace || !dw || batch <= 0 || ph <= 0 || pw <= 0 || gh <= 0 || gw <= 0)
    return TMVS_ERR_ARG;
  if (k < 1 || k > 7 || (stride != 1 && stride != 2)) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_conv2d_wgrad_workspace(batch, ph, pw, a_ch, b_ch, k)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const long np = (long)batch * ph * pw;
  const long ppb = ppb_for(np, 512);
  const int nblk = (int)((np + ppb - 1) / ppb);
  double* part = (double*)workspace;
  int ap = wgrad_ap(a_ch);
  bool done = false;
#define TMVS_WG2(AP, BC)                                                                                         \
  if (!done && ap == AP && b_ch == BC) {                                                                         \
    hipLaunchKernelGGL((conv2d_wgrad_kernel<AP, BC>), xcd_range_tap_grid(k * k, nblk), dim3(kBlk), 0, st, direct,   \
                       a_ch, gathered, batch, ph, pw, gh, gw, k, stride, pad, ppb, nblk, part);                 \
    done = true;                                                                                                 \
  }
  TMVS_WG2(8, 8) TMVS_WG2(8, 16) TMVS_WG2(8, 32) TMVS_WG2(16, 8) TMVS_WG2(16, 16) TMVS_WG2(16, 32) TMVS_WG2(32, 8)
  TMVS_WG2(32, 16) TMVS_WG2(32, 32)
#undef TMVS_WG2
  if (!done && a_ch == 8 && b_ch == 3) {
    hipLaunchKernelGGL((conv2d_wgrad_small_kernel<8, 3>), xcd_range_tap_grid(k * k, nblk), dim3(kBlk), 0, st, direct,
                       gathered, batch, ph, pw, gh, gw, k, stride, pad, ppb, nblk, part);
    ap = 8;
    done = true;
  }
  if (!done) return TMVS_ERR_SHAPE;
  TMVS_CHECK_LAUNCH();
  // combine [nblk][k*k][ap][b] -> [k*k][a][b] (rows >= a_ch are padding)
  const long n = (long)k * k * a_ch * b_ch;
  hipLaunchKernelGGL(sum_partials_rows_kernel, dim3((unsigned)((n + 31) / 32)), dim3(kBlk), 0, st, (const double*)part,
                     nblk, ap, a_ch, b_ch, n, dw);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" size_t tmvs_colsum_workspace(long n, int channels) {
  const long ppb = ppb_for(n, 1024);
  return (size_t)((n + ppb - 1) / ppb) * channels * sizeof(double);
}

extern "C" int tmvs_colsum(const float* x, long n, int channels, void* workspace, size_t workspace_bytes, float* out,
                           void* stream) {
  if (!x || !workspace || !out || n <= 0 || channels <= 0 || channels > 32) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_colsum_workspace(n, channels)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const long ppb = ppb_for(n, 1024);
  const int nblk = (int)((n + ppb - 1) / ppb);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nblk), dim3(kBlk), 0, st, x, n, channels, ppb, part);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_partials_f32_kernel, dim3((unsigned)((channels + 31) / 32)), dim3(kBlk), 0, st,
                     (const double*)part, nblk, (long)channels, out);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

static size_t dcn_partials_bytes(int batch, int cout, int height, int width) {
  const long np = (long)batch * height * width;
  const long ppb = ppb_for(np, 512);
  return ((size_t)((np + ppb - 1) / ppb) * 9 * cout * 32 * sizeof(double) + 255) & ~(size_t)255;
}

static long dcn_data_blocks(int batch, int height, int width) {
  return (long)batch * ((height + dbw::TY - 1) / dbw::TY) * ((width + dbw::TX - 1) / dbw::TX);
}

static size_t dcn_scratch_bytes(int batch, int height, int width) {
  return (size_t)dcn_data_blocks(batch, height, width) * dbw::WR * dbw::WC * 32 * sizeof(float);
}

// [weight-gradient partials (fp64)][per-block scatter windows: blocks x WR*WC x 32 fp32][absmax: 2 u32]
extern "C" size_t tmvs_dcn_backward_workspace(int batch, int cout, int height, int width) {
  return dcn_partials_bytes(batch, cout, height, width) + dcn_scratch_bytes(batch, height, width) + 256;
}

static int dcn_backward_impl(const float* x_nhwc, const float* offset_mask, const float* w_taps, const float* dy_nhwc,
                             int batch, int cin, int cout, int height, int width, void* workspace,
                             size_t workspace_bytes, float* dx_nhwc, float* dom_nhwc, float* dw_taps, float* far,
                             void* stream) {
  if (!x_nhwc || !offset_mask || !w_taps || !dy_nhwc || !workspace || !dx_nhwc || !dom_nhwc || !dw_taps)
    return TMVS_ERR_ARG;
  if (batch <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (cin != 32 || (cout != 8 && cout != 16 && cout != 32)) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_dcn_backward_workspace(batch, cout, height, width)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const unsigned nbd = (unsigned)dcn_data_blocks(batch, height, width);
  const long np = (long)batch * height * width;
  const long ppb = ppb_for(np, 512);
  const int nblk = (int)((np + ppb - 1) / ppb);
  double* part = (double*)workspace;
  float* scratch = (float*)((char*)workspace + dcn_partials_bytes(batch, cout, height, width));
  unsigned* absmax = (unsigned*)((char*)scratch + dcn_scratch_bytes(batch, height, width));
  unsigned* far_flag = absmax + 2;
  if (hipMemsetAsync(absmax, 0, 3 * sizeof(unsigned), st) != hipSuccess) return TMVS_ERR_HIP;
  hipLaunchKernelGGL(absmax2_kernel, dim3((unsigned)std::min<long>(512, (np * cout / 4 + kBlk - 1) / kBlk), 2),
                     dim3(kBlk), 0, st, dy_nhwc, np * cout, w_taps, 9L * cout * 32, absmax);
  TMVS_CHECK_LAUNCH();
#define TMVS_DCNB(CO)                                                                                             \
  case CO:                                                                                                        \
    hipLaunchKernelGGL(dcn_bwd_data_kernel<CO>, dim3(nbd), dim3(kBlk), 0, st, x_nhwc, offset_mask, w_taps, dy_nhwc, \
                       batch, height, width, (const unsigned*)absmax, far ? far : dx_nhwc, dom_nhwc, scratch);    \
    TMVS_CHECK_LAUNCH();                                                                                          \
    hipLaunchKernelGGL(dcn_gather_windows_kernel, dim3((unsigned)((width * 32 + kBlk - 1) / kBlk), height, batch),  \
                       dim3(kBlk), 0, st,                                                                         \
                       (const float*)scratch, batch, height, width, dx_nhwc, far, (const unsigned*)far_flag);     \
    TMVS_CHECK_LAUNCH();                                                                                          \
    hipLaunchKernelGGL(dcn_bwd_weight_kernel<CO>, xcd_range_tap_grid(9, nblk), dim3(kBlk), 0, st, x_nhwc,          \
                       offset_mask, dy_nhwc, batch, height, width, ppb, nblk, part);                            \
    break;
  switch (cout) {
    TMVS_DCNB(8)
    TMVS_DCNB(16)
    TMVS_DCNB(32)
  }
#undef TMVS_DCNB
  TMVS_CHECK_LAUNCH();
  const long n = 9L * cout * 32;
  hipLaunchKernelGGL(sum_partials_f32_kernel, dim3((unsigned)((n + 31) / 32)), dim3(kBlk), 0, st, (const double*)part,
                     nblk, n, dw_taps);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_dcn_backward(const float* x_nhwc, const float* offset_mask, const float* w_taps, const float* dy_nhwc,
                                 int batch, int cin, int cout, int height, int width, void* workspace,
                                 size_t workspace_bytes, float* dx_nhwc, float* dom_nhwc, float* dw_taps, void* stream) {
  return dcn_backward_impl(x_nhwc, offset_mask, w_taps, dy_nhwc, batch, cin, cout, height, width, workspace,
                           workspace_bytes, dx_nhwc, dom_nhwc, dw_taps, nullptr, stream);
}

extern "C" int tmvs_dcn_backward_set(const float* x_nhwc, const float* offset_mask, const float* w_taps,
                                     const float* dy_nhwc, int batch, int cin, int cout, int height, int width,
                                     void* workspace, size_t workspace_bytes, float* dx_nhwc, float* dom_nhwc,
                                     float* dw_taps, float* far_zeroed, void* stream) {
  if (!far_zeroed) return TMVS_ERR_ARG;
  return dcn_backward_impl(x_nhwc, offset_mask, w_taps, dy_nhwc, batch, cin, cout, height, width, workspace,
                           workspace_bytes, dx_nhwc, dom_nhwc, dw_taps, far_zeroed, stream);
}

extern "C" int tmvs_nearest_up2_backward_nhwc(const float* d, int n, int h, int w, int channels, int accumulate,
                                              float* dprev, void* stream) {
  if (!d || !dprev || n <= 0 || h <= 0 || w <= 0 || channels <= 0) return TMVS_ERR_ARG;
  const long tot = (long)n * h * w * channels;
  hipLaunchKernelGGL(nearest_up2_bwd_kernel, dim3((unsigned)((tot + kBlk - 1) / kBlk)), dim3(kBlk), 0,
                     (hipStream_t)stream, d, n, h, w, channels, accumulate, dprev);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_softmax_backward(const float* prob, const float* dprob, int batch, int ndepth, int height, int width,
                                     float* dlogits, void* stream) {
  if (!prob || !dprob || !dlogits || batch <= 0 || ndepth <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  const long HW = (long)height * width;
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3((unsigned)((batch * HW + kBlk - 1) / kBlk)), dim3(kBlk), 0,
                     (hipStream_t)stream, prob, dprob, batch, ndepth, HW, dlogits);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
