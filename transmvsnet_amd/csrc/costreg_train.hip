// CostRegNet training: the train-mode forward and the backward of
// models/module.py:425-456 (Conv3d :108-147, Deconv3d :150-191, nn.BatchNorm3d in train mode).
//
// Every convolution of the network and of its backward is one of two gathers over NDHWC
// activations with weights packed [27][Cout][Cin] (tap = kd*9 + kh*3 + kw):
//   strided    : y[o] = sum_{k,ci} W[k][co][ci] x[o*s - 1 + k]          (Conv3d k3 p1; dgrad of a
//                                                                        ConvTranspose3d)
//   transposed : y[o] = sum_{k,ci} W[k][co][ci] x[(o + 1 - k)/s]  if s | (o + 1 - k)
//                                                                       (ConvTranspose3d k3 s2 p1 op1;
//                                                                        dgrad of a Conv3d, s = 1 or 2)
// and every weight gradient is one reduction
//   dW[k][a][b] = sum_p direct[p][a] * gathered[p*s - 1 + k][b]         (conv: direct = dz, gathered
//                                                                        = x; deconv: direct = x,
//                                                                        gathered = dz)
// The host packs the weights for each use (transposes / flips are index permutations of the
// [27][Cout][Cin] block). BatchNorm3d in train mode: batch mean and biased variance per channel
// over all B*D*H*W voxels (fp64 partial sums, combined in a fixed order: bitwise reproducible),
// y = relu(fmaf(z, alpha, shift)) [+ skip] with alpha = gamma/sqrt(var+eps), shift = beta -
// mean*alpha (the CPU kernel's form); backward dz = alpha/N * (N*g - sum g - xhat * sum g*xhat),
// g = dy * [fmaf(z, alpha, shift) > 0]. No atomics anywhere: every reduction is block partials
// plus a fixed-order combine.
//
// Bounds: the convolutions are fp32 FMA work (VALU; 3 x 3,456 MAC per voxel for forward + both
// gradients), the BN passes HBM (2-3 reads of z per pass).
#include "common.h"
#include "reduce_mfma.h"

namespace tmvs {

constexpr int kTrainBlock = 256;

// ---------------------------------------------------------------- generic direct conv (VALU)
// One thread = one output voxel x COB output channels; the co-block's weights [27][COB][CIN] are
// wave-uniform (scalar loads feeding v_fma_f32 as SGPR operands: no LDS staging per block). Each
// tap's CIN input channels are one contiguous NDHWC row (float4 loads).
template <int CIN, int COB>
__global__ __launch_bounds__(kTrainBlock) void conv3d_generic_kernel(
    const float* __restrict__ x, const float* __restrict__ w, int cout, int B, int Di, int Hi, int Wi, int Do, int Ho,
    int Wo, int stride, int transposed, int accumulate, float* __restrict__ y) {
  const int cob = blockIdx.y;
  const long nvox = (long)B * Do * Ho * Wo;
  const long vl = (long)blockIdx.x * kTrainBlock + threadIdx.x;
  if (vl >= nvox) return;
  int ow = (int)(vl % Wo);
  if (transposed && stride == 2) {  // even columns first, then odd: a wave's lanes share the kw tap set
    const int ne = (Wo + 1) / 2;
    ow = ow < ne ? 2 * ow : 2 * (ow - ne) + 1;
  }
  const long v = vl - (long)(vl % Wo) + ow;
  long t = vl / Wo;
  const int oh = (int)(t % Ho);
  t /= Ho;
  const int od = (int)(t % Do);
  const int b = (int)(t / Do);
  float acc[COB];
#pragma unroll
  for (int c = 0; c < COB; ++c) acc[c] = 0.f;
  const float* xb = x + (size_t)b * Di * Hi * Wi * CIN;
#pragma unroll 1
  for (int k = 0; k < 27; ++k) {
    const int kd = k / 9, kh = (k / 3) % 3, kw = k % 3;
    int id, ih, iw;
    if (transposed) {
      const int td = od + 1 - kd, th = oh + 1 - kh, tw = ow + 1 - kw;
      if (td < 0 || th < 0 || tw < 0 || td % stride || th % stride || tw % stride) continue;
      id = td / stride;
      ih = th / stride;
      iw = tw / stride;
    } else {
      id = od * stride - 1 + kd;
      ih = oh * stride - 1 + kh;
      iw = ow * stride - 1 + kw;
      if (id < 0 || ih < 0 || iw < 0) continue;
    }
    if (id >= Di || ih >= Hi || iw >= Wi) continue;
    const float* xp = xb + (((size_t)id * Hi + ih) * Wi + iw) * CIN;
    const float* wk = w + ((size_t)k * cout + cob * COB) * CIN;  // wave-uniform: scalar loads, SGPR operands
    if constexpr (CIN % 4 == 0) {
#pragma unroll 4
      for (int c4 = 0; c4 < CIN / 4; ++c4) {
        const float4 xv = *reinterpret_cast<const float4*>(xp + 4 * c4);
#pragma unroll
        for (int co = 0; co < COB; ++co) {
          const float4 wv = *reinterpret_cast<const float4*>(wk + co * CIN + 4 * c4);
          acc[co] = fmaf(wv.x, xv.x, acc[co]);
          acc[co] = fmaf(wv.y, xv.y, acc[co]);
          acc[co] = fmaf(wv.z, xv.z, acc[co]);
          acc[co] = fmaf(wv.w, xv.w, acc[co]);
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
  float* yp = y + (size_t)v * cout + cob * COB;
  if (accumulate) {  // y += conv (a gradient reaching a tensor along two paths)
#pragma unroll
    for (int c = 0; c < COB; ++c) acc[c] = yp[c] + acc[c];
  }
  if constexpr (COB % 4 == 0) {
#pragma unroll
    for (int c4 = 0; c4 < COB / 4; ++c4)
      *reinterpret_cast<float4*>(yp + 4 * c4) = make_float4(acc[4 * c4], acc[4 * c4 + 1], acc[4 * c4 + 2], acc[4 * c4 + 3]);
  } else {
#pragma unroll
    for (int c = 0; c < COB; ++c) yp[c] = acc[c];
  }
}

// ---------------------------------------------------------------- weight gradient
// grid (nblk, 27): block (j, k) reduces voxels [j*vpb, (j+1)*vpb) of `direct` for tap k into
// partial[j][k][A][BC]; thread q owns pairs q, q+256, ... of the A x BC block. Rows of both
// operands are staged 32 voxels at a time in LDS (a zero row where the tap falls outside).
template <int A, int BC>
__global__ __launch_bounds__(kTrainBlock) void conv3d_wgrad_kernel(
    const float* __restrict__ direct, const float* __restrict__ gath, int B, int Pd, int Ph, int Pw, int Gd, int Gh,
    int Gw, int stride, long vpb, double* __restrict__ partial) {
  constexpr int NP = (A * BC + kTrainBlock - 1) / kTrainBlock;
  constexpr int CH = 32;
  __shared__ __attribute__((aligned(16))) float sd[CH][A];
  __shared__ __attribute__((aligned(16))) float sg[CH][BC];
  const int k = blockIdx.y;
  const int kd = k / 9, kh = (k / 3) % 3, kw = k % 3;
  const long nvox = (long)B * Pd * Ph * Pw;
  const long v0 = (long)blockIdx.x * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  double acc[NP];  // a 32-voxel chunk sums in fp32, chunks in fp64 (BN-normalised gradients cancel)
#pragma unroll
  for (int j = 0; j < NP; ++j) acc[j] = 0.0;
#pragma unroll 1
  for (long vb = v0; vb < v1; vb += CH) {
    __syncthreads();
    for (int i = threadIdx.x; i < CH * A; i += kTrainBlock) {
      const int r = i / A, a = i % A;
      const long v = vb + r;
      sd[r][a] = v < v1 ? direct[v * A + a] : 0.f;
    }
    for (int i = threadIdx.x; i < CH * BC; i += kTrainBlock) {
      const int r = i / BC, c = i % BC;
      const long v = vb + r;
      float val = 0.f;
      if (v < v1) {
        const int pw = (int)(v % Pw);
        long t = v / Pw;
        const int ph = (int)(t % Ph);
        t /= Ph;
        const int pd = (int)(t % Pd);
        const int b = (int)(t / Pd);
        const int gd = pd * stride - 1 + kd, gh = ph * stride - 1 + kh, gw = pw * stride - 1 + kw;
        if (gd >= 0 && gh >= 0 && gw >= 0 && gd < Gd && gh < Gh && gw < Gw)
          val = gath[((((size_t)b * Gd + gd) * Gh + gh) * Gw + gw) * BC + c];
      }
      sg[r][c] = val;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int q = threadIdx.x + j * kTrainBlock;
      if (q < A * BC) {
        const int a = q / BC, c = q % BC;
        float s = 0.f;
#pragma unroll 8
        for (int r = 0; r < CH; ++r) s = fmaf(sd[r][a], sg[r][c], s);
        acc[j] += (double)s;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int q = threadIdx.x + j * kTrainBlock;
    if (q < A * BC) partial[((size_t)blockIdx.x * 27 + k) * A * BC + q] = acc[j];
  }
}

// Register-tiled form for A, BC >= 8 (the CostRegNet / pathway layers): chunks of 64 voxel rows are
// staged in LDS (float4, the tap's gather computed once per row quad); wave w takes rows w, w+4, ...;
// lane (ai, ci) owns the TA x TB block a in [ai*TA, +TA), c in [ci*TB, +TB) (TA = A/8, TB = BC/8), fp32
// over a chunk's 16 rows then fp64; the 4 waves combine in a fixed order ((w0 + w1) + w2) + w3 through
// the (then idle) staging LDS.
template <int A, int BC>
__global__ __launch_bounds__(kTrainBlock) void conv3d_wgrad_tile_kernel(
    const float* __restrict__ direct, const float* __restrict__ gath, int B, int Pd, int Ph, int Pw, int Gd, int Gh,
    int Gw, int stride, long vpb, int nblk, double* __restrict__ partial) {
  int rb, k;  // the 27 taps of a voxel range on one XCD (common.h)
  if (!xcd_range_tap(27, nblk, rb, k)) return;
  const int kd = k / 9, kh = (k / 3) % 3, kw = k % 3;
  if constexpr (A % 8 == 0 && BC % 8 == 0) {  // on the matrix cores (reduce_mfma.h)
    const long nv = (long)B * Pd * Ph * Pw;
    const long u0 = (long)rb * vpb, u1 = u0 + vpb < nv ? u0 + vpb : nv;
    auto la = [&](long v, int q) { return *reinterpret_cast<const float4*>(direct + v * A + 4 * q); };
    auto lb = [&](long v, int q) {
      int b, pd, ph, pw;
      chunk_row_coords3(v, Pd, Ph, Pw, b, pd, ph, pw);  // rows of 64-aligned chunks (wgrad_vpb: multiples of 2048)
      const int gd = pd * stride - 1 + kd, gh = ph * stride - 1 + kh, gw = pw * stride - 1 + kw;
      if (gd < 0 || gh < 0 || gw < 0 || gd >= Gd || gh >= Gh || gw >= Gw) return make_float4(0.f, 0.f, 0.f, 0.f);
      return *reinterpret_cast<const float4*>(gath + ((((size_t)b * Gd + gd) * Gh + gh) * Gw + gw) * BC + 4 * q);
    };
    tile_reduce_mfma<A, BC>(u0, u1, la, lb, partial + ((size_t)rb * 27 + k) * A * BC);
    return;
  }
  constexpr int CH = 64, TA = A / 8, TB = BC / 8, SA = A + 4, SB = BC + 4;
  static_assert(A >= 8 && BC >= 8, "tile kernel needs 8 x 8 lanes");
  static_assert(CH * (SA + SB) * 4 >= A * BC * 8, "combine buffer fits the staging LDS");
  __shared__ __attribute__((aligned(16))) float lds[CH * (SA + SB)];
  float* sd = lds;
  float* sg = lds + CH * SA;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ci = lane & 7, ai = lane >> 3;
  const long nvox = (long)B * Pd * Ph * Pw;
  const long v0 = (long)rb * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  double acc[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = 0.0;
#pragma unroll 1
  for (long vb = v0; vb < v1; vb += CH) {
    __syncthreads();
    for (int i = threadIdx.x; i < CH * A / 4; i += kTrainBlock) {
      const int r = i / (A / 4), c = (i % (A / 4)) * 4;
      const long v = vb + r;
      *reinterpret_cast<float4*>(sd + r * SA + c) =
          v < v1 ? *reinterpret_cast<const float4*>(direct + v * A + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // the chunk's first voxel once (wave-uniform), then each row by carrying from it
    const int pw0 = (int)(vb % Pw);
    const long t0 = vb / Pw;
    const int ph0 = (int)(t0 % Ph), pd0 = (int)((t0 / Ph) % Pd), b0 = (int)(t0 / ((long)Ph * Pd));
    for (int i = threadIdx.x; i < CH * BC / 4; i += kTrainBlock) {
      const int r = i / (BC / 4), c = (i % (BC / 4)) * 4;
      const long v = vb + r;
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if (v < v1) {
        int pw = pw0 + r, ph = ph0, pd = pd0, b = b0;
        while (pw >= Pw) {
          pw -= Pw;
          if (++ph == Ph) {
            ph = 0;
            if (++pd == Pd) {
              pd = 0;
              ++b;
            }
          }
        }
        const int gd = pd * stride - 1 + kd, gh = ph * stride - 1 + kh, gw = pw * stride - 1 + kw;
        if (gd >= 0 && gh >= 0 && gw >= 0 && gd < Gd && gh < Gh && gw < Gw)
          val = *reinterpret_cast<const float4*>(gath + ((((size_t)b * Gd + gd) * Gh + gh) * Gw + gw) * BC + c);
      }
      *reinterpret_cast<float4*>(sg + r * SB + c) = val;
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
      for (int i = 0; i < TA; ++i) av[i] = sd[r * SA + ai * TA + i];
#pragma unroll
      for (int j = 0; j < TB; ++j) bv[j] = sg[r * SB + ci * TB + j];
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
  if (wv == 0) {
    double* out = partial + ((size_t)rb * 27 + k) * A * BC;
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) out[(ai * TA + i) * BC + ci * TB + j] = acc[i][j];
  }
}

// Few (a, b) pairs (conv0: 8 x 1, prob: 1 x 8): voxel-parallel instead -- thread t takes voxels
// t, t+256, ... of the block's range straight from global memory and accumulates all A*BC pairs, then
// a fixed LDS tree per pair.
template <int A, int BC>
__global__ __launch_bounds__(kTrainBlock) void conv3d_wgrad_small_kernel(
    const float* __restrict__ direct, const float* __restrict__ gath, int B, int Pd, int Ph, int Pw, int Gd, int Gh,
    int Gw, int stride, long vpb, double* __restrict__ partial) {
  constexpr int NPR = A * BC;
  __shared__ double red[NPR][kTrainBlock];
  const int k = blockIdx.y;
  const int kd = k / 9, kh = (k / 3) % 3, kw = k % 3;
  const long nvox = (long)B * Pd * Ph * Pw;
  const long v0 = (long)blockIdx.x * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  double acc[NPR];
#pragma unroll
  for (int q = 0; q < NPR; ++q) acc[q] = 0.0;
  // voxel coordinates advance incrementally (one division per thread, not three per voxel)
  long v = v0 + threadIdx.x;
  int pw = (int)(v % Pw), ph, pd, b;
  {
    const long t = v / Pw;
    ph = (int)(t % Ph);
    pd = (int)((t / Ph) % Pd);
    b = (int)(t / ((long)Ph * Pd));
  }
  for (; v < v1; v += kTrainBlock) {
    const int gd = pd * stride - 1 + kd, gh = ph * stride - 1 + kh, gw = pw * stride - 1 + kw;
    const bool ok = gd >= 0 && gh >= 0 && gw >= 0 && gd < Gd && gh < Gh && gw < Gw;
    const long vv = v;
    const float* gp = gath + ((((size_t)b * Gd + gd) * Gh + gh) * Gw + gw) * BC;  // used only when ok
    pw += kTrainBlock;
    while (pw >= Pw) {
      pw -= Pw;
      if (++ph == Ph) {
        ph = 0;
        if (++pd == Pd) {
          pd = 0;
          ++b;
        }
      }
    }
    if (!ok) continue;
    float dv[A], gv[BC];
#pragma unroll
    for (int a = 0; a < A; ++a) dv[a] = direct[vv * A + a];
#pragma unroll
    for (int c = 0; c < BC; ++c) gv[c] = gp[c];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int c = 0; c < BC; ++c) acc[a * BC + c] += (double)(dv[a] * gv[c]);
  }
#pragma unroll
  for (int q = 0; q < NPR; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int st = kTrainBlock / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st)
#pragma unroll
      for (int q = 0; q < NPR; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + st];
    __syncthreads();
  }
  if ((int)threadIdx.x < NPR) partial[((size_t)blockIdx.x * 27 + k) * NPR + threadIdx.x] = red[threadIdx.x][0];
}

// Few (a, b) pairs, one kd plane of taps per block row (grid.y = 3): a thread reads its voxel's
// `direct` row once per kd and the 9 neighbours' `gathered` rows (L1/L2 hits), keeping 9 x A x BC fp32
// sums over its voxels; then per value a fixed wave butterfly (fp64) and the 4 waves in order.
// Replaces 27 passes over `direct` with 3.
#ifndef TMVS_TAPS_DPP
#define TMVS_TAPS_DPP 1
#endif
template <int A, int BC>
__global__ __launch_bounds__(kTrainBlock) void conv3d_wgrad_taps_kernel(
    const float* __restrict__ direct, const float* __restrict__ gath, int B, int Pd, int Ph, int Pw, int Gd, int Gh,
    int Gw, int stride, long vpb, double* __restrict__ partial) {
  constexpr int NPR = A * BC;
  __shared__ double red[9 * NPR][kTrainBlock / 64];
  const int kd = blockIdx.y;
  const long nvox = (long)B * Pd * Ph * Pw;
  const long v0 = (long)blockIdx.x * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  float acc[9][NPR];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int q = 0; q < NPR; ++q) acc[k][q] = 0.f;
  long v = v0 + threadIdx.x;
  int pw = (int)(v % Pw), ph, pd, b;
  {
    const long t = v / Pw;
    ph = (int)(t % Ph);
    pd = (int)((t / Ph) % Pd);
    b = (int)(t / ((long)Ph * Pd));
  }
  for (; v < v1; v += kTrainBlock) {
    float dv[A];
    if constexpr (A % 4 == 0) {
#pragma unroll
      for (int a = 0; a < A; a += 4) {
        const float4 t4 = *reinterpret_cast<const float4*>(direct + v * A + a);
        dv[a] = t4.x;
        dv[a + 1] = t4.y;
        dv[a + 2] = t4.z;
        dv[a + 3] = t4.w;
      }
    } else {
#pragma unroll
      for (int a = 0; a < A; ++a) dv[a] = direct[v * A + a];
    }
    const float* gb = gath + (size_t)b * Gd * Gh * Gw * BC;
    const int gd = pd * stride - 1 + kd;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int gh = ph * stride - 1 + k / 3, gw = pw * stride - 1 + k % 3;
      const bool ok = gd >= 0 && gh >= 0 && gw >= 0 && gd < Gd && gh < Gh && gw < Gw;
      const float* gp = gb + (ok ? (((size_t)gd * Gh + gh) * Gw + gw) * BC : 0);  // always a valid address
      float gv[BC];  // unconditional loads, zeroed after: no branch per load
      if constexpr (BC % 4 == 0) {
#pragma unroll
        for (int c = 0; c < BC; c += 4) {
          const float4 t4 = *reinterpret_cast<const float4*>(gp + c);
          gv[c] = ok ? t4.x : 0.f;
          gv[c + 1] = ok ? t4.y : 0.f;
          gv[c + 2] = ok ? t4.z : 0.f;
          gv[c + 3] = ok ? t4.w : 0.f;
        }
      } else {
#pragma unroll
        for (int c = 0; c < BC; ++c) {
          const float t1 = gp[c];
          gv[c] = ok ? t1 : 0.f;
        }
      }
#pragma unroll
      for (int a = 0; a < A; ++a)
#pragma unroll
        for (int c = 0; c < BC; ++c) acc[k][a * BC + c] = fmaf(dv[a], gv[c], acc[k][a * BC + c]);
    }
    pw += kTrainBlock;
    while (pw >= Pw) {
      pw -= Pw;
      if (++ph == Ph) {
        ph = 0;
        if (++pd == Pd) {
          pd = 0;
          ++b;
        }
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      double x = (double)acc[k][q];
      if (TMVS_TAPS_DPP) {
        x = wave_xor_sum_dpp(x);  // the same butterfly (common.h)
      } else {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
      }
      if (lane == 0) red[k * NPR + q][wv] = x;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < 9 * NPR; i += kTrainBlock)
    partial[((size_t)blockIdx.x * 27 + kd * 9) * NPR + i] = (red[i][0] + red[i][1]) + (red[i][2] + red[i][3]);
}

// dw[i] = sum_j partial[j][i], j = 0..nblk-1 in order (fp64 accumulation)
__global__ __launch_bounds__(kTrainBlock) void sum_partials_kernel(const double* __restrict__ partial, int nblk, long n,
                                                                   float* __restrict__ out) {
  // 32 outputs per block; 8 interleaved chains (partial j in chain j % 8), then the chains in order:
  // a fixed order (bitwise reproducible) with 8x the loads in flight of one serial chain
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

// ---------------------------------------------------------------- BatchNorm3d, train mode
// Per-block fp64 partials of (sum z, sum z^2) per channel: thread t handles channel t % C of
// rows t / C, t / C + 256/C, ... (C divides 256).
// (grid.y = group: independent statistics of `groups` consecutive [nvox][C] slabs)
__global__ __launch_bounds__(kTrainBlock) void bn_stats_partial_kernel(const float* __restrict__ z, long nvox, int C,
                                                                       long vpb, double* __restrict__ partial) {
  __shared__ double red[2][kTrainBlock];
  z += (size_t)blockIdx.y * nvox * C;
  partial += (size_t)blockIdx.y * gridDim.x * 2 * C;
  const int c = threadIdx.x % C, r0 = threadIdx.x / C, rs = kTrainBlock / C;
  const long v0 = (long)blockIdx.x * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};  // 4 independent chains
  long v = v0 + r0;
  // groups of 4 rows, two in flight: group g+1's loads are issued before group g is accumulated
  // (a block walks up to thousands of rows; one group at a time left each load's latency exposed);
  // the groups are accumulated in order. (A generic ring of 2-4 groups under a rolled loop measured
  // slower than this hand-unrolled pair, r14t.)
  auto load4 = [&](long vv, float (&x)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = z[(vv + (long)j * rs) * C + c];
  };
  auto add4 = [&](const float (&x)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] += (double)x[j];
      q[j] += (double)x[j] * (double)x[j];
    }
  };
  float xa[4], xb[4];
  if (v + 3L * rs < v1) load4(v, xa);
  while (v + 3L * rs < v1) {
    const long vb = v + 4L * rs;
    const bool hb = vb + 3L * rs < v1;
    if (hb) load4(vb, xb);
    add4(xa);
    v = vb;
    if (!hb) break;
    const long va = v + 4L * rs;
    const bool ha = va + 3L * rs < v1;
    if (ha) load4(va, xa);
    add4(xb);
    v = va;
    if (!ha) break;
  }
  for (; v < v1; v += rs) {
    const double x = (double)z[v * C + c];
    s[0] += x;
    q[0] += x * x;
  }
  red[0][threadIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
  red[1][threadIdx.x] = (q[0] + q[1]) + (q[2] + q[3]);
  __syncthreads();
  if (threadIdx.x < C) {
    double ts = 0.0, tq = 0.0;
    for (int r = 0; r < rs; ++r) {
      ts += red[0][r * C + threadIdx.x];
      tq += red[1][r * C + threadIdx.x];
    }
    partial[((size_t)blockIdx.x * 2 + 0) * C + threadIdx.x] = ts;
    partial[((size_t)blockIdx.x * 2 + 1) * C + threadIdx.x] = tq;
  }
}

// out[k] = sum_j partial[j][k] (K values per block row): block k, threads stride j, then a fixed
// LDS tree -- deterministic, and parallel over the (up to 4096) partial rows
__global__ __launch_bounds__(kTrainBlock) void sum_double_partials_kernel(const double* __restrict__ partial, int nblk,
                                                                          int K, double* __restrict__ out) {
  __shared__ double red[kTrainBlock];
  const int k = blockIdx.x;
  partial += (size_t)blockIdx.y * nblk * K;  // grid.y = group
  out += (size_t)blockIdx.y * K;
  double a = 0.0;
  a = strided_sum(partial + k, threadIdx.x, nblk, kTrainBlock, (size_t)K, a);
  red[threadIdx.x] = a;
  __syncthreads();
  for (int st = kTrainBlock / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[k] = red[0];
}

// mean, biased var (fp32) from the summed (sum z, sum z^2)
__device__ __forceinline__ void bn_stats_from_sums(double s, double s2, long nvox, float& mean, float& var) {
  const double m = s / (double)nvox;
  const double v = s2 / (double)nvox - m * m;
  mean = (float)m;
  var = (float)(v > 0.0 ? v : 0.0);
}

// sum_double_partials_kernel's two sums of channel c (sum z, sum z^2; the same thread strides and LDS
// tree) and bn_stats_from_sums in one launch: grid (C, groups)
__global__ __launch_bounds__(kTrainBlock) void bn_sums_stats_kernel(const double* __restrict__ partial, int nblk, int C,
                                                                    long nvox, float* __restrict__ mean,
                                                                    float* __restrict__ var) {
  __shared__ double red[kTrainBlock];
  __shared__ double tot[2];
  const int c = blockIdx.x, K = 2 * C;
  partial += (size_t)blockIdx.y * nblk * K;
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    red[threadIdx.x] = strided_sum(partial + h * C + c, threadIdx.x, nblk, kTrainBlock, (size_t)K, 0.0);
    __syncthreads();
    for (int st = kTrainBlock / 2; st > 0; st >>= 1) {
      if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
      __syncthreads();
    }
    if (threadIdx.x == 0) tot[h] = red[0];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    bn_stats_from_sums(tot[0], tot[1], nvox, mean[(size_t)blockIdx.y * C + c], var[(size_t)blockIdx.y * C + c]);
}

__device__ __forceinline__ void bn_affine(float mean, float var, float g, float bt, float eps, float& al, float& sh) {
  al = (1.f / sqrtf(var + eps)) * g;
  sh = fmaf(-mean, al, bt);
}

// out = relu(fmaf(z, alpha, shift)) [+ skip]; group i / per uses statistics [group][C]
__global__ __launch_bounds__(kTrainBlock) void bn_relu_apply_kernel(const float* __restrict__ z, long n, long per, int C,
                                                                    const float* __restrict__ mean,
                                                                    const float* __restrict__ var,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta, float eps,
                                                                    const float* __restrict__ skip,
                                                                    float* __restrict__ out) {
  const long i = (long)blockIdx.x * kTrainBlock + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long gc = (i / per) * C + c;
  float al, sh;
  bn_affine(mean[gc], var[gc], gamma[c], beta[c], eps, al, sh);
  float y = relu(fmaf(z[i], al, sh));
  if (skip) y = skip[i] + y;
  out[i] = y;
}

// bn_relu_apply_kernel on float4s (C % 4 == 0, 16-byte aligned tensors): the channel / group indices
// and the per-channel affine once per 4 elements instead of a 64-bit divide and a sqrt per element;
// the same arithmetic per element, so the same bits
__global__ __launch_bounds__(kTrainBlock) void bn_relu_apply4_kernel(const float4* __restrict__ z, long n4, long per,
                                                                     int C, const float* __restrict__ mean,
                                                                     const float* __restrict__ var,
                                                                     const float* __restrict__ gamma,
                                                                     const float* __restrict__ beta, float eps,
                                                                     const float4* __restrict__ skip,
                                                                     float4* __restrict__ out) {
  const long i4 = (long)blockIdx.x * kTrainBlock + threadIdx.x;
  if (i4 >= n4) return;
  const long i = 4 * i4;
  const int c0 = (int)(i % C);
  const long g0 = (i / per) * C + c0;
  const float4 zv = z[i4];
  const float zz[4] = {zv.x, zv.y, zv.z, zv.w};
  float y[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float al, sh;
    bn_affine(mean[g0 + j], var[g0 + j], gamma[c0 + j], beta[c0 + j], eps, al, sh);
    y[j] = relu(fmaf(zz[j], al, sh));
  }
  if (skip) {
    const float4 sv = skip[i4];
    y[0] = sv.x + y[0];
    y[1] = sv.y + y[1];
    y[2] = sv.z + y[2];
    y[3] = sv.w + y[3];
  }
  out[i4] = make_float4(y[0], y[1], y[2], y[3]);
}

// backward pass 1: per-block fp64 partials of (sum g, sum g*xhat), g = dy * [fmaf(z, alpha, shift) > 0]
__global__ __launch_bounds__(kTrainBlock) void bn_relu_bwd_partial_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, long nvox, int C, const float* __restrict__ mean,
    const float* __restrict__ var, const float* __restrict__ gamma, const float* __restrict__ beta, float eps, long vpb,
    double* __restrict__ partial) {
  __shared__ double red[2][kTrainBlock];
  const int c = threadIdx.x % C, r0 = threadIdx.x / C, rs = kTrainBlock / C;
  dy += (size_t)blockIdx.y * nvox * C;  // grid.y = group
  z += (size_t)blockIdx.y * nvox * C;
  partial += (size_t)blockIdx.y * gridDim.x * 2 * C;
  mean += (size_t)blockIdx.y * C;
  var += (size_t)blockIdx.y * C;
  float al, sh;
  bn_affine(mean[c], var[c], gamma[c], beta[c], eps, al, sh);
  const float m = mean[c], rstd = 1.f / sqrtf(var[c] + eps);
  const long v0 = (long)blockIdx.x * vpb, v1 = v0 + vpb < nvox ? v0 + vpb : nvox;
  double sg[4] = {0.0, 0.0, 0.0, 0.0}, sgx[4] = {0.0, 0.0, 0.0, 0.0};
  long v = v0 + r0;
  // groups of 4 rows, two in flight (as bn_stats_partial_kernel), accumulated in the same order
  auto load4 = [&](long vv, float (&zz)[4], float (&gg)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      zz[j] = z[(vv + (long)j * rs) * C + c];
      gg[j] = dy[(vv + (long)j * rs) * C + c];
    }
  };
  auto add4 = [&](const float (&zz)[4], const float (&gg)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float g = fmaf(zz[j], al, sh) > 0.f ? gg[j] : 0.f;
      sg[j] += (double)g;
      sgx[j] += (double)g * (double)((zz[j] - m) * rstd);
    }
  };
  float za[4], ga[4], zb[4], gb[4];
  if (v + 3L * rs < v1) load4(v, za, ga);
  while (v + 3L * rs < v1) {
    const long vb = v + 4L * rs;
    const bool hb = vb + 3L * rs < v1;
    if (hb) load4(vb, zb, gb);
    add4(za, ga);
    v = vb;
    if (!hb) break;
    const long va = v + 4L * rs;
    const bool ha = va + 3L * rs < v1;
    if (ha) load4(va, za, ga);
    add4(zb, gb);
    v = va;
    if (!ha) break;
  }
  for (; v < v1; v += rs) {
    const float zz = z[v * C + c];
    const float g = fmaf(zz, al, sh) > 0.f ? dy[v * C + c] : 0.f;
    sg[0] += (double)g;
    sgx[0] += (double)g * (double)((zz - m) * rstd);
  }
  red[0][threadIdx.x] = (sg[0] + sg[1]) + (sg[2] + sg[3]);
  red[1][threadIdx.x] = (sgx[0] + sgx[1]) + (sgx[2] + sgx[3]);
  __syncthreads();
  if (threadIdx.x < C) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < rs; ++r) {
      a += red[0][r * C + threadIdx.x];
      b += red[1][r * C + threadIdx.x];
    }
    partial[((size_t)blockIdx.x * 2 + 0) * C + threadIdx.x] = a;
    partial[((size_t)blockIdx.x * 2 + 1) * C + threadIdx.x] = b;
  }
}

// dbeta = sum g, dgamma = sum g*xhat from the summed partials: per group in fp32, then added over the
// groups in order (as autograd accumulates the per-view gradients of a module called per view)
// (run by the first block of the backward apply kernels, thread c < C: one launch less per BatchNorm)
__device__ __forceinline__ void bn_relu_bwd_finalize(const double* __restrict__ sums, int C, int groups,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = threadIdx.x;
  if (blockIdx.x != 0 || c >= C) return;
  float b = (float)sums[c], g = (float)sums[C + c];
  for (int k = 1; k < groups; ++k) {
    b = b + (float)sums[(size_t)k * 2 * C + c];
    g = g + (float)sums[(size_t)k * 2 * C + C + c];
  }
  dbeta[c] = b;
  dgamma[c] = g;
}

// pass 2: dz = gamma*rstd/N * (N*g - sum g - xhat * sum g*xhat)
__global__ __launch_bounds__(kTrainBlock) void bn_relu_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, long n, int C, long nvox, const float* __restrict__ mean,
    const float* __restrict__ var, const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    const double* __restrict__ sums, int groups, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dz) {
  bn_relu_bwd_finalize(sums, C, groups, dgamma, dbeta);
  const long i = (long)blockIdx.x * kTrainBlock + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long grp = i / (nvox * C);  // statistics and sums of element i's group
  const long gc = grp * C + c;
  const double* sg = sums + (size_t)grp * 2 * C;
  float al, sh;
  bn_affine(mean[gc], var[gc], gamma[c], beta[c], eps, al, sh);
  const float zz = z[i];
  const float rstd = 1.f / sqrtf(var[gc] + eps);
  const float xhat = (zz - mean[gc]) * rstd;
  const float g = fmaf(zz, al, sh) > 0.f ? dy[i] : 0.f;
  const double inv_n = 1.0 / (double)nvox;
  const float mg = (float)(sg[c] * inv_n), mgx = (float)(sg[C + c] * inv_n);
  dz[i] = (gamma[c] * rstd) * ((g - mg) - xhat * mgx);
}

// bn_relu_bwd_apply_kernel on float4s (C % 4 == 0, 16-byte aligned): same per-element arithmetic
__global__ __launch_bounds__(kTrainBlock) void bn_relu_bwd_apply4_kernel(
    const float4* __restrict__ dy, const float4* __restrict__ z, long n4, int C, long nvox,
    const float* __restrict__ mean, const float* __restrict__ var, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, const double* __restrict__ sums, int groups, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float4* __restrict__ dz) {
  bn_relu_bwd_finalize(sums, C, groups, dgamma, dbeta);
  const long i4 = (long)blockIdx.x * kTrainBlock + threadIdx.x;
  if (i4 >= n4) return;
  const long i = 4 * i4;
  const int c0 = (int)(i % C);
  const long grp = i / (nvox * C);
  const long g0 = grp * C + c0;
  const double* sg = sums + (size_t)grp * 2 * C;
  const double inv_n = 1.0 / (double)nvox;
  const float4 zv = z[i4], dv = dy[i4];
  const float zz[4] = {zv.x, zv.y, zv.z, zv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + j;
    const long gc = g0 + j;
    float al, sh;
    bn_affine(mean[gc], var[gc], gamma[c], beta[c], eps, al, sh);
    const float rstd = 1.f / sqrtf(var[gc] + eps);
    const float xhat = (zz[j] - mean[gc]) * rstd;
    const float g = fmaf(zz[j], al, sh) > 0.f ? dd[j] : 0.f;
    const float mg = (float)(sg[c] * inv_n), mgx = (float)(sg[C + c] * inv_n);
    o[j] = (gamma[c] * rstd) * ((g - mg) - xhat * mgx);
  }
  dz[i4] = make_float4(o[0], o[1], o[2], o[3]);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
#ifndef TMVS_BN_VEC4
#define TMVS_BN_VEC4 1
#endif

// ---------------------------------------------------------------- dispatch helpers
template <int CIN, int COB>
static int launch_generic(const float* x, const float* w, int cout, int B, int Di, int Hi, int Wi, int Do, int Ho,
                          int Wo, int stride, int transposed, int accumulate, float* y, hipStream_t st) {
  const long nvox = (long)B * Do * Ho * Wo;
  hipLaunchKernelGGL((conv3d_generic_kernel<CIN, COB>), dim3((unsigned)((nvox + kTrainBlock - 1) / kTrainBlock),
                                                             cout / COB),
                     dim3(kTrainBlock), 0, st, x, w, cout, B, Di, Hi, Wi, Do, Ho, Wo, stride, transposed, accumulate, y);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

static long wgrad_vpb(long nvox) {
  long vpb = 2048;
  while ((nvox + vpb - 1) / vpb > 512) vpb *= 2;
  return vpb;
}

template <int A, int BC>
static int launch_wgrad(const float* direct, const float* gath, int B, int Pd, int Ph, int Pw, int Gd, int Gh, int Gw,
                        int stride, double* ws, float* dw, hipStream_t st) {
  const long nvox = (long)B * Pd * Ph * Pw;
  const long vpb = wgrad_vpb(nvox);
  const int nblk = (int)((nvox + vpb - 1) / vpb);
  if constexpr (A * BC <= 8)
    hipLaunchKernelGGL((conv3d_wgrad_taps_kernel<A, BC>), dim3(nblk, 3), dim3(kTrainBlock), 0, st, direct, gath, B,
                       Pd, Ph, Pw, Gd, Gh, Gw, stride, vpb, ws);
  else if constexpr (A * BC <= 16)
    hipLaunchKernelGGL((conv3d_wgrad_small_kernel<A, BC>), dim3(nblk, 27), dim3(kTrainBlock), 0, st, direct, gath, B,
                       Pd, Ph, Pw, Gd, Gh, Gw, stride, vpb, ws);
  else if constexpr (A >= 8 && BC >= 8)
    hipLaunchKernelGGL((conv3d_wgrad_tile_kernel<A, BC>), xcd_range_tap_grid(27, nblk), dim3(kTrainBlock), 0, st, direct,
                       gath, B, Pd, Ph, Pw, Gd, Gh, Gw, stride, vpb, nblk, ws);
  else
    hipLaunchKernelGGL((conv3d_wgrad_kernel<A, BC>), dim3(nblk, 27), dim3(kTrainBlock), 0, st, direct, gath, B, Pd,
                       Ph, Pw, Gd, Gh, Gw, stride, vpb, ws);
  TMVS_CHECK_LAUNCH();
  const long n = 27L * A * BC;
  hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)((n + 31) / 32)), dim3(kTrainBlock), 0,
                     st, ws, nblk, n, dw);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

static bool valid_ch(int c) { return c == 1 || c == 8 || c == 16 || c == 32 || c == 64; }

static long bn_vpb(long nvox) {
  long vpb = 1024;
  while ((nvox + vpb - 1) / vpb > 4096) vpb *= 2;
  return vpb;
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_conv3d_generic(const float* x, int batch, int cin, int d_in, int h_in, int w_in, const float* w,
                                   int cout, int d_out, int h_out, int w_out, int stride, int flags, float* y,
                                   void* stream) {
  const int transposed = (flags & TMVS_CONV_TRANSPOSED) ? 1 : 0, accumulate = (flags & TMVS_CONV_ACCUMULATE) ? 1 : 0;
  if (!x || !w || !y || batch <= 0 || d_in <= 0 || h_in <= 0 || w_in <= 0 || d_out <= 0 || h_out <= 0 || w_out <= 0)
    return TMVS_ERR_ARG;
  if (!valid_ch(cin) || !valid_ch(cout) || (stride != 1 && stride != 2)) return TMVS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
#define TMVS_GEN(CI, CB) \
  return launch_generic<CI, CB>(x, w, cout, batch, d_in, h_in, w_in, d_out, h_out, w_out, stride, transposed, \
                                accumulate, y, st)
  if (cout == 1) {
    switch (cin) {
      case 1: TMVS_GEN(1, 1);
      case 8: TMVS_GEN(8, 1);
      case 16: TMVS_GEN(16, 1);
      case 32: TMVS_GEN(32, 1);
      case 64: TMVS_GEN(64, 1);
    }
  } else if (cin == 64) {
    TMVS_GEN(64, 4);
  } else {
    switch (cin) {
      case 1: TMVS_GEN(1, 8);
      case 8: TMVS_GEN(8, 8);
      case 16: TMVS_GEN(16, 8);
      case 32: TMVS_GEN(32, 8);
    }
  }
#undef TMVS_GEN
  return TMVS_ERR_SHAPE;
}

extern "C" size_t tmvs_conv3d_wgrad_workspace(int batch, int d, int h, int w, int a_ch, int b_ch) {
  const long nvox = (long)batch * d * h * w;
  const long vpb = wgrad_vpb(nvox);
  return (size_t)((nvox + vpb - 1) / vpb) * 27 * a_ch * b_ch * sizeof(double);
}

extern "C" int tmvs_conv3d_wgrad(const float* direct, int a_ch, int batch, int pd, int ph, int pw, const float* gathered,
                                 int b_ch, int gd, int gh, int gw, int stride, void* workspace, size_t workspace_bytes,
                                 float* dw, void* stream) {
  if (!direct || !gathered || !workspace || !dw || batch <= 0 || pd <= 0 || ph <= 0 || pw <= 0 || gd <= 0 ||
      gh <= 0 || gw <= 0)
    return TMVS_ERR_ARG;
  if (stride != 1 && stride != 2) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_conv3d_wgrad_workspace(batch, pd, ph, pw, a_ch, b_ch)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  double* ws = (double*)workspace;
#define TMVS_WG(AA, BB)                                                                                             \
  if (a_ch == AA && b_ch == BB)                                                                                     \
    return launch_wgrad<AA, BB>(direct, gathered, batch, pd, ph, pw, gd, gh, gw, stride, ws, dw, st);
  // (direct, gathered) channel pairs of CostRegNet's layers: conv (dz, x) and deconv (x, dz)
  TMVS_WG(8, 1) TMVS_WG(16, 8) TMVS_WG(16, 16) TMVS_WG(32, 16) TMVS_WG(32, 32) TMVS_WG(64, 32) TMVS_WG(64, 64)
  TMVS_WG(1, 8) TMVS_WG(8, 16) TMVS_WG(16, 32) TMVS_WG(32, 64) TMVS_WG(8, 8)
#undef TMVS_WG
  return TMVS_ERR_SHAPE;
}

static size_t bn_group_ws(long nvox, int channels) {
  const long vpb = bn_vpb(nvox);
  return (size_t)((nvox + vpb - 1) / vpb) * 2 * channels * sizeof(double) + 2 * channels * sizeof(double);
}

extern "C" size_t tmvs_bn_train_workspace(long nvox, int channels) { return bn_group_ws(nvox, channels); }
extern "C" size_t tmvs_bn_train_workspace_grouped(int groups, long nvox, int channels) {
  return groups > 0 ? (size_t)groups * bn_group_ws(nvox, channels) : 0;
}

// workspace: [groups][nblk][2][C] partials, then [groups][2][C] sums
extern "C" int tmvs_bn_stats_grouped(const float* z, int groups, long nvox, int channels, void* workspace,
                                     size_t workspace_bytes, float* mean, float* var, void* stream) {
  if (!z || !workspace || !mean || !var || nvox <= 0 || groups <= 0) return TMVS_ERR_ARG;
  if (channels <= 0 || kTrainBlock % channels) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_bn_train_workspace_grouped(groups, nvox, channels)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const long vpb = bn_vpb(nvox);
  const int nblk = (int)((nvox + vpb - 1) / vpb);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(nblk, groups), dim3(kTrainBlock), 0, st, z, nvox, channels, vpb,
                     part);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_sums_stats_kernel, dim3(channels, groups), dim3(kTrainBlock), 0, st, (const double*)part,
                     nblk, channels, nvox, mean, var);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_bn_stats(const float* z, long nvox, int channels, void* workspace, size_t workspace_bytes,
                             float* mean, float* var, void* stream) {
  return tmvs_bn_stats_grouped(z, 1, nvox, channels, workspace, workspace_bytes, mean, var, stream);
}

extern "C" int tmvs_bn_relu_train_grouped(const float* z, int groups, long nvox, int channels, const float* mean,
                                          const float* var, const float* gamma, const float* beta, float eps,
                                          const float* skip, float* out, void* stream) {
  if (!z || !mean || !var || !gamma || !beta || !out || nvox <= 0 || channels <= 0 || groups <= 0)
    return TMVS_ERR_ARG;
  const long per = nvox * channels, n = per * groups;
  if (TMVS_BN_VEC4 && channels % 4 == 0 && aligned16(z) && aligned16(out) && (!skip || aligned16(skip))) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(bn_relu_apply4_kernel, dim3((unsigned)((n4 + kTrainBlock - 1) / kTrainBlock)), dim3(kTrainBlock),
                       0, (hipStream_t)stream, (const float4*)z, n4, per, channels, mean, var, gamma, beta, eps,
                       (const float4*)skip, (float4*)out);
  } else {
    hipLaunchKernelGGL(bn_relu_apply_kernel, dim3((unsigned)((n + kTrainBlock - 1) / kTrainBlock)), dim3(kTrainBlock),
                       0, (hipStream_t)stream, z, n, per, channels, mean, var, gamma, beta, eps, skip, out);
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_bn_relu_train(const float* z, long nvox, int channels, const float* mean, const float* var,
                                  const float* gamma, const float* beta, float eps, const float* skip, float* out,
                                  void* stream) {
  return tmvs_bn_relu_train_grouped(z, 1, nvox, channels, mean, var, gamma, beta, eps, skip, out, stream);
}

extern "C" int tmvs_bn_relu_backward_grouped(const float* dy, const float* z, int groups, long nvox, int channels,
                                             const float* mean, const float* var, const float* gamma,
                                             const float* beta, float eps, void* workspace, size_t workspace_bytes,
                                             float* dz, float* dgamma, float* dbeta, void* stream) {
  if (!dy || !z || !mean || !var || !gamma || !beta || !workspace || !dz || !dgamma || !dbeta || nvox <= 0 ||
      groups <= 0)
    return TMVS_ERR_ARG;
  if (channels <= 0 || kTrainBlock % channels) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_bn_train_workspace_grouped(groups, nvox, channels)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const long vpb = bn_vpb(nvox);
  const int nblk = (int)((nvox + vpb - 1) / vpb);
  double* part = (double*)workspace;
  double* sums = part + (size_t)groups * nblk * 2 * channels;
  hipLaunchKernelGGL(bn_relu_bwd_partial_kernel, dim3(nblk, groups), dim3(kTrainBlock), 0, st, dy, z, nvox, channels,
                     mean, var, gamma, beta, eps, vpb, part);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_double_partials_kernel, dim3(2 * channels, groups), dim3(kTrainBlock), 0, st,
                     (const double*)part, nblk, 2 * channels, sums);
  TMVS_CHECK_LAUNCH();
  const long n = nvox * channels * groups;
  if (TMVS_BN_VEC4 && channels % 4 == 0 && aligned16(dy) && aligned16(z) && aligned16(dz)) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(bn_relu_bwd_apply4_kernel, dim3((unsigned)((n4 + kTrainBlock - 1) / kTrainBlock)),
                       dim3(kTrainBlock), 0, st, (const float4*)dy, (const float4*)z, n4, channels, nvox, mean, var,
                       gamma, beta, eps, (const double*)sums, groups, dgamma, dbeta, (float4*)dz);
  } else {
    hipLaunchKernelGGL(bn_relu_bwd_apply_kernel, dim3((unsigned)((n + kTrainBlock - 1) / kTrainBlock)),
                       dim3(kTrainBlock), 0, st, dy, z, n, channels, nvox, mean, var, gamma, beta, eps,
                       (const double*)sums, groups, dgamma, dbeta, dz);
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_bn_relu_backward(const float* dy, const float* z, long nvox, int channels, const float* mean,
                                     const float* var, const float* gamma, const float* beta, float eps,
                                     void* workspace, size_t workspace_bytes, float* dz, float* dgamma, float* dbeta,
                                     void* stream) {
  return tmvs_bn_relu_backward_grouped(dy, z, 1, nvox, channels, mean, var, gamma, beta, eps, workspace,
                                       workspace_bytes, dz, dgamma, dbeta, stream);
}
