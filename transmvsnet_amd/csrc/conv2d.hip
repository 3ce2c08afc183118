// FeatureNet's plain convolution blocks, models/module.py:24-61 (Conv2d(bias=False) -> eval BatchNorm
// -> ReLU), as used by the trunk (:349-360: 3->8 3x3, 8->8 3x3, 8->16 5x5/2, 16->16 3x3, 16->32 5x5/2,
// 32->32 3x3) and the stage-1 head's 1x1 (:362). NHWC fp32 in and out (the first layer reads the
// NCHW image directly), BN + ReLU fused into the epilogue.
//
// Implicit GEMM on fp32 MFMA (v_mfma_f32_16x16x4f32): M = 16 output channels (x MT tiles), N = 16
// output pixels of one row, K = taps x channels. The K axis is walked in "k-blocks" of 4 k-steps:
// in k-block b, lane group j owns the (tap, 4-channel chunk) pair idx = 4b + j of the flattened
// list [tap][chunk] (G = CIP/4 chunks per pixel) and feeds its 4 channels to the 4 k-steps, so each
// k-block is ONE ds_read_b128 per lane and 4 x MT MFMAs; the weights are packed in that order.
//
// Work unit = (image, 8 output rows, 16 output columns): wave w of the 512-thread block owns output
// row 8*band + w. Per unit the block stages the input window (rows 7S+K, columns 15S+K, zeros
// outside the image) in LDS; the next unit's window is loaded into registers during this unit's
// MFMAs (persistent grid, XCD-contiguous unit ranges) -- the DCN kernels' scheme (featurenet.hip).
#include "common.h"

#include <algorithm>

namespace tmvs {

template <int CI, int CO, int K, int S, bool NCHW>
struct Conv2dCfg {
  static constexpr int CIP = CI < 4 ? 4 : CI;  // channels per pixel in LDS (3 -> 4, zero pad)
  static constexpr int G = CIP / 4;            // 16-byte chunks per pixel
  static constexpr int MT = (CO + 15) / 16;
  static constexpr int NIDX = K * K * G;       // (tap, chunk) pairs
  static constexpr int NB = (NIDX + 3) / 4;    // k-blocks
  static constexpr int WR = 7 * S + K, WC = 15 * S + K, WP = WR * WC;
  static constexpr int WIN4 = WP * G;
  static constexpr int STAGE = (WIN4 + 511) / 512;
  static constexpr int PAD = K / 2;
  static constexpr int SH = G == 8 ? 0 : G == 4 ? 2 : 3;  // chunk swizzle: c ^ ((P >> SH) & (G - 1))
  static constexpr int NA4 = NB * MT * 64;
};

template <int G, int SH>
__device__ __forceinline__ int c2_slot(int P, int c) {
  return G == 1 ? P : P * G + (c ^ ((P >> SH) & (G - 1)));
}

#ifndef TMVS_C2D_ABL
#define TMVS_C2D_ABL 0
#endif
template <int CI, int CO, int K, int S, bool NCHW>
__global__ __launch_bounds__(512) void conv2d_bn_relu_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ shift, int relu, int B, int H,
                                                             int W, int Ho, int Wo, float* __restrict__ out) {
  using C = Conv2dCfg<CI, CO, K, S, NCHW>;
  __shared__ floatx4_t wl[C::NA4];
  __shared__ floatx4_t win[C::WIN4];
  // BN alpha / shift in LDS for the epilogue (from global there, each was a serialised L2 round trip per unit)
  __shared__ __attribute__((aligned(16))) float cst[2][C::MT * 16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < C::NA4; i += 512) wl[i] = reinterpret_cast<const floatx4_t*>(wpk)[i];
  if (tid < C::MT * 16) {
    cst[0][tid] = alpha && tid < CO ? alpha[tid] : 1.f;
    cst[1][tid] = alpha && tid < CO ? shift[tid] : 0.f;
  }
  const int nbx = (Wo + 15) / 16, nby = (Ho + 7) / 8, nunits = B * nby * nbx;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int u_begin = (int)((long long)nunits * bid / gridDim.x);
  const int u_end = (int)((long long)nunits * (bid + 1) / gridDim.x);
  const int j = lane >> 4, n = lane & 15;
  const size_t img = (size_t)H * W * (NCHW ? CI : C::CIP);
  floatx4_t stg[C::STAGE];
  auto fetch = [&](int u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    const int iy0 = band * 8 * S - C::PAD, ix0 = xs * 16 * S - C::PAD;
    const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + b * img, (unsigned)(img * 4));
#pragma unroll
    for (int i = 0; i < C::STAGE; ++i) {
      const int idx = min(tid + 512 * i, C::WIN4 - 1), pix = idx / C::G, ch = idx - pix * C::G;
      const int r = pix / C::WC, c = pix - r * C::WC;
      const int gy = iy0 + r, gx = ix0 + c;
      const bool ok = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      if (NCHW) {  // CI = 3 planes -> (c0, c1, c2, 0)
        const unsigned o = ok ? (unsigned)(gy * W + gx) * 4u : kOffOut;
        const unsigned plane = (unsigned)(H * W) * 4u;
        stg[i] = floatx4_t{buf_load_f32(rx, o), buf_load_f32(rx, ok ? o + plane : kOffOut),
                           buf_load_f32(rx, ok ? o + 2 * plane : kOffOut), 0.f};
      } else {
        stg[i] = buf_load_f32x4(rx, ok ? ((unsigned)(gy * W + gx) * C::CIP + 4u * ch) * 4u : kOffOut);
      }
    }
  };
  if (u_begin < u_end) fetch(u_begin);
  for (int u = u_begin; u < u_end; ++u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    __syncthreads();  // previous unit's window reads done (first time: weights staged)
#pragma unroll
    for (int i = 0; i < C::STAGE; ++i) {
      const int idx = tid + 512 * i;
      if (idx < C::WIN4) {
        const int pix = idx / C::G;
        win[c2_slot<C::G, C::SH>(pix, idx - pix * C::G)] = stg[i];
      }
    }
    __syncthreads();
    if (u + 1 < u_end) fetch(u + 1);
    const int row = band * 8 + wv, x0 = xs * 16, nvalid = min(16, Wo - x0);
    if (row >= Ho) continue;
    floatx4_t acc[C::MT];
#pragma unroll
    for (int m = 0; m < C::MT; ++m) acc[m] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    // k-block kb + 1's fragments are read during kb's MFMAs
    floatx4_t fb[2], fa[2][C::MT];
    auto frag = [&](int kb, int bf) {
      const int idx = min(4 * kb + j, C::NIDX - 1);  // padded pairs carry zero weights
      const int tap = idx / C::G, ch = idx - tap * C::G, ki = tap / K, kj = tap - ki * K;
      const int P = (wv * S + ki) * C::WC + n * S + kj;
      fb[bf] = win[c2_slot<C::G, C::SH>(P, ch)];
#pragma unroll
      for (int m = 0; m < C::MT; ++m) fa[bf][m] = wl[(kb * C::MT + m) * 64 + lane];
    };
    frag(0, 0);
#pragma unroll
    for (int kb = 0; kb < C::NB; ++kb) {
      if (kb + 1 < C::NB) frag(kb + 1, (kb + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const floatx4_t bv = fb[kb & 1];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int m = 0; m < C::MT; ++m) {
          if (TMVS_C2D_ABL) {  // timing ablation (wrong outputs): no MFMAs
            acc[m][0] += fa[kb & 1][m][e] * bv[e];
            continue;
          }
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[kb & 1][m][e], bv[e], acc[m], 0, 0, 0);
        }
    }
    if (n < nvalid) {
      float* o = out + (((size_t)b * Ho + row) * Wo + x0 + n) * CO;
#pragma unroll
      for (int m = 0; m < C::MT; ++m) {
        const int co0 = 16 * m + 4 * j;
        if (co0 >= CO) continue;
        const floatx4_t ca = *reinterpret_cast<const floatx4_t*>(&cst[0][co0]);
        const floatx4_t cs = *reinterpret_cast<const floatx4_t*>(&cst[1][co0]);
        float r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float y = acc[m][i];
          if (alpha) y = fmaf(y, ca[i], cs[i]);
          if (relu) y = fmaxf(y, 0.f);
          r[i] = y;
        }
        *reinterpret_cast<float4*>(o + co0) = make_float4(r[0], r[1], r[2], r[3]);
      }
    }
  }
}

template <int CI, int CO, int K, int S, bool NCHW>
static int conv2d_launch(const float* x, const float* w, const float* alpha, const float* shift, int relu, int B,
                         int H, int W, float* out, hipStream_t st) {
  static int grid = 0;
  if (!grid) {
    int dev = 0, ncu = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TMVS_ERR_HIP;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv2d_bn_relu_kernel<CI, CO, K, S, NCHW>, 512, 0);
    grid = std::max(1, ncu * std::max(occ, 1));
  }
  const int pad = K / 2, Ho = (H + 2 * pad - K) / S + 1, Wo = (W + 2 * pad - K) / S + 1;
  const long long nunits = (long long)B * ((Ho + 7) / 8) * ((Wo + 15) / 16);
  const int nblk = (int)std::min<long long>(grid, nunits);
  hipLaunchKernelGGL((conv2d_bn_relu_kernel<CI, CO, K, S, NCHW>), dim3(nblk), dim3(512), 0, st, x, w, alpha, shift,
                     relu, B, H, W, Ho, Wo, out);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// the FeatureNet layer shapes: (cin, cout, k, stride); cin = 3 reads the NCHW image
static int conv2d_dispatch(int cin, int cout, int k, int s, const float* x, const float* w, const float* a,
                           const float* sh, int relu, int B, int H, int W, float* out, hipStream_t st) {
#define TMVS_C2D(CI, CO, K, S, NC) \
  if (cin == CI && cout == CO && k == K && s == S) return conv2d_launch<CI, CO, K, S, NC>(x, w, a, sh, relu, B, H, W, out, st)
  TMVS_C2D(3, 8, 3, 1, true);
  TMVS_C2D(8, 8, 3, 1, false);
  TMVS_C2D(8, 16, 5, 2, false);
  TMVS_C2D(16, 16, 3, 1, false);
  TMVS_C2D(16, 32, 5, 2, false);
  TMVS_C2D(32, 32, 3, 1, false);
  TMVS_C2D(32, 32, 1, 1, false);
#undef TMVS_C2D
  return TMVS_ERR_SHAPE;
}

static bool conv2d_supported(int cin, int cout, int k, int s) {
  return (cin == 3 && cout == 8 && k == 3 && s == 1) || (cin == 8 && cout == 8 && k == 3 && s == 1) ||
         (cin == 8 && cout == 16 && k == 5 && s == 2) || (cin == 16 && cout == 16 && k == 3 && s == 1) ||
         (cin == 16 && cout == 32 && k == 5 && s == 2) || (cin == 32 && cout == 32 && k == 3 && s == 1) ||
         (cin == 32 && cout == 32 && k == 1 && s == 1);
}

}  // namespace tmvs

using namespace tmvs;

extern "C" size_t tmvs_conv2d_packed_floats(int cout, int cin, int k) {
  const int cip = cin < 4 ? 4 : cin, g = cip / 4, nb = (k * k * g + 3) / 4, mt = (cout + 15) / 16;
  return (size_t)nb * mt * 64 * 4;
}

// A fragments [k-block b][m-tile][lane l][e]: lane l = (row r = l & 15, group j = l >> 4) holds
// W[co = 16m + r][c = 4 chunk + e][ki][kj] for the (tap, chunk) pair idx = 4b + j (tap = ki*k + kj),
// zero for co >= cout, c >= cin or idx past the last pair.
extern "C" int tmvs_conv2d_pack(const float* weight, int cout, int cin, int k, float* packed) {
  if (!weight || !packed || cout <= 0 || cin <= 0 || (k != 1 && k != 3 && k != 5)) return TMVS_ERR_ARG;
  const int cip = cin < 4 ? 4 : cin, g = cip / 4, nidx = k * k * g, nb = (nidx + 3) / 4, mt = (cout + 15) / 16;
  if (cip % 4) return TMVS_ERR_SHAPE;
  for (int b = 0; b < nb; ++b)
    for (int m = 0; m < mt; ++m)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) {
          const int idx = 4 * b + (l >> 4), co = 16 * m + (l & 15);
          float v = 0.f;
          if (idx < nidx && co < cout) {
            const int tap = idx / g, c = 4 * (idx % g) + e;
            if (c < cin) v = weight[(((size_t)co * cin + c) * k + tap / k) * k + tap % k];
          }
          packed[(((size_t)b * mt + m) * 64 + l) * 4 + e] = v;
        }
  return TMVS_OK;
}

extern "C" int tmvs_conv2d_bn_relu(const float* x, int batch, int cin, int height, int width, const float* w_packed,
                                   int cout, int k, int stride, const float* bn_alpha, const float* bn_shift, int relu,
                                   float* out_nhwc, void* stream) {
  if (!x || !w_packed || !out_nhwc || batch <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if ((bn_alpha == nullptr) != (bn_shift == nullptr)) return TMVS_ERR_ARG;
  if (!conv2d_supported(cin, cout, k, stride)) return TMVS_ERR_SHAPE;
  if ((long long)height * width * (cin < 4 ? 4 : cin) * 4 >= (1LL << 31)) return TMVS_ERR_SHAPE;
  return conv2d_dispatch(cin, cout, k, stride, x, w_packed, bn_alpha, bn_shift, relu, batch, height, width, out_nhwc,
                         (hipStream_t)stream);
}
