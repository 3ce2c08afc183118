// FeatureNet heads (models/module.py:362-395): the modulated deformable convolution DCNv2
// (models/dcn.py:66-80 -> torchvision.ops.deform_conv2d, torchvision 0.10.1) with the head's
// bias / BatchNorm / ReLU fused into the epilogue.
//
// deform_conv2d, stride 1, padding 1, dilation 1, one offset group, 3x3 taps k = 3i + j:
//   (py, px) = (y + i - 1 + om[2k], x + j - 1 + om[2k+1]),   mask_k = sigmoid(om[18 + k])
//   inside   = py > -1 && py < H && px > -1 && px < W; corners outside the image read 0
//   val_c    = ((hy*hx*v00 + hy*lx*v01) + ly*hx*v10) + ly*lx*v11          (l* = frac, h* = 1 - l*)
//   out[co]  = Σ_{k,c} W[co][c][k] * (mask_k * val_c) + bias[co]
// where om = conv_offset_mask(x) is the [27][H][W] output of the DCN's offset/mask conv, whose
// first 18 channels ARE cat(o1, o2) (models/dcn.py:75-77): channel 2k = dy_k, 2k+1 = dx_k.
//
// Implicit GEMM on fp32 MFMA (v_mfma_f32_16x16x4f32, exact fp32 products): M = 16 output
// channels, N = 16 pixels, K = 9 taps x 32 input channels. The B operand is produced in registers
// by the bilinear sampler itself: lane (j = lane/16, n = lane%16) samples pixel n's tap and holds
// input channels 8j .. 8j+7 -- two 16-byte loads per corner from the NHWC input -- and k-step s of
// the tap feeds channel 8j + s (the weights are packed in that K order). A wave owns 4 N-tiles
// (64 pixels); the A fragments (all taps) sit in LDS.
#include "common.h"

namespace tmvs {

namespace dcn {
constexpr int CI = 32;  // input channels (FeatureNet heads: 4 * base_channels)
constexpr int NT = 4;   // 16-pixel N-tiles per wave
}  // namespace dcn

template <int CO>
__global__ __launch_bounds__(256) void dcn_kernel(const float* __restrict__ x, const float* __restrict__ om,
                                                  const float* __restrict__ wpk, const float* __restrict__ bias,
                                                  const float* __restrict__ alpha, const float* __restrict__ shift,
                                                  int relu, int H, int W, float* __restrict__ out,
                                                  float* __restrict__ out_nhwc) {
  constexpr int MT = (CO + 15) / 16;
  constexpr int NA = 9 * 8 * MT * 64;
  __shared__ float wl[NA];  // A fragments [tap][s][mt][lane]
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < NA; i += 256) wl[i] = wpk[i];
  __syncthreads();
  const int HW = H * W, b = blockIdx.y;
  const int j = lane >> 4, n = lane & 15;
  const int base = (blockIdx.x * 4 + (tid >> 6)) * (16 * dcn::NT);
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)b * HW * dcn::CI, (unsigned)HW * dcn::CI * 4);
  const float* omb = om + (size_t)b * 27 * HW;
  int pix[dcn::NT], yy[dcn::NT], xx[dcn::NT];
#pragma unroll
  for (int t = 0; t < dcn::NT; ++t) {
    pix[t] = min(base + 16 * t + n, HW - 1);
    yy[t] = pix[t] / W;
    xx[t] = pix[t] - yy[t] * W;
  }
  floatx4_t acc[dcn::NT][MT];
#pragma unroll
  for (int t = 0; t < dcn::NT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = floatx4_t{0.f, 0.f, 0.f, 0.f};
  const float fH = (float)H, fW = (float)W;
#pragma unroll 1
  for (int k = 0; k < 9; ++k) {
    const int ki = k / 3, kj = k - 3 * ki;
    float col[dcn::NT][8];
#pragma unroll
    for (int t = 0; t < dcn::NT; ++t) {
      const float dy = omb[(size_t)(2 * k) * HW + pix[t]];
      const float dx = omb[(size_t)(2 * k + 1) * HW + pix[t]];
      const float ml = omb[(size_t)(18 + k) * HW + pix[t]];
      const float mk = 1.f / (1.f + expf(-ml));
      const float py = (float)(yy[t] + ki - 1) + dy;
      const float px = (float)(xx[t] + kj - 1) + dx;
      const bool inside = py > -1.f && py < fH && px > -1.f && px < fW;
      const float y0 = floorf(py), x0 = floorf(px);
      const float ly = py - y0, lx = px - x0;
      const float hy = 1.f - ly, hx = 1.f - lx;
      const int y0i = (int)fmaxf(fminf(y0, 32766.f), -2.f), x0i = (int)fmaxf(fminf(x0, 32766.f), -2.f);
      const float w4[4] = {hy * hx, hy * lx, ly * hx, ly * lx};
      floatx4_t v[4][2];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cy = y0i + (c >> 1), cx = x0i + (c & 1);
        const bool ok = inside && (unsigned)cy < (unsigned)H && (unsigned)cx < (unsigned)W;
        const unsigned o = ok ? ((unsigned)(cy * W + cx) * dcn::CI + 8u * j) * 4u : kOffOut;  // outside: reads 0
        v[c][0] = buf_load_f32x4(rx, o);
        v[c][1] = buf_load_f32x4(rx, o + 16u);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        float val = w4[0] * v[0][s >> 2][s & 3];
        val = val + w4[1] * v[1][s >> 2][s & 3];
        val = val + w4[2] * v[2][s >> 2][s & 3];
        val = val + w4[3] * v[3][s >> 2][s & 3];
        col[t][s] = mk * val;
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      float a[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) a[m] = wl[((k * 8 + s) * MT + m) * 64 + lane];
#pragma unroll
      for (int t = 0; t < dcn::NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[t][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], col[t][s], acc[t][m], 0, 0, 0);
    }
  }
  // D fragment: lane (j, n) holds output channels 16m + 4j .. +3 of pixel n of each N-tile
#pragma unroll
  for (int t = 0; t < dcn::NT; ++t) {
    const int p = base + 16 * t + n;
    if (p >= HW) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int co0 = 16 * m + 4 * j;
      if (co0 >= CO) continue;
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[t][m][i] + bias[co0 + i];
        if (alpha) v = fmaf(v, alpha[co0 + i], shift[co0 + i]);
        if (relu) v = fmaxf(v, 0.f);
        r[i] = v;
        out[((size_t)b * CO + co0 + i) * HW + p] = v;
      }
      if (out_nhwc)
        *reinterpret_cast<float4*>(out_nhwc + ((size_t)b * HW + p) * CO + co0) = make_float4(r[0], r[1], r[2], r[3]);
    }
  }
}

}  // namespace tmvs

using namespace tmvs;

extern "C" size_t tmvs_deform_conv2d_packed_floats(int cout) { return (size_t)9 * 8 * ((cout + 15) / 16) * 64; }

extern "C" int tmvs_deform_conv2d_pack(const float* weight, int cout, int cin, float* packed) {
  if (!weight || !packed || cin != dcn::CI || (cout != 8 && cout != 16 && cout != 32)) return TMVS_ERR_ARG;
  const int mt_n = (cout + 15) / 16;
  for (int k = 0; k < 9; ++k)
    for (int s = 0; s < 8; ++s)
      for (int mt = 0; mt < mt_n; ++mt)
        for (int l = 0; l < 64; ++l) {
          const int co = 16 * mt + (l & 15), ci = 8 * (l >> 4) + s;
          packed[((k * 8 + s) * mt_n + mt) * 64 + l] = co < cout ? weight[((size_t)co * cin + ci) * 9 + k] : 0.f;
        }
  return TMVS_OK;
}

extern "C" int tmvs_deform_conv2d(const float* x_nhwc, const float* offset_mask, const float* w_packed,
                                  const float* bias, const float* bn_alpha, const float* bn_shift, int relu,
                                  int batch, int cin, int cout, int height, int width, float* out,
                                  float* out_nhwc, void* stream) {
  if (!x_nhwc || !offset_mask || !w_packed || !bias || !out || batch <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  if ((bn_alpha == nullptr) != (bn_shift == nullptr)) return TMVS_ERR_ARG;
  if (cin != dcn::CI || (cout != 8 && cout != 16 && cout != 32)) return TMVS_ERR_SHAPE;
  if ((long long)height * width * cin * 4 >= (1LL << 31) || height > 32766 || width > 32766) return TMVS_ERR_SHAPE;
  const int HW = height * width;
  const dim3 grid((HW + 4 * 16 * dcn::NT - 1) / (4 * 16 * dcn::NT), batch);
  hipStream_t st = (hipStream_t)stream;
#define TMVS_DCN(CO)                                                                                             \
  hipLaunchKernelGGL(dcn_kernel<CO>, grid, dim3(256), 0, st, x_nhwc, offset_mask, w_packed, bias, bn_alpha, \
                     bn_shift, relu, height, width, out, out_nhwc)
  if (cout == 32)
    TMVS_DCN(32);
  else if (cout == 16)
    TMVS_DCN(16);
  else
    TMVS_DCN(8);
#undef TMVS_DCN
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
