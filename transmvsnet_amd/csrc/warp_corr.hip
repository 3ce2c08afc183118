// Fused cost-volume build for one cascade stage (DepthNet steps 1-2,
// reference models/TransMVSNet.py:58-93 and homo_warping models/module.py:284-322).
//
// A pixel is owned by C/4 adjacent lanes (see warp_corr_kernel); per source view they project
// the pixel's depth planes into the view, bilinearly sample the channels-last source features
// (one contiguous C*4-byte row per tap per lane group) and form the single-group correlation
// against the reference features held in registers; the warped [C,D,H,W] volume never exists.
//
// fp32 op order follows the reference's PyTorch-CPU kernels (DESIGN.md "Numerics"):
//   rot·(x,y,1)   : fmaf(r1, y, r0*x) + r2            (bmm, FMA chain)
//   X = rot_xyz*d + t ; px = X/Z ; xn = px/((W-1)/2) - 1 ; z < 1e-6 -> xn = yn = -99
//   ix = (xn + 1) * ((W-1)/2)                          (grid_sample, align_corners=True)
//   v  = fmaf(se_v,se, fmaf(sw_v,sw, fmaf(ne_v,ne, nw_v*nw)))  (zeros padding)
//   sim = (Σ_c v_c*ref_c) / C ; sim_sum += sim*w ; w_sum = 1e-5 + Σ w ; sim_sum / w_sum
// (the channel sum: serial within each lane's 4 channels, then a fixed xor tree over lanes)
#include "common.h"

namespace tmvs {

struct WarpArgs {
  float proj[TMVS_MAX_VIEWS][12];
  float pw[TMVS_PW_NPARAMS];
};

__device__ __forceinline__ float pixelwise_logit(float s, const float* __restrict__ pw) {
  // PixelwiseNet (TransMVSNet.py:20-26): 1x1x1 convs 1->16 (BN,ReLU) ->8 (BN,ReLU) ->1 (+bias)
  const float* w0 = pw;
  const float* a0 = pw + 16;
  const float* s0 = pw + 32;
  const float* w1 = pw + 48;
  const float* a1 = pw + 176;
  const float* s1 = pw + 184;
  const float* w2 = pw + 192;
  const float b2 = pw[200];
  float h0[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) h0[o] = relu(fmaf(w0[o] * s, a0[o], s0[o]));
  float out = 0.f;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    float acc = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o) acc = fmaf(w1[p * 16 + o], h0[o], acc);
    out = fmaf(w2[p], relu(fmaf(acc, a1[p], s1[p])), out);
  }
  return out + b2;
}

// Lane layout: a pixel is served by LPS = C/4 adjacent lanes ("group"); lane k of the group
// owns channel quad k (4 channels, one 16-byte load per tap) and depth planes k, k+LPS, ...
// For every depth plane the group issues one 16-byte load per lane per tap, i.e. the C
// channels of a tap arrive as one contiguous row (C*4 bytes) per group: a wave-instruction
// touches 64/LPS rows instead of 64 scattered 16-byte pieces. Each lane projects only its own
// depth planes; the tap geometry (x0, y0, fractional x, fractional y) of plane j*LPS+t is
// broadcast from lane t with lane shuffles, and the channel dot product is reduced across the
// group with xor shuffles (channel order: 4-channel serial sums, then a fixed tree).
template <int C>
struct Tap {
  int x0, y0;
  float fx, fy;
};

__device__ __forceinline__ void project(const float rx, const float ry, const float rz, const float tx,
                                        const float ty, const float tz, const float dep, const float halfw,
                                        const float halfh, int& x0i, int& y0i, float& fx, float& fy) {
  const float X = rx * dep + tx;
  const float Y = ry * dep + ty;
  const float Z = rz * dep + tz;
  float xn = (X / Z) / halfw - 1.f;
  float yn = (Y / Z) / halfh - 1.f;
  if (Z < 1e-6f) {
    xn = -99.f;
    yn = -99.f;
  }
  const float ix = (xn + 1.f) * halfw;
  const float iy = (yn + 1.f) * halfh;
  const float x0 = floorf(ix), y0 = floorf(iy);
  fx = ix - x0;
  fy = iy - y0;
  // clamp far-away samples (all four taps outside) to a sentinel that stays outside
  x0i = (int)fminf(fmaxf(x0, -2.f), 65536.f);
  y0i = (int)fminf(fmaxf(y0, -2.f), 65536.f);
}

template <int C, int D, bool PW, bool PARTIAL>
__global__ __launch_bounds__(256) void warp_corr_kernel(
    const float* __restrict__ ref, const float* __restrict__ src, const float* __restrict__ hyp,
    const float* __restrict__ vw_in, float* __restrict__ sim_out, float* __restrict__ wsum_out,
    float* __restrict__ vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total, WarpArgs args) {
  constexpr int LPS = C / 4;          // lanes per pixel
  constexpr int SPW = 64 / LPS;       // pixels per wave
  constexpr int PIX = 4 * SPW;        // pixels per block
  constexpr int DPT = D / LPS;        // depth planes owned per lane
  static_assert(D % LPS == 0, "D must be a multiple of C/4");
  const int HW = H * W;
  const int nblk = (HW + PIX - 1) / PIX;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int lane = threadIdx.x & 63;
  const int k = lane % LPS;
  const int gbase = lane - k;
  int p = tile * PIX + (threadIdx.x >> 6) * SPW + lane / LPS;
  const bool active = p < HW;
  if (!active) p = HW - 1;
  const int py = p / W, px = p - py * W;
  const float fxp = (float)px, fyp = (float)py;

  const float4 r4 = *reinterpret_cast<const float4*>(ref + (size_t)p * C + 4 * k);
  float dep[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) dep[j] = hyp[(size_t)(j * LPS + k) * HW + p];
  const float halfw = (float)(W - 1) / 2.f;
  const float halfh = (float)(H - 1) / 2.f;
  float ssum[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) ssum[j] = 0.f;
  float wsum = PARTIAL ? 0.f : 1e-5f;

  for (int v = 0; v < V; ++v) {
    const float* R = args.proj[v];
    const float rx = fmaf(R[1], fyp, R[0] * fxp) + R[2];
    const float ry = fmaf(R[5], fyp, R[4] * fxp) + R[6];
    const float rz = fmaf(R[9], fyp, R[8] * fxp) + R[10];
    const float* __restrict__ sv = src + (size_t)v * HW * C + 4 * k;
    float sim[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      int mx0, my0;
      float mfx, mfy;
      project(rx, ry, rz, R[3], R[7], R[11], dep[j], halfw, halfh, mx0, my0, mfx, mfy);
#pragma unroll
      for (int t = 0; t < LPS; ++t) {
        int x0 = mx0, y0 = my0;
        float we = mfx, n = mfy;
        if constexpr (LPS > 1) {
          x0 = __shfl(mx0, gbase + t, 64);
          y0 = __shfl(my0, gbase + t, 64);
          we = __shfl(mfx, gbase + t, 64);
          n = __shfl(mfy, gbase + t, 64);
        }
        const float ea = 1.f - we, s = 1.f - n;
        const float wnw = s * ea, wne = s * we, wsw = n * ea, wse = n * we;
        const bool vx0 = x0 >= 0 && x0 <= W - 1, vx1 = x0 + 1 >= 0 && x0 + 1 <= W - 1;
        const bool vy0 = y0 >= 0 && y0 <= H - 1, vy1 = y0 + 1 >= 0 && y0 + 1 <= H - 1;
        const int xa = vx0 ? x0 : 0, xb = vx1 ? x0 + 1 : 0;
        const int ya = vy0 ? y0 : 0, yb = vy1 ? y0 + 1 : 0;
        float4 a = *reinterpret_cast<const float4*>(sv + ((size_t)ya * W + xa) * C);
        float4 b = *reinterpret_cast<const float4*>(sv + ((size_t)ya * W + xb) * C);
        float4 c = *reinterpret_cast<const float4*>(sv + ((size_t)yb * W + xa) * C);
        float4 d = *reinterpret_cast<const float4*>(sv + ((size_t)yb * W + xb) * C);
        if (!(vy0 && vx0)) a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!(vy0 && vx1)) b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!(vy1 && vx0)) c = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!(vy1 && vx1)) d = make_float4(0.f, 0.f, 0.f, 0.f);
        float acc = 0.f;
        acc = acc + fmaf(d.x, wse, fmaf(c.x, wsw, fmaf(b.x, wne, a.x * wnw))) * r4.x;
        acc = acc + fmaf(d.y, wse, fmaf(c.y, wsw, fmaf(b.y, wne, a.y * wnw))) * r4.y;
        acc = acc + fmaf(d.z, wse, fmaf(c.z, wsw, fmaf(b.z, wne, a.z * wnw))) * r4.z;
        acc = acc + fmaf(d.w, wse, fmaf(c.w, wsw, fmaf(b.w, wne, a.w * wnw))) * r4.w;
#pragma unroll
        for (int off = 1; off < LPS; off <<= 1) acc += __shfl_xor(acc, off, 64);
        if (k == t) sim[j] = acc / (float)C;
      }
    }
    float w;
    if constexpr (PW) {
      float wm = 0.f;  // sigmoid > 0: 0 is neutral for the max
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        const float lg = pixelwise_logit(sim[j], args.pw);
        wm = fmaxf(wm, 1.f / (1.f + expf(-lg)));
      }
#pragma unroll
      for (int off = 1; off < LPS; off <<= 1) wm = fmaxf(wm, __shfl_xor(wm, off, 64));
      w = wm;
      if (active && k == 0) vw_out[(size_t)(vw_offset + v) * HW + p] = w;
    } else {
      const int Ws = W >> vw_shift, Hs = H >> vw_shift;
      w = vw_in[(size_t)(vw_offset + v) * Hs * Ws + (py >> vw_shift) * Ws + (px >> vw_shift)];
    }
#pragma unroll
    for (int j = 0; j < DPT; ++j) ssum[j] = ssum[j] + sim[j] * w;
    wsum = wsum + w;
  }
  if (!active) return;
  if constexpr (PARTIAL) {
#pragma unroll
    for (int j = 0; j < DPT; ++j) sim_out[(size_t)(j * LPS + k) * HW + p] = ssum[j];
    if (k == 0) wsum_out[p] = wsum;
  } else {
#pragma unroll
    for (int j = 0; j < DPT; ++j) sim_out[(size_t)(j * LPS + k) * HW + p] = ssum[j] / wsum;
  }
}

__global__ void aggregate_finalize_kernel(float* __restrict__ sim, const float* __restrict__ wsum, int D, int HW) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  const float ws = 1e-5f + wsum[(size_t)blockIdx.y * HW + p];
  float* s = sim + (size_t)blockIdx.y * D * HW + p;
  for (int d = 0; d < D; ++d) s[(size_t)d * HW] = s[(size_t)d * HW] / ws;
}

// Materialising homo_warping for the reference seam: out [C][D][H][W] from NCHW src.
__global__ void homo_warping_kernel(const float* __restrict__ src, const float* __restrict__ hyp,
                                    float* __restrict__ out, int C, int D, int H, int W, WarpArgs args) {
  const int HW = H * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= D * HW) return;
  const int d = idx / HW, p = idx - d * HW;
  const int py = p / W, px = p - py * W;
  const float* R = args.proj[0];
  const float fx = (float)px, fy = (float)py;
  const float rx = fmaf(R[1], fy, R[0] * fx) + R[2];
  const float ry = fmaf(R[5], fy, R[4] * fx) + R[6];
  const float rz = fmaf(R[9], fy, R[8] * fx) + R[10];
  const float dep = hyp[idx];
  const float X = rx * dep + R[3], Y = ry * dep + R[7], Z = rz * dep + R[11];
  const float halfw = (float)(W - 1) / 2.f, halfh = (float)(H - 1) / 2.f;
  float xn = (X / Z) / halfw - 1.f, yn = (Y / Z) / halfh - 1.f;
  if (Z < 1e-6f) {
    xn = -99.f;
    yn = -99.f;
  }
  const float ix = (xn + 1.f) * halfw, iy = (yn + 1.f) * halfh;
  const float x0 = floorf(ix), y0 = floorf(iy);
  const float we = ix - x0, ea = 1.f - we, n = iy - y0, s = 1.f - n;
  const float wnw = s * ea, wne = s * we, wsw = n * ea, wse = n * we;
  const bool vx0 = x0 >= 0.f && x0 <= (float)(W - 1), vx1 = x0 + 1.f >= 0.f && x0 + 1.f <= (float)(W - 1);
  const bool vy0 = y0 >= 0.f && y0 <= (float)(H - 1), vy1 = y0 + 1.f >= 0.f && y0 + 1.f <= (float)(H - 1);
  const int xi0 = vx0 ? (int)x0 : 0, xi1 = vx1 ? (int)x0 + 1 : 0;
  const int yi0 = vy0 ? (int)y0 : 0, yi1 = vy1 ? (int)y0 + 1 : 0;
  for (int c = 0; c < C; ++c) {
    const float* sc = src + (size_t)c * HW;
    const float a = (vy0 && vx0) ? sc[yi0 * W + xi0] : 0.f;
    const float b = (vy0 && vx1) ? sc[yi0 * W + xi1] : 0.f;
    const float cc = (vy1 && vx0) ? sc[yi1 * W + xi0] : 0.f;
    const float dd = (vy1 && vx1) ? sc[yi1 * W + xi1] : 0.f;
    out[(size_t)c * D * HW + idx] = fmaf(dd, wse, fmaf(cc, wsw, fmaf(b, wne, a * wnw)));
  }
}

template <int C, int D, bool PW, bool PARTIAL>
static int launch_warp(const float* ref, const float* src, const float* hyp, const float* vw_in, float* sim,
                       float* wsum, float* vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total,
                       const WarpArgs& args, hipStream_t st) {
  constexpr int PIX = 4 * (64 / (C / 4));
  const int nblk = (H * W + PIX - 1) / PIX;
  hipLaunchKernelGGL((warp_corr_kernel<C, D, PW, PARTIAL>), dim3(nblk), dim3(256), 0, st, ref, src, hyp, vw_in, sim,
                     wsum, vw_out, V, H, W, vw_shift, vw_offset, vw_total, args);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int C, bool PW, bool PARTIAL>
static int dispatch_depth(int D, const float* ref, const float* src, const float* hyp, const float* vw_in, float* sim,
                          float* wsum, float* vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total,
                          const WarpArgs& a, hipStream_t st) {
#define TMVS_WARP_CASE(DD)                                                                                        \
  if (D == DD)                                                                                                    \
    return launch_warp<C, DD, PW, PARTIAL>(ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift, vw_offset, \
                                           vw_total, a, st);
  TMVS_WARP_CASE(48)
  TMVS_WARP_CASE(32)
  TMVS_WARP_CASE(16)
  TMVS_WARP_CASE(8)
  TMVS_WARP_CASE(64)
  TMVS_WARP_CASE(24)
#undef TMVS_WARP_CASE
  return TMVS_ERR_SHAPE;
}

template <int C>
static int dispatch_mode(bool pw, bool partial, int D, const float* ref, const float* src, const float* hyp,
                         const float* vw_in, float* sim, float* wsum, float* vw_out, int V, int H, int W, int vw_shift,
                         int vw_offset, int vw_total, const WarpArgs& a, hipStream_t st) {
  if (pw && partial)
    return dispatch_depth<C, true, true>(D, ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift, vw_offset,
                                         vw_total, a, st);
  if (pw)
    return dispatch_depth<C, true, false>(D, ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift, vw_offset,
                                          vw_total, a, st);
  if (partial)
    return dispatch_depth<C, false, true>(D, ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift, vw_offset,
                                          vw_total, a, st);
  return dispatch_depth<C, false, false>(D, ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift, vw_offset,
                                         vw_total, a, st);
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_warp_corr(const float* ref_fea, const float* src_fea, const float* proj, const float* hyp,
                              const float* view_w_in, int vw_shift, int vw_offset, int vw_total,
                              const float* pw_params, int batch, int n_src, int channels, int ndepth, int height,
                              int width, int flags, float* sim_out, float* wsum_out, float* view_w_out,
                              void* stream) {
  if (!ref_fea || !src_fea || !proj || !hyp || !sim_out) return TMVS_ERR_ARG;
  if (batch <= 0 || n_src <= 0 || n_src > TMVS_MAX_VIEWS || height <= 0 || width <= 0 || ndepth <= 0)
    return TMVS_ERR_ARG;
  const bool pw = view_w_in == nullptr;
  const bool partial = (flags & TMVS_WARP_PARTIAL) != 0;
  if (pw && (!pw_params || !view_w_out)) return TMVS_ERR_ARG;
  if (partial && !wsum_out) return TMVS_ERR_ARG;
  if (vw_offset < 0 || vw_offset + n_src > vw_total || vw_shift < 0) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const size_t HW = (size_t)height * width;
  for (int b = 0; b < batch; ++b) {
    WarpArgs a;
    for (int v = 0; v < n_src; ++v)
      for (int k = 0; k < 12; ++k) a.proj[v][k] = proj[((size_t)b * n_src + v) * 12 + k];
    if (pw)
      for (int k = 0; k < TMVS_PW_NPARAMS; ++k) a.pw[k] = pw_params[k];
    else
      for (int k = 0; k < TMVS_PW_NPARAMS; ++k) a.pw[k] = 0.f;
    const float* rb = ref_fea + (size_t)b * HW * channels;
    const float* sb = src_fea + (size_t)b * n_src * HW * channels;
    const float* hb = hyp + (size_t)b * ndepth * HW;
    const size_t hs = (size_t)(height >> vw_shift) * (width >> vw_shift);
    const float* vib = pw ? nullptr : view_w_in + (size_t)b * vw_total * hs;
    float* sob = sim_out + (size_t)b * ndepth * HW;
    float* wob = partial ? wsum_out + (size_t)b * HW : nullptr;
    float* vob = pw ? view_w_out + (size_t)b * vw_total * HW : nullptr;
    int rc;
    switch (channels) {
      case 32:
        rc = dispatch_mode<32>(pw, partial, ndepth, rb, sb, hb, vib, sob, wob, vob, n_src, height, width, vw_shift,
                               vw_offset, vw_total, a, st);
        break;
      case 16:
        rc = dispatch_mode<16>(pw, partial, ndepth, rb, sb, hb, vib, sob, wob, vob, n_src, height, width, vw_shift,
                               vw_offset, vw_total, a, st);
        break;
      case 8:
        rc = dispatch_mode<8>(pw, partial, ndepth, rb, sb, hb, vib, sob, wob, vob, n_src, height, width, vw_shift,
                              vw_offset, vw_total, a, st);
        break;
      default:
        return TMVS_ERR_SHAPE;
    }
    if (rc != TMVS_OK) return rc;
  }
  return TMVS_OK;
}

extern "C" int tmvs_aggregate_finalize(float* sim_sum, const float* w_sum, int batch, int ndepth, int height,
                                       int width, void* stream) {
  if (!sim_sum || !w_sum || batch <= 0 || ndepth <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  const int HW = height * width;
  hipLaunchKernelGGL(aggregate_finalize_kernel, dim3((HW + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream,
                     sim_sum, w_sum, ndepth, HW);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_homo_warping(const float* src_fea, const float* proj, const float* hyp, int batch, int channels,
                                 int ndepth, int height, int width, float* out, void* stream) {
  if (!src_fea || !proj || !hyp || !out || batch <= 0 || channels <= 0 || ndepth <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  const size_t HW = (size_t)height * width;
  for (int b = 0; b < batch; ++b) {
    WarpArgs a = {};
    for (int k = 0; k < 12; ++k) a.proj[0][k] = proj[(size_t)b * 12 + k];
    const int n = ndepth * (int)HW;
    hipLaunchKernelGGL(homo_warping_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       src_fea + (size_t)b * channels * HW, hyp + (size_t)b * ndepth * HW,
                       out + (size_t)b * channels * ndepth * HW, channels, ndepth, height, width, a);
    TMVS_CHECK_LAUNCH();
  }
  return TMVS_OK;
}
