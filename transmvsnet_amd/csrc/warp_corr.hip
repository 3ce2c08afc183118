// Fused cost-volume build for one cascade stage (DepthNet steps 1-2,
// reference models/TransMVSNet.py:58-93 and homo_warping models/module.py:284-322).
//
// One thread owns one reference pixel and DPT consecutive depth planes; the G = D/DPT
// threads of a pixel are adjacent lanes of one wave (the PixelwiseNet max over D is a
// lane-shuffle reduction among them). Per source view the thread projects its pixel into
// the view, bilinearly samples the channels-last source features (4 taps x C floats,
// float4 loads) and forms the single-group correlation against the reference features it
// keeps in registers; the warped [C,D,H,W] volume of the reference never exists.
//
// fp32 op order follows the reference's PyTorch-CPU kernels (DESIGN.md "Numerics"):
//   rot·(x,y,1)   : fmaf(r1, y, r0*x) + r2            (bmm, FMA chain)
//   X = rot_xyz*d + t ; px = X/Z ; xn = px/((W-1)/2) - 1 ; z < 1e-6 -> xn = yn = -99
//   ix = (xn + 1) * ((W-1)/2)                          (grid_sample, align_corners=True)
//   v  = fmaf(se_v,se, fmaf(sw_v,sw, fmaf(ne_v,ne, nw_v*nw)))  (zeros padding)
//   sim = (Σ_c v_c*ref_c) / C ; sim_sum += sim*w ; w_sum = 1e-5 + Σ w ; sim_sum / w_sum
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

template <int C, int DPT, int G, bool PW, bool PARTIAL>
__global__ __launch_bounds__(256) void warp_corr_kernel(
    const float* __restrict__ ref, const float* __restrict__ src, const float* __restrict__ hyp,
    const float* __restrict__ vw_in, float* __restrict__ sim_out, float* __restrict__ wsum_out,
    float* __restrict__ vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total, WarpArgs args) {
  constexpr int PIX_PER_BLOCK = 256 / G;
  const int HW = H * W;
  const int nblk = (HW + PIX_PER_BLOCK - 1) / PIX_PER_BLOCK;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int g = threadIdx.x % G;
  int p = tile * PIX_PER_BLOCK + threadIdx.x / G;
  const bool active = p < HW;
  if (!active) p = HW - 1;  // keep the lane alive for the G-lane shuffles; never stores
  const int py = p / W, px = p - py * W;
  const float fx = (float)px, fy = (float)py;
  const int d0 = g * DPT;

  float refv[C];
#pragma unroll
  for (int c4 = 0; c4 < C / 4; ++c4) {
    const float4 r = *reinterpret_cast<const float4*>(ref + (size_t)p * C + c4 * 4);
    refv[c4 * 4 + 0] = r.x;
    refv[c4 * 4 + 1] = r.y;
    refv[c4 * 4 + 2] = r.z;
    refv[c4 * 4 + 3] = r.w;
  }
  float dep[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) dep[j] = hyp[(size_t)(d0 + j) * HW + p];

  const float halfw = (float)(W - 1) / 2.f;  // (width - 1) / 2, exact
  const float halfh = (float)(H - 1) / 2.f;
  float ssum[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) ssum[j] = 0.f;
  float wsum = PARTIAL ? 0.f : 1e-5f;

  for (int v = 0; v < V; ++v) {
    const float* R = args.proj[v];
    const float rx = fmaf(R[1], fy, R[0] * fx) + R[2];
    const float ry = fmaf(R[5], fy, R[4] * fx) + R[6];
    const float rz = fmaf(R[9], fy, R[8] * fx) + R[10];
    const float tx = R[3], ty = R[7], tz = R[11];
    const float* __restrict__ sv = src + (size_t)v * HW * C;
    float sim[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const float X = rx * dep[j] + tx;
      const float Y = ry * dep[j] + ty;
      const float Z = rz * dep[j] + tz;
      float xn = (X / Z) / halfw - 1.f;
      float yn = (Y / Z) / halfh - 1.f;
      if (Z < 1e-6f) {
        xn = -99.f;
        yn = -99.f;
      }
      const float ix = (xn + 1.f) * halfw;
      const float iy = (yn + 1.f) * halfh;
      const float x0 = floorf(ix), y0 = floorf(iy);
      const float we = ix - x0, ea = 1.f - we;
      const float n = iy - y0, s = 1.f - n;
      const float wnw = s * ea, wne = s * we, wsw = n * ea, wse = n * we;
      const bool vx0 = x0 >= 0.f && x0 <= (float)(W - 1);
      const bool vx1 = x0 + 1.f >= 0.f && x0 + 1.f <= (float)(W - 1);
      const bool vy0 = y0 >= 0.f && y0 <= (float)(H - 1);
      const bool vy1 = y0 + 1.f >= 0.f && y0 + 1.f <= (float)(H - 1);
      const int xi0 = vx0 ? (int)x0 : 0, xi1 = vx1 ? (int)x0 + 1 : 0;
      const int yi0 = vy0 ? (int)y0 : 0, yi1 = vy1 ? (int)y0 + 1 : 0;
      const float* t00 = sv + ((size_t)yi0 * W + xi0) * C;
      const float* t01 = sv + ((size_t)yi0 * W + xi1) * C;
      const float* t10 = sv + ((size_t)yi1 * W + xi0) * C;
      const float* t11 = sv + ((size_t)yi1 * W + xi1) * C;
      const bool m00 = vy0 && vx0, m01 = vy0 && vx1, m10 = vy1 && vx0, m11 = vy1 && vx1;
      float acc = 0.f;
#pragma unroll
      for (int c4 = 0; c4 < C / 4; ++c4) {
        float4 a = *reinterpret_cast<const float4*>(t00 + c4 * 4);
        float4 b = *reinterpret_cast<const float4*>(t01 + c4 * 4);
        float4 c = *reinterpret_cast<const float4*>(t10 + c4 * 4);
        float4 d = *reinterpret_cast<const float4*>(t11 + c4 * 4);
        if (!m00) a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!m01) b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!m10) c = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!m11) d = make_float4(0.f, 0.f, 0.f, 0.f);
        const float va[4] = {a.x, a.y, a.z, a.w};
        const float vb[4] = {b.x, b.y, b.z, b.w};
        const float vc[4] = {c.x, c.y, c.z, c.w};
        const float vd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float val = fmaf(vd[k], wse, fmaf(vc[k], wsw, fmaf(vb[k], wne, va[k] * wnw)));
          acc = acc + val * refv[c4 * 4 + k];
        }
      }
      sim[j] = acc / (float)C;
    }
    float w;
    if constexpr (PW) {
      float wm = 0.f;  // sigmoid > 0, so 0 is a neutral start for the max
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        const float lg = pixelwise_logit(sim[j], args.pw);
        const float sg = 1.f / (1.f + expf(-lg));
        wm = fmaxf(wm, sg);
      }
#pragma unroll
      for (int off = 1; off < G; off <<= 1) wm = fmaxf(wm, __shfl_xor(wm, off, G));
      w = wm;
      if (active && g == 0) vw_out[(size_t)(vw_offset + v) * HW + p] = w;
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
    for (int j = 0; j < DPT; ++j) sim_out[(size_t)(d0 + j) * HW + p] = ssum[j];
    if (g == 0) wsum_out[p] = wsum;
  } else {
#pragma unroll
    for (int j = 0; j < DPT; ++j) sim_out[(size_t)(d0 + j) * HW + p] = ssum[j] / wsum;
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

template <int C, int DPT, int G, bool PW, bool PARTIAL>
static int launch_warp(const float* ref, const float* src, const float* hyp, const float* vw_in, float* sim,
                       float* wsum, float* vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total,
                       const WarpArgs& args, hipStream_t st) {
  constexpr int PIX = 256 / G;
  const int nblk = (H * W + PIX - 1) / PIX;
  hipLaunchKernelGGL((warp_corr_kernel<C, DPT, G, PW, PARTIAL>), dim3(nblk), dim3(256), 0, st, ref, src, hyp, vw_in,
                     sim, wsum, vw_out, V, H, W, vw_shift, vw_offset, vw_total, args);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int C, bool PW, bool PARTIAL>
static int dispatch_depth(int D, const float* ref, const float* src, const float* hyp, const float* vw_in, float* sim,
                          float* wsum, float* vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total,
                          const WarpArgs& a, hipStream_t st) {
#define TMVS_WARP_CASE(DD, DPT, G)                                                                                \
  if (D == DD)                                                                                                    \
    return launch_warp<C, DPT, G, PW, PARTIAL>(ref, src, hyp, vw_in, sim, wsum, vw_out, V, H, W, vw_shift,        \
                                                vw_offset, vw_total, a, st);
  TMVS_WARP_CASE(48, 12, 4)
  TMVS_WARP_CASE(32, 8, 4)
  TMVS_WARP_CASE(16, 8, 2)
  TMVS_WARP_CASE(8, 8, 1)
  TMVS_WARP_CASE(64, 16, 4)
  TMVS_WARP_CASE(24, 12, 2)
  TMVS_WARP_CASE(4, 4, 1)
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
