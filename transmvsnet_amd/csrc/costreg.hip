// CostRegNet (models/module.py:425-456) on MI355X.
//
// Layout: NDHWC fp32 activations. Eval-mode BN is an (alpha, shift) epilogue,
// y = relu(fmaf(acc, alpha, shift)) (tmvs_bn_fold; the reference CPU kernel's exact form).
//
// Mid layers (conv1..conv6, deconv conv7/9/11) are implicit GEMMs on the exact-fp32 matrix
// cores, v_mfma_f32_16x16x4_f32 (64 FLOP/clk/SIMD, the fp32 peak; no xf32 on gfx950):
//   A (16 x 4) = weights   [cout][k]   lane l: cout = l&15, k = l>>4
//   B (4 x 16) = input     [k][voxel]  lane l: k = l>>4,   voxel = l&15
//   D (16 x16)                          lane l: cout = 4*(l>>4)+r, voxel = l&15  -> one float4
//                                       store of 4 consecutive channels (NDHWC) per lane.
// K runs over (tap, channel): per tap and CK-channel chunk a lane loads CK/4 consecutive
// channels of one voxel (float4/float2) and issues CK/4 MFMAs, MFMA j taking channel
// chunk + (l>>4)*(CK/4) + j in both operands. A "task" (one wave) is NBW rows of 16 output
// voxels x MBW blocks of 16 output channels; the 4 waves of a workgroup share the rows and
// split the output channels, so their input taps hit in L1.
// The transposed convs (ConvTranspose3d k3 s2 p1 op1) use the sub-pixel decomposition: a
// wave's 16 outputs share one parity per dimension, hence one tap set of 1, 2, 4 or 8 taps.
// conv0 (Cin 1) and prob (Cout 1) are direct VALU convolutions.
#include "common.h"

namespace tmvs {

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int N>
struct VecN;
template <>
struct VecN<4> {
  float v[4];
  __device__ __forceinline__ void load(const float* p) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  }
  __device__ __forceinline__ void zero() { v[0] = v[1] = v[2] = v[3] = 0.f; }
};
template <>
struct VecN<2> {
  float v[2];
  __device__ __forceinline__ void load(const float* p) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x;
    v[1] = t.y;
  }
  __device__ __forceinline__ void zero() { v[0] = v[1] = 0.f; }
};

struct Geo {
  int Di, Hi, Wi;  // input dims
  int Do, Ho, Wo;  // output dims
};

// ---------------------------------------------------------------- conv3d k3 p1, stride S
template <int CIN, int COUT, int S, int NBW, int MBW>
__global__ __launch_bounds__(256) void conv3d_mfma_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                          const float* __restrict__ alpha,
                                                          const float* __restrict__ shift, float* __restrict__ y,
                                                          Geo g, int n_tasks) {
  constexpr int CK = CIN < 16 ? CIN : 16;  // channels per K chunk
  constexpr int PL = CK / 4;               // channels per lane per chunk (= MFMAs per chunk)
  constexpr int MB = (COUT + 15) / 16;     // 16-channel output blocks
  constexpr int MG = MB / MBW;             // wave groups along cout
  static_assert(MB % MBW == 0, "MBW must divide MB");
  const int lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= n_tasks) return;
  // task -> (mg fastest, wseg, hgrp, od, n)
  int t = task;
  const int mg = t % MG;
  t /= MG;
  const int nws = (g.Wo + 15) / 16;
  const int wseg = t % nws;
  t /= nws;
  const int nhg = (g.Ho + NBW - 1) / NBW;
  const int hg = t % nhg;
  t /= nhg;
  const int od = t % g.Do;
  const int n = t / g.Do;

  const int col = lane & 15;
  const int kgrp = lane >> 4;
  const int ow = wseg * 16 + col;
  const size_t in_n = (size_t)n * g.Di * g.Hi * g.Wi;

  floatx4 acc[NBW][MBW];
#pragma unroll
  for (int r = 0; r < NBW; ++r)
#pragma unroll
    for (int m = 0; m < MBW; ++m) acc[r][m] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int kd = 0; kd < 3; ++kd) {
    const int id = od * S - 1 + kd;
    if (id < 0 || id >= g.Di) continue;  // wave-uniform
    for (int kh = 0; kh < 3; ++kh) {
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kd * 9 + kh * 3 + kw;
        const int iw = ow * S - 1 + kw;
        const bool wok = iw >= 0 && iw < g.Wi && ow < g.Wo;
#pragma unroll
        for (int ch = 0; ch < CIN / CK; ++ch) {
          const int cbase = ch * CK + kgrp * PL;
          VecN<PL> a[MBW];
#pragma unroll
          for (int m = 0; m < MBW; ++m) {
            const int co = (mg * MBW + m) * 16 + col;
            if (co < COUT)
              a[m].load(wpk + ((size_t)tap * COUT + co) * CIN + cbase);
            else
              a[m].zero();
          }
          VecN<PL> b[NBW];
#pragma unroll
          for (int r = 0; r < NBW; ++r) {
            const int oh = hg * NBW + r;
            const int ih = oh * S - 1 + kh;
            if (wok && oh < g.Ho && ih >= 0 && ih < g.Hi)
              b[r].load(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * CIN + cbase);
            else
              b[r].zero();
          }
#pragma unroll
          for (int j = 0; j < PL; ++j)
#pragma unroll
            for (int r = 0; r < NBW; ++r)
#pragma unroll
              for (int m = 0; m < MBW; ++m)
                acc[r][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m].v[j], b[r].v[j], acc[r][m], 0, 0, 0);
        }
      }
    }
  }
  // epilogue: lane holds couts 4*kgrp..+3 of block m for voxel `col`
  if (ow >= g.Wo) return;
  const size_t out_n = (size_t)n * g.Do * g.Ho * g.Wo;
#pragma unroll
  for (int m = 0; m < MBW; ++m) {
    const int co = (mg * MBW + m) * 16 + kgrp * 4;
    if (co >= COUT) continue;
    const float4 al = *reinterpret_cast<const float4*>(alpha + co);
    const float4 sh = *reinterpret_cast<const float4*>(shift + co);
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int oh = hg * NBW + r;
      if (oh >= g.Ho) continue;
      float4 o;
      o.x = relu(fmaf(acc[r][m][0], al.x, sh.x));
      o.y = relu(fmaf(acc[r][m][1], al.y, sh.y));
      o.z = relu(fmaf(acc[r][m][2], al.z, sh.z));
      o.w = relu(fmaf(acc[r][m][3], al.w, sh.w));
      *reinterpret_cast<float4*>(y + (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co) = o;
    }
  }
}

// ---------------------------------------------------------------- ConvTranspose3d k3 s2 p1 op1
// output o = 2i - 1 + k: parity 0 -> (k=1, i=o/2); parity 1 -> (k=0, i=o/2+1), (k=2, i=o/2)
__device__ __forceinline__ void deconv_tap(int par, int t, int half, int& k, int& i) {
  if (par == 0) {
    k = 1;
    i = half;
  } else if (t == 0) {
    k = 0;
    i = half + 1;
  } else {
    k = 2;
    i = half;
  }
}

template <int CIN, int COUT, int NBW, int MBW>
__global__ __launch_bounds__(256) void deconv3d_mfma_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ wpk,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ skip, float* __restrict__ y,
                                                            Geo g, int n_tasks) {
  constexpr int CK = CIN < 16 ? CIN : 16;
  constexpr int PL = CK / 4;
  constexpr int MB = (COUT + 15) / 16;
  constexpr int MG = MB / MBW;
  static_assert(MB % MBW == 0, "MBW must divide MB");
  const int lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= n_tasks) return;
  // task -> (mg, pw, wseg, hgrp, ph, od, n); output w = 2*(wseg*16+col)+pw, h = 2*(hg*NBW+r)+ph
  int t = task;
  const int mg = t % MG;
  t /= MG;
  const int pw = t & 1;
  t >>= 1;
  const int nws = (g.Wi + 15) / 16;
  const int wseg = t % nws;
  t /= nws;
  const int nhg = (g.Hi + NBW - 1) / NBW;
  const int hg = t % nhg;
  t /= nhg;
  const int ph = t & 1;
  t >>= 1;
  const int od = t % g.Do;
  const int n = t / g.Do;

  const int col = lane & 15;
  const int kgrp = lane >> 4;
  const int mw = wseg * 16 + col;  // input-grid column of this lane's output
  const int ow = 2 * mw + pw;
  const size_t in_n = (size_t)n * g.Di * g.Hi * g.Wi;
  const int pd = od & 1;

  floatx4 acc[NBW][MBW];
#pragma unroll
  for (int r = 0; r < NBW; ++r)
#pragma unroll
    for (int m = 0; m < MBW; ++m) acc[r][m] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int td = 0; td < 1 + pd; ++td) {
    int kd, id;
    deconv_tap(pd, td, od >> 1, kd, id);
    if (id >= g.Di) continue;
    for (int th = 0; th < 1 + ph; ++th) {
      int kh, dh;
      deconv_tap(ph, th, 0, kh, dh);  // dh = input-row offset relative to oh/2
      for (int tw = 0; tw < 1 + pw; ++tw) {
        int kw, iw;
        deconv_tap(pw, tw, mw, kw, iw);
        const int tap = kd * 9 + kh * 3 + kw;
        const bool wok = mw < g.Wi && iw < g.Wi;
#pragma unroll
        for (int ch = 0; ch < CIN / CK; ++ch) {
          const int cbase = ch * CK + kgrp * PL;
          VecN<PL> a[MBW];
#pragma unroll
          for (int m = 0; m < MBW; ++m) {
            const int co = (mg * MBW + m) * 16 + col;
            if (co < COUT)
              a[m].load(wpk + ((size_t)tap * COUT + co) * CIN + cbase);
            else
              a[m].zero();
          }
          VecN<PL> b[NBW];
#pragma unroll
          for (int r = 0; r < NBW; ++r) {
            const int mh = hg * NBW + r;
            const int ih = mh + dh;
            if (wok && mh < g.Hi && ih < g.Hi)
              b[r].load(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * CIN + cbase);
            else
              b[r].zero();
          }
#pragma unroll
          for (int j = 0; j < PL; ++j)
#pragma unroll
            for (int r = 0; r < NBW; ++r)
#pragma unroll
              for (int m = 0; m < MBW; ++m)
                acc[r][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m].v[j], b[r].v[j], acc[r][m], 0, 0, 0);
        }
      }
    }
  }
  if (mw >= g.Wi) return;
  const size_t out_n = (size_t)n * g.Do * g.Ho * g.Wo;
#pragma unroll
  for (int m = 0; m < MBW; ++m) {
    const int co = (mg * MBW + m) * 16 + kgrp * 4;
    if (co >= COUT) continue;
    const float4 al = *reinterpret_cast<const float4*>(alpha + co);
    const float4 sh = *reinterpret_cast<const float4*>(shift + co);
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int mh = hg * NBW + r;
      if (mh >= g.Hi) continue;
      const int oh = 2 * mh + ph;
      const size_t o = (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co;
      const float4 s = *reinterpret_cast<const float4*>(skip + o);
      float4 v;
      v.x = s.x + relu(fmaf(acc[r][m][0], al.x, sh.x));
      v.y = s.y + relu(fmaf(acc[r][m][1], al.y, sh.y));
      v.z = s.z + relu(fmaf(acc[r][m][2], al.z, sh.z));
      v.w = s.w + relu(fmaf(acc[r][m][3], al.w, sh.w));
      *reinterpret_cast<float4*>(y + o) = v;
    }
  }
}

// ---------------------------------------------------------------- conv0: Cin=1 -> 8, VALU
__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ x, float* __restrict__ y, int D, int H,
                                                    int W, const float* __restrict__ wt,
                                                    const float* __restrict__ alpha,
                                                    const float* __restrict__ shift) {
  const int HW = H * W;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= D * HW) return;
  const int n = blockIdx.y;
  const int d = v / HW, rem = v - d * HW, h = rem / W, w = rem - h * W;
  const float* xn = x + (size_t)n * D * HW;
  float acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int id = d - 1 + kd;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = h - 1 + kh;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = w - 1 + kw;
        const bool ok = id >= 0 && id < D && ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float xv = ok ? xn[((size_t)id * H + ih) * W + iw] : 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(wt[c * 27 + kd * 9 + kh * 3 + kw], xv, acc[c]);
      }
    }
  }
  float4 o0, o1;
  o0.x = relu(fmaf(acc[0], alpha[0], shift[0]));
  o0.y = relu(fmaf(acc[1], alpha[1], shift[1]));
  o0.z = relu(fmaf(acc[2], alpha[2], shift[2]));
  o0.w = relu(fmaf(acc[3], alpha[3], shift[3]));
  o1.x = relu(fmaf(acc[4], alpha[4], shift[4]));
  o1.y = relu(fmaf(acc[5], alpha[5], shift[5]));
  o1.z = relu(fmaf(acc[6], alpha[6], shift[6]));
  o1.w = relu(fmaf(acc[7], alpha[7], shift[7]));
  float4* yo = reinterpret_cast<float4*>(y + ((size_t)n * D * HW + v) * 8);
  yo[0] = o0;
  yo[1] = o1;
}

// ---------------------------------------------------------------- prob: 8 -> 1, VALU
__global__ __launch_bounds__(256) void prob_kernel(const float* __restrict__ x, float* __restrict__ y, int D, int H,
                                                   int W, const float* __restrict__ wt) {
  const int HW = H * W;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= D * HW) return;
  const int n = blockIdx.y;
  const int d = v / HW, rem = v - d * HW, h = rem / W, w = rem - h * W;
  const float* xn = x + (size_t)n * D * HW * 8;
  float acc = 0.f;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int id = d - 1 + kd;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = h - 1 + kh;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = w - 1 + kw;
        const bool ok = id >= 0 && id < D && ih >= 0 && ih < H && iw >= 0 && iw < W;
        if (!ok) continue;
        const float4* p = reinterpret_cast<const float4*>(xn + (((size_t)id * H + ih) * W + iw) * 8);
        const float4 u = p[0], q = p[1];
        const int tap = kd * 9 + kh * 3 + kw;
        acc = fmaf(wt[0 * 27 + tap], u.x, acc);
        acc = fmaf(wt[1 * 27 + tap], u.y, acc);
        acc = fmaf(wt[2 * 27 + tap], u.z, acc);
        acc = fmaf(wt[3 * 27 + tap], u.w, acc);
        acc = fmaf(wt[4 * 27 + tap], q.x, acc);
        acc = fmaf(wt[5 * 27 + tap], q.y, acc);
        acc = fmaf(wt[6 * 27 + tap], q.z, acc);
        acc = fmaf(wt[7 * 27 + tap], q.w, acc);
      }
    }
  }
  y[(size_t)n * D * HW + v] = acc;
}

// ---------------------------------------------------------------- launchers
template <int CIN, int COUT, int S, int NBW, int MBW>
static int launch_conv(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                       const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBW;
  const long n_tasks = (long)B * g.Do * ((g.Ho + NBW - 1) / NBW) * ((g.Wo + 15) / 16) * MG;
  const int nblk = (int)((n_tasks + 3) / 4);
  hipLaunchKernelGGL((conv3d_mfma_kernel<CIN, COUT, S, NBW, MBW>), dim3(nblk), dim3(256), 0, st, x, w, al, sh, y, g,
                     (int)n_tasks);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int CIN, int COUT, int NBW, int MBW>
static int launch_deconv(const float* x, const float* w, const float* al, const float* sh, const float* skip,
                         float* y, int B, const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBW;
  const long n_tasks = (long)B * g.Do * 2 * ((g.Hi + NBW - 1) / NBW) * ((g.Wi + 15) / 16) * 2 * MG;
  const int nblk = (int)((n_tasks + 3) / 4);
  hipLaunchKernelGGL((deconv3d_mfma_kernel<CIN, COUT, NBW, MBW>), dim3(nblk), dim3(256), 0, st, x, w, al, sh, skip,
                     y, g, (int)n_tasks);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

static int conv_dispatch(const float* x, int B, int cin, int d, int h, int w, const float* wpk, const float* al,
                         const float* sh, int cout, int stride, float* y, hipStream_t st) {
  Geo g;
  g.Di = d;
  g.Hi = h;
  g.Wi = w;
  if (stride == 1) {
    g.Do = d;
    g.Ho = h;
    g.Wo = w;
  } else {
    g.Do = (d - 1) / 2 + 1;
    g.Ho = (h - 1) / 2 + 1;
    g.Wo = (w - 1) / 2 + 1;
  }
#define TMVS_CONV_CASE(CI, CO, S, NBW, MBW) \
  if (cin == CI && cout == CO && stride == S) return launch_conv<CI, CO, S, NBW, MBW>(x, wpk, al, sh, y, B, g, st);
  TMVS_CONV_CASE(8, 16, 2, 4, 1)
  TMVS_CONV_CASE(16, 16, 1, 4, 1)
  TMVS_CONV_CASE(16, 32, 2, 4, 1)
  TMVS_CONV_CASE(32, 32, 1, 4, 1)
  TMVS_CONV_CASE(32, 64, 2, 2, 1)
  TMVS_CONV_CASE(64, 64, 1, 2, 1)
  TMVS_CONV_CASE(8, 8, 1, 4, 1)
  TMVS_CONV_CASE(16, 16, 2, 4, 1)
#undef TMVS_CONV_CASE
  return TMVS_ERR_SHAPE;
}

static int deconv_dispatch(const float* x, int B, int cin, int d, int h, int w, const float* wpk, const float* al,
                           const float* sh, int cout, const float* skip, float* y, hipStream_t st) {
  Geo g;
  g.Di = d;
  g.Hi = h;
  g.Wi = w;
  g.Do = 2 * d;
  g.Ho = 2 * h;
  g.Wo = 2 * w;
#define TMVS_DECONV_CASE(CI, CO, NBW, MBW) \
  if (cin == CI && cout == CO) return launch_deconv<CI, CO, NBW, MBW>(x, wpk, al, sh, skip, y, B, g, st);
  TMVS_DECONV_CASE(64, 32, 2, 1)
  TMVS_DECONV_CASE(32, 16, 4, 1)
  TMVS_DECONV_CASE(16, 8, 4, 1)
#undef TMVS_DECONV_CASE
  return TMVS_ERR_SHAPE;
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_conv3d_bn_relu(const float* x, int batch, int cin, int d, int h, int w, const float* wpk,
                                   const float* alpha, const float* shift, int cout, int stride, float* y,
                                   void* stream) {
  if (!x || !wpk || !alpha || !shift || !y || batch <= 0 || d <= 0 || h <= 0 || w <= 0) return TMVS_ERR_ARG;
  if (stride != 1 && stride != 2) return TMVS_ERR_ARG;
  return conv_dispatch(x, batch, cin, d, h, w, wpk, alpha, shift, cout, stride, y, (hipStream_t)stream);
}

extern "C" int tmvs_deconv3d_bn_relu_add(const float* x, int batch, int cin, int d, int h, int w, const float* wpk,
                                         const float* alpha, const float* shift, int cout, const float* skip,
                                         float* y, void* stream) {
  if (!x || !wpk || !alpha || !shift || !skip || !y || batch <= 0 || d <= 0 || h <= 0 || w <= 0)
    return TMVS_ERR_ARG;
  return deconv_dispatch(x, batch, cin, d, h, w, wpk, alpha, shift, cout, skip, y, (hipStream_t)stream);
}

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

extern "C" size_t tmvs_costregnet_workspace(int batch, int depth, int height, int width, int base_ch) {
  const size_t v0 = (size_t)batch * depth * height * width;
  const size_t v1 = v0 / 8, v2 = v0 / 64, v3 = v0 / 512;
  const size_t c = (size_t)base_ch;
  // conv0, conv1, conv2, conv3, conv4, conv5, conv6, x7, x9, x11
  size_t bytes = 0;
  bytes += align_up(v0 * c * 4);          // conv0
  bytes += align_up(v1 * 2 * c * 4) * 2;  // conv1, conv2
  bytes += align_up(v2 * 4 * c * 4) * 2;  // conv3, conv4
  bytes += align_up(v3 * 8 * c * 4) * 2;  // conv5, conv6
  bytes += align_up(v2 * 4 * c * 4);      // conv4 + conv7(x)
  bytes += align_up(v1 * 2 * c * 4);      // conv2 + conv9(x)
  bytes += align_up(v0 * c * 4);          // conv0 + conv11(x)
  return bytes;
}

extern "C" int tmvs_costregnet(const float* x, int batch, int depth, int height, int width,
                               const TmvsCostRegWeights* w, void* workspace, size_t workspace_bytes, float* logits,
                               void* stream) {
  if (!x || !w || !workspace || !logits || batch <= 0) return TMVS_ERR_ARG;
  if (depth % 8 || height % 8 || width % 8) return TMVS_ERR_SHAPE;
  if (w->base_ch != 8) return TMVS_ERR_SHAPE;
  for (int i = 0; i < 11; ++i)
    if (!w->w[i]) return TMVS_ERR_ARG;
  for (int i = 0; i < 10; ++i)
    if (!w->alpha[i] || !w->shift[i]) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_costregnet_workspace(batch, depth, height, width, w->base_ch)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int c = w->base_ch;
  const size_t v0 = (size_t)batch * depth * height * width;
  const size_t v1 = v0 / 8, v2 = v0 / 64, v3 = v0 / 512;
  char* ws = (char*)workspace;
  auto take = [&](size_t n) {
    float* p = (float*)ws;
    ws += align_up(n * 4);
    return p;
  };
  float* c0 = take(v0 * c);
  float* c1 = take(v1 * 2 * c);
  float* c2 = take(v1 * 2 * c);
  float* c3 = take(v2 * 4 * c);
  float* c4 = take(v2 * 4 * c);
  float* c5 = take(v3 * 8 * c);
  float* c6 = take(v3 * 8 * c);
  float* x7 = take(v2 * 4 * c);
  float* x9 = take(v1 * 2 * c);
  float* x11 = take(v0 * c);
  const int D0 = depth, H0 = height, W0 = width;
  const int D1 = D0 / 2, H1 = H0 / 2, W1 = W0 / 2;
  const int D2 = D1 / 2, H2 = H1 / 2, W2 = W1 / 2;
  const int D3 = D2 / 2, H3 = H2 / 2, W3 = W2 / 2;
  int rc;
  const dim3 g0((unsigned)((D0 * H0 * W0 + 255) / 256), (unsigned)batch);
  hipLaunchKernelGGL(conv0_kernel, g0, dim3(256), 0, st, x, c0, D0, H0, W0, w->w[0], w->alpha[0], w->shift[0]);
  TMVS_CHECK_LAUNCH();
  if ((rc = conv_dispatch(c0, batch, c, D0, H0, W0, w->w[1], w->alpha[1], w->shift[1], 2 * c, 2, c1, st))) return rc;
  if ((rc = conv_dispatch(c1, batch, 2 * c, D1, H1, W1, w->w[2], w->alpha[2], w->shift[2], 2 * c, 1, c2, st)))
    return rc;
  if ((rc = conv_dispatch(c2, batch, 2 * c, D1, H1, W1, w->w[3], w->alpha[3], w->shift[3], 4 * c, 2, c3, st)))
    return rc;
  if ((rc = conv_dispatch(c3, batch, 4 * c, D2, H2, W2, w->w[4], w->alpha[4], w->shift[4], 4 * c, 1, c4, st)))
    return rc;
  if ((rc = conv_dispatch(c4, batch, 4 * c, D2, H2, W2, w->w[5], w->alpha[5], w->shift[5], 8 * c, 2, c5, st)))
    return rc;
  if ((rc = conv_dispatch(c5, batch, 8 * c, D3, H3, W3, w->w[6], w->alpha[6], w->shift[6], 8 * c, 1, c6, st)))
    return rc;
  if ((rc = deconv_dispatch(c6, batch, 8 * c, D3, H3, W3, w->w[7], w->alpha[7], w->shift[7], 4 * c, c4, x7, st)))
    return rc;
  if ((rc = deconv_dispatch(x7, batch, 4 * c, D2, H2, W2, w->w[8], w->alpha[8], w->shift[8], 2 * c, c2, x9, st)))
    return rc;
  if ((rc = deconv_dispatch(x9, batch, 2 * c, D1, H1, W1, w->w[9], w->alpha[9], w->shift[9], c, c0, x11, st)))
    return rc;
  hipLaunchKernelGGL(prob_kernel, g0, dim3(256), 0, st, x11, logits, D0, H0, W0, w->w[10]);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
