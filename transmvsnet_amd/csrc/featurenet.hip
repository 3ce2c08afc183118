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
// channels, N = 16 pixels, K = 9 taps x 32 input channels. Lane (j, n) of the B operand samples
// pixel n itself and holds channels {4j..4j+3} (k-steps 0-3) and {16+4j..16+4j+3} (k-steps 4-7)
// of the tap: the weights are packed in that K order, as the kernel's LDS image.
//
// Work unit = (image, NW-row band, 16-pixel column step); wave w of the NW*64-thread block owns row
// NW*band + w of the unit (NW = 12 by default: 3 waves/SIMD). Per unit the block stages the source
// window rows [NW*band - HL, +NW+2HL) x columns [x0 - HL, +16+2HL) x 32 channels in LDS (HL = 3:
// 50 KB), so the 4 bilinear corners of every tap whose offsets stay within the window (|offset| up to
// ~HL - 1 px; the reference's zero-initialised offsets, models/dcn.py:62-64, always) are LDS reads; a
// wave whose unit has a sample beyond the window runs the same taps with per-lane global fallback
// gathers (dcn_taps_slow). The next unit's window is fetched into registers during the current unit's
// taps. Window layout: 16-byte chunk c of window pixel P at P*8 + (c ^ (P & 7)), which makes both the
// staging writes (one 128-byte pixel row per 8 lanes) and the B-layout reads (chunks j and j+4 of 16
// pixels per lane group) bank-conflict-free. Per (tap, pixel) 16-byte sampling records (the bilinear
// fractions, window index, mask) are built once per unit and shared by the 4 lanes of a pixel.
#include "common.h"

#include <algorithm>

namespace tmvs {

namespace dcn {
constexpr int CI = 32;     // input channels (FeatureNet heads: 4 * base_channels)
constexpr int WAVES = 8;   // waves per block = rows per unit (the 3x3 conv's unit; the DCN's: DcnWin)
constexpr int TW = 16;     // pixels per wave row
constexpr int NREC = 9 * TW;                               // (tap, pixel) records per wave
}  // namespace dcn

// The DCN's unit / window geometry: NW waves = NW rows of 16 pixels per unit, a window margin of HL
// pixels on every side (samples whose 4 corners stay inside it read LDS; others take the global path)
template <int NW, int HL>
struct DcnWin {
  static constexpr int WAVES = NW, HALO = HL, NT = NW * 64;
  static constexpr int WR = NW + 2 * HL, WC = dcn::TW + 2 * HL;  // window rows, columns
  static constexpr int WIN4 = WR * WC * 8;                       // window float4s (8 per pixel)
  static constexpr int STAGE = (WIN4 + NT - 1) / NT;             // float4 per thread per window copy
};

typedef float float2_t __attribute__((ext_vector_type(2)));

// Window slot of chunk c of window pixel P.
__device__ __forceinline__ int dcn_slot(int P, int c) { return P * 8 + (c ^ (P & 7)); }

// Timing ablations (wrong outputs by construction; A/B builds only): bit 1 drops the offset-conv MFMAs,
// 2 the bilinear blend (a tap's B operand is its first corner), 4 the tap MFMAs, 8 the window stores.
#ifndef TMVS_DCN_ABL
#define TMVS_DCN_ABL 0
#endif
#ifndef TMVS_DCN_OB12
#define TMVS_DCN_OB12 1  // offset-conv fragment buffers at 12 waves (A/B: 2 = read one tap ahead)
#endif
#ifndef TMVS_DCN_SB12
#define TMVS_DCN_SB12 1  // single tap buffers at 12 waves (A/B: 0 = double)
#endif
#ifndef TMVS_DCN_PK
#define TMVS_DCN_PK 1  // the bilinear blend on packed fp32 (A/B: 0 = scalar)
#endif

// The 9 taps of one wave-unit: gather (window LDS; beyond it, global, unless FAST), blend,
// modulate, MT x 8 MFMAs per tap.
// SB: one gather / A-fragment buffer (a tap's blend consumes the gathers before the next tap's refill
// them; the next tap's A fragments are read after this tap's MFMAs): the register budget of 3 waves/SIMD
template <int MT, bool FAST, int WC, bool SB = false>
__device__ __forceinline__ void dcn_taps(floatx4_t (&acc)[MT], const floatx4_t* __restrict__ wl,
                                         const floatx4_t* __restrict__ win, const floatx4_t* __restrict__ recs,
                                         __amdgpu_buffer_rsrc_t rx, int H, int W, int lane) {
  const int j = lane >> 4, n = lane & 15;
  floatx4_t alt = floatx4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int NB = SB ? 1 : 2;
  floatx4_t v[NB][4][2], w4[NB];
  float mk[NB];
  // the records of the next tap to gather, read one tap before its gathers (their addresses come from
  // them: read just before, each tap had waited out an LDS round trip between its MFMA blocks)
  // record = (ly, lx, window pixel of corner (y0, x0) | fallback code, mask); a sample outside the
  // image has ly = lx = 0 and mask 0, so its B operand is 0
  floatx4_t rw;
  auto rec = [&](int k) { rw = recs[k * dcn::TW + n]; };
  // gathers of the tap whose record is in rw into buffer bb (issued one tap ahead of their use); the
  // bilinear weights are formed here from the fractions, the same products the record builder formed
  auto gather = [&](int bb) {
    {
      const float ly = rw[0], lx = rw[1], hy = 1.f - ly, hx = 1.f - lx;
      w4[bb] = floatx4_t{hy * hx, hy * lx, ly * hx, ly * lx};
    }
    const int2 bm = make_int2(__float_as_int(rw[2]), 0);
    mk[bb] = rw[3];
    if (FAST || bm.x >= 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int Pc = bm.x + (c >> 1) * WC + (c & 1);
        v[bb][c][0] = win[dcn_slot(Pc, j)];
        v[bb][c][1] = win[dcn_slot(Pc, j + 4)];
      }
    } else {  // sample beyond the window: global gather (corners outside the image read 0)
      const int code = -1 - bm.x, y0 = (code >> 15) - 1, x0 = (code & 32767) - 1;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cy = y0 + (c >> 1), cx = x0 + (c & 1);
        const bool ok = (unsigned)cy < (unsigned)H && (unsigned)cx < (unsigned)W;
        const unsigned off = ok ? ((unsigned)(cy * W + cx) * dcn::CI + 4u * j) * 4u : kOffOut;
        v[bb][c][0] = buf_load_f32x4(rx, off);
        v[bb][c][1] = buf_load_f32x4(rx, off == kOffOut ? kOffOut : off + 64u);
      }
    }
  };
  // A fragments of tap k into buffer ab, read one tap ahead too: in LDS order they then precede the
  // tap's gathers, so the MFMAs never wait on the gathers issued just before them
  floatx4_t af[NB][MT][2];
  auto lda = [&](int k, int ab) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      af[ab][m][0] = wl[((k * MT + m) * 2 + 0) * 64 + lane];
      af[ab][m][1] = wl[((k * MT + m) * 2 + 1) * 64 + lane];
    }
  };
  // bilinear blend and modulation of the gathers in buffer bb into the tap's B operands
  auto blend = [&](int bb, float (&b)[8]) {
    // two channels per packed fp32 instruction (v_pk_mul_f32 / v_pk_add_f32: the same IEEE operations
    // per element as the scalar form, half the VALU issue)
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      if (TMVS_DCN_ABL & 2) {
        b[e] = v[bb][0][e >> 2][e & 3];
        b[e + 1] = v[bb][0][e >> 2][(e & 3) + 1];
        continue;
      }
      if (!TMVS_DCN_PK) {
#pragma unroll
        for (int f = e; f < e + 2; ++f) {
          float val = w4[bb][0] * v[bb][0][f >> 2][f & 3];
          val = val + w4[bb][1] * v[bb][1][f >> 2][f & 3];
          val = val + w4[bb][2] * v[bb][2][f >> 2][f & 3];
          val = val + w4[bb][3] * v[bb][3][f >> 2][f & 3];
          b[f] = mk[bb] * val;
        }
        continue;
      }
      auto pr = [&](int c) { return float2_t{v[bb][c][e >> 2][e & 3], v[bb][c][e >> 2][(e & 3) + 1]}; };
      auto bc = [](float t) { return float2_t{t, t}; };
      float2_t val = bc(w4[bb][0]) * pr(0);
      val = val + bc(w4[bb][1]) * pr(1);
      val = val + bc(w4[bb][2]) * pr(2);
      val = val + bc(w4[bb][3]) * pr(3);
      const float2_t r = bc(mk[bb]) * val;
      b[e] = r.x;
      b[e + 1] = r.y;
    }
  };
  auto mfmas = [&](const floatx4_t(&a)[MT][2], const float (&b)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (TMVS_DCN_ABL & 4) {
          acc[m][0] += b[s];
          continue;
        }
        if (MT == 1 && (s & 1))  // one output tile: two interleaved chains hide the dependent latency
          alt = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s >> 2][s & 3], b[s], alt, 0, 0, 0);
        else
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s >> 2][s & 3], b[s], acc[m], 0, 0, 0);
      }
  };
  rec(0);
  lda(0, 0);
  gather(0);
  rec(1);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int bb = SB ? 0 : k & 1;
    float b[8];
    blend(bb, b);
    if (k < 8) {
      if (!SB) lda(k + 1, bb ^ 1);
      gather(SB ? 0 : bb ^ 1);
      if (k < 7) rec(k + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(af[bb], b);
    __builtin_amdgcn_sched_barrier(0);
    if (SB && k < 8) lda(k + 1, 0);
  }
  if (MT == 1) acc[0] = acc[0] + alt;
}

// The taps of a wave-unit with a sample beyond the window (rare: offsets over ~HALO - 1 px), in the
// simplest form -- one tap at a time, no read-ahead -- so it does not raise the kernel's register
// budget: the same gathers (window or global), blend and MFMA chains as dcn_taps, so the same results.
template <int MT, int WC>
__device__ __forceinline__ void dcn_taps_slow(floatx4_t (&acc)[MT], const floatx4_t* __restrict__ wl,
                                           const floatx4_t* __restrict__ win, const floatx4_t* __restrict__ recs,
                                           __amdgpu_buffer_rsrc_t rx, int H, int W, int lane) {
  const int j = lane >> 4, n = lane & 15;
  floatx4_t alt = floatx4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int k = 0; k < 9; ++k) {
    const floatx4_t rw = recs[k * dcn::TW + n];
    const float ly = rw[0], lx = rw[1], hy = 1.f - ly, hx = 1.f - lx;
    const floatx4_t w4 = floatx4_t{hy * hx, hy * lx, ly * hx, ly * lx};
    const int code = __float_as_int(rw[2]);
    const float mk = rw[3];
    floatx4_t v[4][2];
    if (code >= 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int Pc = code + (c >> 1) * WC + (c & 1);
        v[c][0] = win[dcn_slot(Pc, j)];
        v[c][1] = win[dcn_slot(Pc, j + 4)];
      }
    } else {
      const int cd = -1 - code, y0 = (cd >> 15) - 1, x0 = (cd & 32767) - 1;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cy = y0 + (c >> 1), cx = x0 + (c & 1);
        const bool ok = (unsigned)cy < (unsigned)H && (unsigned)cx < (unsigned)W;
        const unsigned off = ok ? ((unsigned)(cy * W + cx) * dcn::CI + 4u * j) * 4u : kOffOut;
        v[c][0] = buf_load_f32x4(rx, off);
        v[c][1] = buf_load_f32x4(rx, off == kOffOut ? kOffOut : off + 64u);
      }
    }
    float b[8];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      auto pr = [&](int c) { return float2_t{v[c][e >> 2][e & 3], v[c][e >> 2][(e & 3) + 1]}; };
      auto bc = [](float t) { return float2_t{t, t}; };
      float2_t val = bc(w4[0]) * pr(0);
      val = val + bc(w4[1]) * pr(1);
      val = val + bc(w4[2]) * pr(2);
      val = val + bc(w4[3]) * pr(3);
      const float2_t r = bc(mk) * val;
      b[e] = r.x;
      b[e + 1] = r.y;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const floatx4_t a0 = wl[((k * MT + m) * 2 + 0) * 64 + lane], a1 = wl[((k * MT + m) * 2 + 1) * 64 + lane];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float a = s < 4 ? a0[s] : a1[s - 4];
        if (MT == 1 && (s & 1))
          alt = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[s], alt, 0, 0, 0);
        else
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[s], acc[m], 0, 0, 0);
      }
    }
  }
  if (MT == 1) acc[0] = acc[0] + alt;
}

// FUSED: the DCN's offset/mask conv (conv_offset_mask, models/dcn.py:58-64: 3x3, 32 -> 27, bias)
// is computed in-kernel from the same LDS window (implicit GEMM on MFMA, M = 27 padded to 32), so
// the [27][H][W] offset/mask tensor never exists in HBM; otherwise `om` is read from global.
template <int CO, bool FUSED, int NW, int HL>
__global__ __launch_bounds__(NW * 64) void dcn_window_kernel(const float* __restrict__ x, const float* __restrict__ om,
                                                         const float* __restrict__ wom, const float* __restrict__ bom,
                                                         const float* __restrict__ wpk,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ shift, int relu, int B, int H,
                                                         int W, float* __restrict__ out,
                                                         float* __restrict__ out_nhwc,
                                                         float* __restrict__ om_out) {
  using Cfg = DcnWin<NW, HL>;
  constexpr int NT = Cfg::NT;
  constexpr int MT = (CO + 15) / 16;
  constexpr int NA4 = 9 * MT * 2 * 64;  // A fragments [tap][mt][half][lane] float4
  constexpr int NO4 = FUSED ? 9 * 2 * 2 * 64 : 1;  // offset-conv A fragments (27 rows padded to 32)
  __shared__ floatx4_t wl[NA4];
  __shared__ floatx4_t wo[NO4];
  __shared__ floatx4_t win[Cfg::WIN4];                  // swizzled [row][col] pixels of 8 chunks
  __shared__ floatx4_t recs[NW][dcn::NREC];             // [tap][px] sampling records (16 B)
                                                        // (FUSED: first the [px][33] offset/mask tile)
  // per-channel constants: bias, BN alpha, BN shift (CO), offset-conv bias (27): read from LDS in the
  // epilogues (read from global there, each was a serialised L2 round trip per unit)
  __shared__ __attribute__((aligned(16))) float cst[4][32];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < 32) {
    cst[0][tid] = tid < CO ? bias[tid] : 0.f;
    cst[1][tid] = alpha && tid < CO ? alpha[tid] : 1.f;
    cst[2][tid] = alpha && tid < CO ? shift[tid] : 0.f;
    cst[3][tid] = FUSED && tid < 27 ? bom[tid] : 0.f;
  }
  for (int i = tid; i < NA4; i += NT) wl[i] = reinterpret_cast<const floatx4_t*>(wpk)[i];
  if (FUSED)
    for (int i = tid; i < NO4; i += NT) wo[i] = reinterpret_cast<const floatx4_t*>(wom)[i];
  const int HW = H * W, nbx = (W + dcn::TW - 1) / dcn::TW, nby = (H + NW - 1) / NW;
  const int nunits = B * nby * nbx;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int u_begin = (int)((long long)nunits * bid / gridDim.x);
  const int u_end = (int)((long long)nunits * (bid + 1) / gridDim.x);
  const int j = lane >> 4, n = lane & 15;  // MFMA layout
  const float fH = (float)H, fW = (float)W;

  // global -> register copy of a unit's window (zeros outside the image) and (not FUSED) of the
  // offsets/mask logits of the (tap, pixel) records this lane builds (r = lane + 64 i < 144)
  floatx4_t stg[Cfg::STAGE];
  float omv[9];
  auto fetch = [&](int u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    const int wy0 = band * NW - HL, wx0 = xs * dcn::TW - HL;
    const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)b * HW * dcn::CI, (unsigned)HW * dcn::CI * 4);
#pragma unroll
    for (int i = 0; i < Cfg::STAGE; ++i) {
      const int idx = min(tid + NT * i, Cfg::WIN4 - 1), pix = idx >> 3, ch = idx & 7;
      const int r = pix / Cfg::WC, c = pix - r * Cfg::WC;
      const int gy = wy0 + r, gx = wx0 + c;
      const bool ok = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      stg[i] = buf_load_f32x4(rx, ok ? ((unsigned)(gy * W + gx) * dcn::CI + 4u * ch) * 4u : kOffOut);
    }
    if (!FUSED) {
      const int row = min(band * NW + wv, H - 1), x0t = xs * dcn::TW;
      const float* omb = om + (size_t)b * 27 * HW + (size_t)row * W + x0t;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = lane + 64 * i, tap = r >> 4, px = min(r & 15, W - 1 - x0t);
        if (r < dcn::NREC) {
          omv[3 * i + 0] = omb[(size_t)(2 * tap) * HW + px];
          omv[3 * i + 1] = omb[(size_t)(2 * tap + 1) * HW + px];
          omv[3 * i + 2] = omb[(size_t)(18 + tap) * HW + px];
        }
      }
    }
  };

  if (u_begin < u_end) fetch(u_begin);
  for (int u = u_begin; u < u_end; ++u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    const int wy0 = band * NW - HL, wx0 = xs * dcn::TW - HL;
    __syncthreads();  // previous unit's window reads are done (and, first time, the weights are staged)
#pragma unroll
    for (int i = 0; i < Cfg::STAGE; ++i) {
      const int idx = tid + NT * i;
      if ((Cfg::WIN4 % NT == 0 || idx < Cfg::WIN4) && (!(TMVS_DCN_ABL & 8) || u == u_begin))
        win[dcn_slot(idx >> 3, idx & 7)] = stg[i];
    }
    __syncthreads();
    if (u + 1 < u_end) fetch(u + 1);  // next window in flight during this unit's work
    const int row = band * NW + wv;
    const int x0t = xs * dcn::TW, nvalid = min(dcn::TW, W - x0t);
    if (row >= H) continue;
    if (FUSED) {
      // conv_offset_mask of this wave's 16 pixels from the window: B lane (j, n) = chunks j, j+4 of
      // window pixel (wv + HALO + ki - 1, HALO + n + kj - 1); D lane (j, n) = channels 16m + 4j + i
      // (tap k + 1's fragments are read during tap k's MFMAs)
      floatx4_t ao[2] = {floatx4_t{0.f, 0.f, 0.f, 0.f}, floatx4_t{0.f, 0.f, 0.f, 0.f}};
      constexpr int OB = NW > 8 ? TMVS_DCN_OB12 : 2;  // 3 waves/SIMD: read each tap's fragments just before it
      floatx4_t fb[OB][2], fa[OB][2][2];
      auto frag = [&](int k, int bf) {
        const int ki = k / 3, kj = k - 3 * ki;
        const int P = (wv + HL + ki - 1) * Cfg::WC + HL + n + kj - 1;
        fb[bf][0] = win[dcn_slot(P, j)];
        fb[bf][1] = win[dcn_slot(P, j + 4)];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          fa[bf][m][0] = wo[((k * 2 + m) * 2 + 0) * 64 + lane];
          fa[bf][m][1] = wo[((k * 2 + m) * 2 + 1) * 64 + lane];
        }
      };
      if (OB == 2) frag(0, 0);
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (OB == 1)
          frag(k, 0);
        else if (k < 8)
          frag(k + 1, (k + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);  // keep those reads ahead of this tap's MFMAs
        const int ob = OB == 1 ? 0 : k & 1;
        const floatx4_t b0 = fb[ob][0], b1 = fb[ob][1];
        const floatx4_t(&a)[2][2] = fa[ob];
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            if (TMVS_DCN_ABL & 1) {
              ao[m][0] += (s < 4 ? b0[s] : b1[s - 4]) * a[m][s >> 2][s & 3];
              continue;
            }
            ao[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s >> 2][s & 3], s < 4 ? b0[s] : b1[s - 4], ao[m], 0,
                                                         0, 0);
          }
      }
      // [px][33] tile (odd row stride: the record builders' column reads hit 16 distinct banks),
      // consumed before the records overwrite it
      float* omt = reinterpret_cast<float*>(recs[wv]);
      static_assert(16 * 33 <= 4 * dcn::NREC, "offset tile fits a wave's records");
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * m + 4 * j + i;
          if (c < 27) {
            const float o = ao[m][i] + cst[3][c];
            omt[n * 33 + c] = o;
            // training: the offset/mask tensor the backward needs ([B][27][H][W])
            if (om_out && n < nvalid) om_out[((size_t)b * 27 + c) * HW + (size_t)row * W + x0t + n] = o;
          }
        }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = lane + 64 * i;
        if (r < dcn::NREC) {
          const int tap = r >> 4, px = r & 15;
          omv[3 * i + 0] = omt[px * 33 + 2 * tap];
          omv[3 * i + 1] = omt[px * 33 + 2 * tap + 1];
          omv[3 * i + 2] = omt[px * 33 + 18 + tap];
        }
      }
    }
    // sampling records of this wave's 16 pixels x 9 taps: window pixel of corner (y0, x0), or for a
    // sample beyond the window -1 - ((y0 + 1) << 15 | (x0 + 1)); the 4 bilinear weights (zero when
    // the sample point is outside the image: the column is then 0, as in torchvision); the mask
    bool lane_fast = true;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int r = lane + 64 * i;
      if (r < dcn::NREC) {
        const int tap = r >> 4, px = r & 15, ki = tap / 3, kj = tap - 3 * ki;
        const float py = (float)(row + ki - 1) + omv[3 * i + 0];
        const float pxf = (float)(x0t + min(px, nvalid - 1) + kj - 1) + omv[3 * i + 1];
        const bool inside = py > -1.f && py < fH && pxf > -1.f && pxf < fW;
        const float y0 = floorf(py), x0 = floorf(pxf);
        const float ly = py - y0, lx = pxf - x0;
        const float hy = 1.f - ly, hx = 1.f - lx;
        const int y0i = (int)fmaxf(fminf(y0, 32766.f), -2.f), x0i = (int)fmaxf(fminf(x0, 32766.f), -2.f);
        const int ry = y0i - wy0, rxw = x0i - wx0;
        const bool inwin = (unsigned)ry < (unsigned)(Cfg::WR - 1) && (unsigned)rxw < (unsigned)(Cfg::WC - 1);
        lane_fast = lane_fast && (inwin || !inside);
        const float mk = __frcp_rn(1.f + __expf(-omv[3 * i + 2]));  // sigmoid (fast exp / rcp)
        // inside => y0 in [-1, H-1], x0 in [-1, W-1]: the fallback code fits 30 bits
        const int code = !inside ? 0 : inwin ? ry * Cfg::WC + rxw : -1 - (((y0i + 1) << 15) | (x0i + 1));
        (void)hy;
        (void)hx;
        recs[wv][r] = inside ? floatx4_t{ly, lx, __int_as_float(code), mk} : floatx4_t{0.f, 0.f, __int_as_float(0), 0.f};
      }
    }
    // every sample of the wave's unit inside the window: the branch-free tap loop
    const bool fast = __all(lane_fast);
    const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)b * HW * dcn::CI, (unsigned)HW * dcn::CI * 4);
    floatx4_t acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    constexpr bool SB = NW > 8 && TMVS_DCN_SB12;  // 3 waves/SIMD: single buffers
    if (fast)
      dcn_taps<MT, true, Cfg::WC, SB>(acc, wl, win, recs[wv], rx, H, W, lane);
    else if (SB)
      dcn_taps_slow<MT, Cfg::WC>(acc, wl, win, recs[wv], rx, H, W, lane);
    else
      dcn_taps<MT, false, Cfg::WC, SB>(acc, wl, win, recs[wv], rx, H, W, lane);
    // D fragment: lane (j, n) holds output channels 16m + 4j .. +3 of pixel (row, x0t + n)
    if (n < nvalid) {
      const int pq = row * W + x0t + n;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int co0 = 16 * m + 4 * j;
        if (co0 >= CO) continue;
        const floatx4_t cb = *reinterpret_cast<const floatx4_t*>(&cst[0][co0]);
        const floatx4_t ca = *reinterpret_cast<const floatx4_t*>(&cst[1][co0]);
        const floatx4_t cs = *reinterpret_cast<const floatx4_t*>(&cst[2][co0]);
        float r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float y = acc[m][i] + cb[i];
          if (alpha) y = fmaf(y, ca[i], cs[i]);
          if (relu) y = fmaxf(y, 0.f);
          r[i] = y;
          if (out) out[((size_t)b * CO + co0 + i) * HW + pq] = y;
        }
        if (out_nhwc)
          *reinterpret_cast<float4*>(out_nhwc + ((size_t)b * HW + pq) * CO + co0) = make_float4(r[0], r[1], r[2], r[3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The heads' first layer Conv2d(32, 32, 3, 1, 1, bias=False) + BatchNorm + ReLU (models/module.py:24-61,
// 373/385) in NHWC: the DCN kernel's unit/window scheme with a 1-pixel halo (23 KB window, two
// blocks per CU) and its B-layout window reads feeding MFMA directly (the weights packed as a DCN
// weight). Output NHWC (the next DCN's input) and optionally NCHW.
namespace c3 {
constexpr int HALO = 1;
constexpr int WR = dcn::WAVES + 2 * HALO, WC = dcn::TW + 2 * HALO;
constexpr int WIN4 = WR * WC * 8;
constexpr int STAGE = (WIN4 + 511) / 512;
}  // namespace c3

__global__ __launch_bounds__(512) void conv3x3_window_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ wpk,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ shift, int relu, int B, int H,
                                                             int W, float* __restrict__ out,
                                                             float* __restrict__ out_nhwc) {
  constexpr int NA4 = 9 * 2 * 2 * 64;
  __shared__ floatx4_t wl[NA4];
  __shared__ floatx4_t win[c3::WIN4];
  __shared__ __attribute__((aligned(16))) float cst[3][32];  // bias, BN alpha, BN shift (as the DCN's)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < NA4; i += 512) wl[i] = reinterpret_cast<const floatx4_t*>(wpk)[i];
  if (tid < 32) {
    cst[0][tid] = bias ? bias[tid] : 0.f;
    cst[1][tid] = alpha ? alpha[tid] : 1.f;
    cst[2][tid] = alpha ? shift[tid] : 0.f;
  }
  const int HW = H * W, nbx = (W + dcn::TW - 1) / dcn::TW, nby = (H + dcn::WAVES - 1) / dcn::WAVES;
  const int nunits = B * nby * nbx;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int u_begin = (int)((long long)nunits * bid / gridDim.x);
  const int u_end = (int)((long long)nunits * (bid + 1) / gridDim.x);
  const int j = lane >> 4, n = lane & 15;
  floatx4_t stg[c3::STAGE];
  auto fetch = [&](int u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    const int wy0 = band * dcn::WAVES - c3::HALO, wx0 = xs * dcn::TW - c3::HALO;
    const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)b * HW * dcn::CI, (unsigned)HW * dcn::CI * 4);
#pragma unroll
    for (int i = 0; i < c3::STAGE; ++i) {
      const int idx = min(tid + 512 * i, c3::WIN4 - 1), pix = idx >> 3, ch = idx & 7;
      const int r = pix / c3::WC, c = pix - r * c3::WC;
      const int gy = wy0 + r, gx = wx0 + c;
      const bool ok = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      stg[i] = buf_load_f32x4(rx, ok ? ((unsigned)(gy * W + gx) * dcn::CI + 4u * ch) * 4u : kOffOut);
    }
  };
  if (u_begin < u_end) fetch(u_begin);
  for (int u = u_begin; u < u_end; ++u) {
    const int b = u / (nby * nbx), rem = u - b * (nby * nbx), band = rem / nbx, xs = rem - band * nbx;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < c3::STAGE; ++i) {
      const int idx = tid + 512 * i;
      if (idx < c3::WIN4) win[dcn_slot(idx >> 3, idx & 7)] = stg[i];
    }
    __syncthreads();
    if (u + 1 < u_end) fetch(u + 1);
    const int row = band * dcn::WAVES + wv;
    const int x0t = xs * dcn::TW, nvalid = min(dcn::TW, W - x0t);
    if (row >= H) continue;
    floatx4_t acc[2] = {floatx4_t{0.f, 0.f, 0.f, 0.f}, floatx4_t{0.f, 0.f, 0.f, 0.f}};
    // tap k + 1's fragments are read during tap k's MFMAs (the DCN's offset conv does the same)
    floatx4_t fb[2][2], fa[2][2][2];
    auto frag = [&](int k, int bf) {
      const int ki = k / 3, kj = k - 3 * ki;
      const int P = (wv + c3::HALO + ki - 1) * c3::WC + c3::HALO + n + kj - 1;
      fb[bf][0] = win[dcn_slot(P, j)];
      fb[bf][1] = win[dcn_slot(P, j + 4)];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        fa[bf][m][0] = wl[((k * 2 + m) * 2 + 0) * 64 + lane];
        fa[bf][m][1] = wl[((k * 2 + m) * 2 + 1) * 64 + lane];
      }
    };
    frag(0, 0);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (k < 8) frag(k + 1, (k + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const floatx4_t b0 = fb[k & 1][0], b1 = fb[k & 1][1];
      const floatx4_t(&a)[2][2] = fa[k & 1];
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m)
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s >> 2][s & 3], s < 4 ? b0[s] : b1[s - 4], acc[m], 0, 0,
                                                        0);
    }
    if (n < nvalid) {
      const int pq = row * W + x0t + n;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int co0 = 16 * m + 4 * j;
        const floatx4_t cb = *reinterpret_cast<const floatx4_t*>(&cst[0][co0]);
        const floatx4_t ca = *reinterpret_cast<const floatx4_t*>(&cst[1][co0]);
        const floatx4_t cs = *reinterpret_cast<const floatx4_t*>(&cst[2][co0]);
        float r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float y = acc[m][i];
          if (bias) y = y + cb[i];
          if (alpha) y = fmaf(y, ca[i], cs[i]);
          if (relu & 1) y = fmaxf(y, 0.f);
          r[i] = y;
          if (out) out[((size_t)b * 32 + co0 + i) * HW + pq] = y;
        }
        if (out_nhwc) {
          float4* op = reinterpret_cast<float4*>(out_nhwc + ((size_t)b * HW + pq) * 32 + co0);
          if (relu & 2) {  // accumulate (tmvs_conv3x3_nhwc_acc): out + conv, the operand order of out += conv
            const float4 o = *op;
            r[0] = o.x + r[0];
            r[1] = o.y + r[1];
            r[2] = o.z + r[2];
            r[3] = o.w + r[3];
          }
          *op = make_float4(r[0], r[1], r[2], r[3]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// FPN merge of FeatureNet.forward (models/module.py:409-417):
//   intra = interpolate(prev, scale 2, nearest) + inner(lat)      inner = Conv2d(cl, 32, 1, bias=True)
// NHWC in and out: prev [B][h][w][32], lat [B][2h][2w][cl], out [B][2h][2w][32]. Four lanes per
// pixel, 8 output channels each; inner's weights/bias in LDS. HBM-bound elementwise work.
template <int CL>
__global__ __launch_bounds__(256) void fpn_merge_kernel(const float* __restrict__ prev, const float* __restrict__ lat,
                                                        const float* __restrict__ wi, const float* __restrict__ bi,
                                                        int B, int h, int w, float* __restrict__ out) {
  __shared__ float ws[32 * CL + 32];
  for (int i = threadIdx.x; i < 32 * CL; i += 256) ws[i] = wi[i];  // [co][ci]
  if (threadIdx.x < 32) ws[32 * CL + threadIdx.x] = bi[threadIdx.x];
  __syncthreads();
  const int H2 = 2 * h, W2 = 2 * w;
  const long long npix = (long long)B * H2 * W2;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long pix = t >> 2;
  if (pix >= npix) return;
  const int g = (int)(t & 3);  // output channels 8g .. 8g+7
  const int b = (int)(pix / ((long long)H2 * W2));
  const int rem = (int)(pix - (long long)b * H2 * W2), y = rem / W2, xx = rem - y * W2;
  float lv[CL];
#pragma unroll
  for (int c = 0; c < CL; c += 4) {
    const float4 v = *reinterpret_cast<const float4*>(lat + pix * CL + c);
    lv[c] = v.x; lv[c + 1] = v.y; lv[c + 2] = v.z; lv[c + 3] = v.w;
  }
  const float* pv = prev + (((size_t)b * h + (y >> 1)) * w + (xx >> 1)) * 32 + 8 * g;
  const float4 p0 = *reinterpret_cast<const float4*>(pv), p1 = *reinterpret_cast<const float4*>(pv + 4);
  const float up[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
  float r[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    const int co = 8 * g + o;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < CL; ++c) acc = fmaf(ws[co * CL + c], lv[c], acc);
    r[o] = up[o] + (acc + ws[32 * CL + co]);
  }
  float* ov = out + pix * 32 + 8 * g;
  *reinterpret_cast<float4*>(ov) = make_float4(r[0], r[1], r[2], r[3]);
  *reinterpret_cast<float4*>(ov + 4) = make_float4(r[4], r[5], r[6], r[7]);
}

}  // namespace tmvs

using namespace tmvs;

extern "C" size_t tmvs_deform_conv2d_packed_floats(int cout) { return (size_t)9 * 8 * ((cout + 15) / 16) * 64; }

// A fragments in the kernel's LDS order [tap k][m-tile][half h][lane l][e], k-step s = 4h + e:
// lane l holds W[co = 16m + (l & 15)][ci = 16h + 4 (l >> 4) + e][k] (zero for co >= cout).
// cout 8 / 16 / 32: a DCN weight; 27: a conv_offset_mask weight (for tmvs_dcn_fused).
extern "C" int tmvs_deform_conv2d_pack(const float* weight, int cout, int cin, float* packed) {
  if (!weight || !packed || cin != dcn::CI || (cout != 8 && cout != 16 && cout != 27 && cout != 32))
    return TMVS_ERR_ARG;
  const int mt_n = (cout + 15) / 16;
  for (int k = 0; k < 9; ++k)
    for (int mt = 0; mt < mt_n; ++mt)
      for (int h = 0; h < 2; ++h)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 4; ++e) {
            const int co = 16 * mt + (l & 15), ci = 16 * h + 4 * (l >> 4) + e;
            packed[((((size_t)k * mt_n + mt) * 2 + h) * 64 + l) * 4 + e] =
                co < cout ? weight[((size_t)co * cin + ci) * 9 + k] : 0.f;
          }
  return TMVS_OK;
}

namespace {

// The DCN unit: TMVS_DCN_NW waves (rows) per workgroup with a TMVS_DCN_HALO-pixel window margin
#ifndef TMVS_DCN_NW
#define TMVS_DCN_NW 12
#endif
#ifndef TMVS_DCN_HALO
#define TMVS_DCN_HALO 3
#endif
template <int CO, bool FUSED>
int dcn_launch(const float* x, const float* om, const float* wom, const float* bom, const float* w,
               const float* bias, const float* alpha, const float* shift, int relu, int batch, int height, int width,
               float* out, float* out_nhwc, hipStream_t st, float* om_out = nullptr) {
  constexpr int NW = TMVS_DCN_NW, HL = TMVS_DCN_HALO;
  // persistent grid: one block per CU slot the kernel's LDS/VGPR footprint allows
  static int grid = 0;
  if (!grid) {
    int dev = 0, ncu = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TMVS_ERR_HIP;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, dcn_window_kernel<CO, FUSED, NW, HL>, NW * 64, 0);
    grid = std::max(1, ncu * std::max(occ, 1));
  }
  const long long nunits = (long long)batch * ((height + NW - 1) / NW) * ((width + dcn::TW - 1) / dcn::TW);
  const int nblk = (int)std::min<long long>(grid, nunits);
  hipLaunchKernelGGL((dcn_window_kernel<CO, FUSED, NW, HL>), dim3(nblk), dim3(NW * 64), 0, st, x, om, wom, bom, w,
                     bias, alpha, shift, relu, batch, height, width, out, out_nhwc, om_out);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

int dcn_check(const float* x_nhwc, const float* w_packed, const float* bias, const float* bn_alpha,
              const float* bn_shift, int batch, int cin, int cout, int height, int width) {
  if (!x_nhwc || !w_packed || !bias || batch <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if ((bn_alpha == nullptr) != (bn_shift == nullptr)) return TMVS_ERR_ARG;
  if (cin != dcn::CI || (cout != 8 && cout != 16 && cout != 32)) return TMVS_ERR_SHAPE;
  if ((long long)height * width * cin * 4 >= (1LL << 31) || height > 32766 || width > 32766) return TMVS_ERR_SHAPE;
  return TMVS_OK;
}

}  // namespace

extern "C" int tmvs_deform_conv2d(const float* x_nhwc, const float* offset_mask, const float* w_packed,
                                  const float* bias, const float* bn_alpha, const float* bn_shift, int relu,
                                  int batch, int cin, int cout, int height, int width, float* out,
                                  float* out_nhwc, void* stream) {
  if (!offset_mask || !out) return TMVS_ERR_ARG;
  const int rc = dcn_check(x_nhwc, w_packed, bias, bn_alpha, bn_shift, batch, cin, cout, height, width);
  if (rc != TMVS_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (cout == 32)
    return dcn_launch<32, false>(x_nhwc, offset_mask, nullptr, nullptr, w_packed, bias, bn_alpha, bn_shift, relu,
                                 batch, height, width, out, out_nhwc, st);
  if (cout == 16)
    return dcn_launch<16, false>(x_nhwc, offset_mask, nullptr, nullptr, w_packed, bias, bn_alpha, bn_shift, relu,
                                 batch, height, width, out, out_nhwc, st);
  return dcn_launch<8, false>(x_nhwc, offset_mask, nullptr, nullptr, w_packed, bias, bn_alpha, bn_shift, relu, batch,
                              height, width, out, out_nhwc, st);
}

extern "C" int tmvs_dcn_forward_train(const float* x_nhwc, const float* wom_packed, const float* bom,
                                      const float* w_packed, const float* bias, int batch, int cin, int cout, int height,
                                      int width, float* out, float* out_nhwc, float* offset_mask_out, void* stream) {
  if (!wom_packed || !bom || !offset_mask_out || (!out && !out_nhwc)) return TMVS_ERR_ARG;
  const int rc = dcn_check(x_nhwc, w_packed, bias, nullptr, nullptr, batch, cin, cout, height, width);
  if (rc != TMVS_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (cout == 32)
    return dcn_launch<32, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, nullptr, nullptr, 0, batch, height,
                                width, out, out_nhwc, st, offset_mask_out);
  if (cout == 16)
    return dcn_launch<16, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, nullptr, nullptr, 0, batch, height,
                                width, out, out_nhwc, st, offset_mask_out);
  return dcn_launch<8, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, nullptr, nullptr, 0, batch, height,
                             width, out, out_nhwc, st, offset_mask_out);
}

extern "C" int tmvs_dcn_fused(const float* x_nhwc, const float* wom_packed, const float* bom, const float* w_packed,
                              const float* bias, const float* bn_alpha, const float* bn_shift, int relu, int batch,
                              int cin, int cout, int height, int width, float* out, float* out_nhwc, void* stream) {
  if (!wom_packed || !bom || (!out && !out_nhwc)) return TMVS_ERR_ARG;
  const int rc = dcn_check(x_nhwc, w_packed, bias, bn_alpha, bn_shift, batch, cin, cout, height, width);
  if (rc != TMVS_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (cout == 32)
    return dcn_launch<32, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, bn_alpha, bn_shift, relu, batch,
                                height, width, out, out_nhwc, st);
  if (cout == 16)
    return dcn_launch<16, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, bn_alpha, bn_shift, relu, batch,
                                height, width, out, out_nhwc, st);
  return dcn_launch<8, true>(x_nhwc, nullptr, wom_packed, bom, w_packed, bias, bn_alpha, bn_shift, relu, batch,
                             height, width, out, out_nhwc, st);
}

static int conv3x3_launch(const float* x_nhwc, const float* w_packed, const float* bias, const float* bn_alpha,
                          const float* bn_shift, int flags, int batch, int height, int width, float* out,
                          float* out_nhwc, void* stream) {
  if ((long long)height * width * 32 * 4 >= (1LL << 31)) return TMVS_ERR_SHAPE;
  static int grid = 0;
  if (!grid) {
    int dev = 0, ncu = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TMVS_ERR_HIP;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv3x3_window_kernel, 512, 0);
    grid = std::max(1, ncu * std::max(occ, 1));
  }
  const long long nunits =
      (long long)batch * ((height + dcn::WAVES - 1) / dcn::WAVES) * ((width + dcn::TW - 1) / dcn::TW);
  const int nblk = (int)std::min<long long>(grid, nunits);
  hipLaunchKernelGGL(conv3x3_window_kernel, dim3(nblk), dim3(512), 0, (hipStream_t)stream, x_nhwc, w_packed, bias,
                     bn_alpha, bn_shift, flags, batch, height, width, out, out_nhwc);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" int tmvs_conv3x3_nhwc(const float* x_nhwc, const float* w_packed, const float* bias, const float* bn_alpha,
                                 const float* bn_shift, int relu, int batch, int cin, int cout, int height, int width,
                                 float* out, float* out_nhwc, void* stream) {
  if (!x_nhwc || !w_packed || (!out && !out_nhwc) || batch <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if ((bn_alpha == nullptr) != (bn_shift == nullptr)) return TMVS_ERR_ARG;
  if (cin != 32 || cout != 32) return TMVS_ERR_SHAPE;
  return conv3x3_launch(x_nhwc, w_packed, bias, bn_alpha, bn_shift, relu ? 1 : 0, batch, height, width, out, out_nhwc,
                        stream);
}

// out_nhwc += conv3x3(x_nhwc) (no bias / BN / ReLU): the FeatureNet backward's data gradient of a 3x3 conv
// added into an existing gradient in the conv's epilogue instead of a separate add pass
extern "C" int tmvs_conv3x3_nhwc_acc(const float* x_nhwc, const float* w_packed, int batch, int cin, int cout,
                                     int height, int width, float* out_nhwc, void* stream) {
  if (!x_nhwc || !w_packed || !out_nhwc || batch <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (cin != 32 || cout != 32) return TMVS_ERR_SHAPE;
  return conv3x3_launch(x_nhwc, w_packed, nullptr, nullptr, nullptr, 2, batch, height, width, nullptr, out_nhwc,
                        stream);
}

extern "C" int tmvs_fpn_merge(const float* prev_nhwc, const float* lat_nhwc, int lat_channels, const float* w_inner,
                              const float* b_inner, int batch, int height, int width, float* out_nhwc, void* stream) {
  if (!prev_nhwc || !lat_nhwc || !w_inner || !b_inner || !out_nhwc || batch <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  if (lat_channels != 8 && lat_channels != 16) return TMVS_ERR_SHAPE;
  const long long threads = (long long)batch * 4 * height * width * 4;
  if (threads / 256 + 1 >= (1LL << 31)) return TMVS_ERR_SHAPE;
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (lat_channels == 8)
    hipLaunchKernelGGL(fpn_merge_kernel<8>, grid, dim3(256), 0, (hipStream_t)stream, prev_nhwc, lat_nhwc, w_inner,
                       b_inner, batch, height, width, out_nhwc);
  else
    hipLaunchKernelGGL(fpn_merge_kernel<16>, grid, dim3(256), 0, (hipStream_t)stream, prev_nhwc, lat_nhwc, w_inner,
                       b_inner, batch, height, width, out_nhwc);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
