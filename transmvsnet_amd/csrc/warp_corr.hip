// Fused cost-volume build for one cascade stage (DepthNet steps 1-2,
// reference models/TransMVSNet.py:58-93 and homo_warping models/module.py:284-322).
//
// A pixel is owned by C/4 adjacent lanes (see warp_corr_kernel); per source view they project
// the pixel's depth planes into the view, bilinearly sample the channels-last source features
// (one contiguous C*4-byte row per tap per lane group) and form the single-group correlation
// against the reference features held in registers; the warped [C,D,H,W] volume never exists.
//
// fp32 op order follows the reference's PyTorch-CPU kernels (DESIGN.md "Numerics"):
//   rot·(x,y,1)   : fmaf(r1, y, r0*x) + r2            (bmm as MKL runs it on AVX-512 Xeons: FMA chain)
//               or (r0*x + r1*y) + r2                  (bmm as MKL runs it on AMD EPYC: TMVS_WARP_ROT_PLAIN)
//   X = rot_xyz*d + t ; px = X/Z ; xn = px/((W-1)/2) - 1 ; z < 1e-6 -> xn = yn = -99
//   ix = (xn + 1) * ((W-1)/2)                          (grid_sample, align_corners=True)
//   v  = fmaf(se_v,se, fmaf(sw_v,sw, fmaf(ne_v,ne, nw_v*nw)))  (zeros padding)
//   sim = (Σ_c v_c*ref_c) / C ; sim_sum += sim*w ; w_sum = 1e-5 + Σ w ; sim_sum / w_sum
// (the channel sum: serial within each lane's 4 channels, then a fixed xor tree over lanes)
#include "common.h"

namespace tmvs {

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct WarpArgs {
  float proj[TMVS_MAX_VIEWS][12];
  float pw[TMVS_PW_NPARAMS];
  int rot_plain;  // TMVS_WARP_ROT_PLAIN: the host BLAS's rounding of rot·(x, y, 1)
};

// One row of rot·(x, y, 1) (homo_warping's torch.matmul, models/module.py:303) in the op order of
// the host BLAS the reference runs on: MKL contracts it into an FMA chain on AVX-512 Xeons and does
// not on AMD EPYC (measured, scripts/diag/warp_bits.py); the coordinate then differs by up to 1.2e-4.
__device__ __forceinline__ float rot_row(const float* R, float x, float y, int plain) {
  return plain ? (R[0] * x + R[1] * y) + R[2] : fmaf(R[1], y, R[0] * x) + R[2];
}

__device__ __forceinline__ float pixelwise_logit(float s, const float* __restrict__ pw) {
  // PixelwiseNet (TransMVSNet.py:20-26): 1x1x1 convs 1->16 (BN,ReLU) ->8 (BN,ReLU) ->1 (+bias).
  // pw is in LDS; the hidden-unit loop is not unrolled so the 201 parameters are re-read
  // (broadcast ds_read_b128) rather than hoisted into VGPRs.
  const float* w0 = pw;
  const float* a0 = pw + 16;
  const float* s0 = pw + 32;
  const float* w1 = pw + 48;
  const float* a1 = pw + 176;
  const float* s1 = pw + 184;
  const float* w2 = pw + 192;
  float h0[16];
#pragma unroll
  for (int o4 = 0; o4 < 4; ++o4) {
    const float4 w = reinterpret_cast<const float4*>(w0)[o4];
    const float4 a = reinterpret_cast<const float4*>(a0)[o4];
    const float4 sh = reinterpret_cast<const float4*>(s0)[o4];
    h0[4 * o4 + 0] = relu(fmaf(w.x * s, a.x, sh.x));
    h0[4 * o4 + 1] = relu(fmaf(w.y * s, a.y, sh.y));
    h0[4 * o4 + 2] = relu(fmaf(w.z * s, a.z, sh.z));
    h0[4 * o4 + 3] = relu(fmaf(w.w * s, a.w, sh.w));
  }
  float out = 0.f;
#pragma unroll 1
  for (int p = 0; p < 8; ++p) {
    float acc = 0.f;
#pragma unroll
    for (int o4 = 0; o4 < 4; ++o4) {
      const float4 w = reinterpret_cast<const float4*>(w1 + p * 16)[o4];
      acc = fmaf(w.x, h0[4 * o4 + 0], acc);
      acc = fmaf(w.y, h0[4 * o4 + 1], acc);
      acc = fmaf(w.z, h0[4 * o4 + 2], acc);
      acc = fmaf(w.w, h0[4 * o4 + 3], acc);
    }
    out = fmaf(w2[p], relu(fmaf(acc, a1[p], s1[p])), out);
  }
  return out + pw[200];
}

// Lane layout: a pixel is served by LPS = C/4 adjacent lanes ("group"); lane k of the group
// owns channel quad k (4 channels, one 16-byte load per tap) and depth planes j*LPS + k.
// Each lane projects only its own planes. For plane slot j the group runs LPS rounds: in
// round t all lanes take plane t's tap geometry (broadcast from lane t: DPP quad permute, or
// ds_swizzle for groups of 8 -- no LDS memory traffic) and load their channel quad of the
// four taps, so the C channels of a tap arrive as one contiguous C*4-byte row per group and a
// wave-instruction touches 64/LPS full rows (measured: anything that splits a row over
// several instructions, or mixes planes inside a group, costs up to 2x). All rounds' loads
// are issued before any is consumed; a butterfly reduce-scatter then gives lane t the full
// channel sum of plane t.
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
  x0i = (int)fminf(fmaxf(x0, -2.f), 32766.f);
  y0i = (int)fminf(fmaxf(y0, -2.f), 32766.f);
}

// x from lane (lane ^ R) inside an aligned group of 8 (R compile-time)
template <int R>
__device__ __forceinline__ int lane_xor(int x) {
  if constexpr (R == 0) return x;
  else if constexpr (R == 1) return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  else if constexpr (R == 2) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  else if constexpr (R == 3) return __builtin_amdgcn_mov_dpp(x, 0x1B, 0xF, 0xF, false);  // quad_perm [3,2,1,0]
  else return __builtin_amdgcn_ds_swizzle(x, 0x1F | (R << 10));                           // bit mode, xor R
}
template <int R>
__device__ __forceinline__ float lane_xor_f(float x) {
  return __int_as_float(lane_xor<R>(__float_as_int(x)));
}

template <int LPS>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (LPS >= 2) v = fmaxf(v, lane_xor_f<1>(v));
  if constexpr (LPS >= 4) v = fmaxf(v, lane_xor_f<2>(v));
  if constexpr (LPS >= 8) v = fmaxf(v, lane_xor_f<4>(v));
  return v;
}

// Buffer resource over one sample's source views: raw (stride 0) addressing with 32-bit byte
// offsets. An offset at or past num_records reads as 0 -- exactly grid_sample's zero padding --
// so an out-of-image tap only needs an out-of-range offset: each axis term is kAxisOut when
// invalid, and any sum containing one is >= kAxisOut >= num_records (< 2^30, checked).
constexpr unsigned kAxisOut = 0x40000000u;

struct Geom {
  int x0, y0;
  float fx, fy;
};

// x from lane t of this lane's aligned group of LPS lanes (t compile-time): the group's
// lanes all receive the same value -- DPP quad permutes for LPS <= 4, ds_swizzle (bit mode,
// no memory access) for LPS = 8
template <int LPS, int T>
__device__ __forceinline__ int group_bcast(int x) {
  if constexpr (LPS == 1) return x;
  else if constexpr (LPS == 2) return __builtin_amdgcn_mov_dpp(x, T | (T << 2) | ((T + 2) << 4) | ((T + 2) << 6), 0xF, 0xF, false);
  else if constexpr (LPS == 4) return __builtin_amdgcn_mov_dpp(x, T * 0x55, 0xF, 0xF, false);
  else return __builtin_amdgcn_ds_swizzle(x, 0x18 | (T << 5));  // lane' = (lane & 0x18) | T
}

template <int LPS, int T>
__device__ __forceinline__ Geom geom_bcast(const Geom& g) {
  return Geom{group_bcast<LPS, T>(g.x0), group_bcast<LPS, T>(g.y0),
              __int_as_float(group_bcast<LPS, T>(__float_as_int(g.fx))),
              __int_as_float(group_bcast<LPS, T>(__float_as_int(g.fy)))};
}


// Tap reuse across consecutive planes. A pixel's depth planes project to nearby points on the
// epipolar line, so consecutive planes mostly share bilinear taps (unique taps per pixel-view,
// synthetic DTU rig: 129 / 48 / 14 of 192 / 128 / 32 tap loads in stages 1 / 2 / 3). The 4
// taps of a plane always occupy the 4 (x parity, y parity) classes, so tap (X, Y) is cached in
// register slot (X&1, Y&1) with its position as tag: a plane loads only the slots whose tag
// changed. The address unit's cost scales with the lanes that make a memory request (measured,
// scripts/micro/ta_mask.hip: exec-masked and out-of-range lanes are equally free), so skipped
// loads are skipped work.
struct Slots {
  floatx4 v[4];
  unsigned pos[4];
};

__device__ __forceinline__ void slots_reset(Slots& S) {
#pragma unroll
  for (int s = 0; s < 4; ++s) S.pos[s] = 0xFFFFFFFFu;  // no position packs to this
}

template <int C>
__device__ __forceinline__ void fetch_reuse(const __amdgpu_buffer_rsrc_t rsrc, unsigned vbase, unsigned rowb, int W,
                                            int H, const Geom& g, Slots& S, floatx4 (&val)[4], float (&w)[4]) {
  constexpr unsigned CB = C * 4;
  const float we = g.fx, n = g.fy;
  const float ea = 1.f - we, s = 1.f - n;
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    const int px = sl & 1, py = sl >> 1;
    const int X = g.x0 + ((g.x0 ^ px) & 1), Y = g.y0 + ((g.y0 ^ py) & 1);
    const unsigned key = (unsigned)(X + 2) | ((unsigned)(Y + 2) << 16);  // X, Y in [-2, 32767]
    // branch-free: a lane whose slot still holds the tap issues the load with an out-of-range
    // offset (no memory request; costs the address unit what an exec-masked lane costs, measured)
    const bool need = key != S.pos[sl];
    S.pos[sl] = key;
    const bool inside = (unsigned)X < (unsigned)W && (unsigned)Y < (unsigned)H;  // outside: reads 0
    const unsigned off = (need && inside) ? vbase + (unsigned)Y * rowb + (unsigned)X * CB : kOffOut;
    const floatx4 ld = buf_load_f32x4(rsrc, off);
    S.v[sl] = need ? ld : S.v[sl];
    val[sl] = S.v[sl];
    // grid_sample's weights: (y weight) * (x weight), nw = (1-fy)(1-fx) ...
    w[sl] = ((Y == g.y0) ? s : n) * ((X == g.x0) ? ea : we);
  }
}

// Without the cache (stage 1: uniform planes ~1.4 px apart share few taps): the 4 taps in
// grid_sample's order nw, ne, sw, se, so the interpolation's fma chain is the reference's.
template <int C>
__device__ __forceinline__ void fetch_full(const __amdgpu_buffer_rsrc_t rsrc, unsigned vbase, unsigned rowb, int W,
                                           int H, const Geom& g, floatx4 (&val)[4], float (&w)[4]) {
  constexpr unsigned CB = C * 4;
  const float we = g.fx, n = g.fy;
  const float ea = 1.f - we, s = 1.f - n;
  w[0] = s * ea;
  w[1] = s * we;
  w[2] = n * ea;
  w[3] = n * we;
  const unsigned xa = (unsigned)g.x0 < (unsigned)W ? (unsigned)g.x0 * CB : kAxisOut;
  const unsigned xb = (unsigned)(g.x0 + 1) < (unsigned)W ? (unsigned)(g.x0 + 1) * CB : kAxisOut;
  const unsigned yrow = vbase + (unsigned)g.y0 * rowb;
  const unsigned ya = (unsigned)g.y0 < (unsigned)H ? yrow : kAxisOut;
  const unsigned yb = (unsigned)(g.y0 + 1) < (unsigned)H ? yrow + rowb : kAxisOut;
  val[0] = buf_load_f32x4(rsrc, ya + xa);
  val[1] = buf_load_f32x4(rsrc, ya + xb);
  val[2] = buf_load_f32x4(rsrc, yb + xa);
  val[3] = buf_load_f32x4(rsrc, yb + xb);
}

// bilinear value of each channel (fixed slot order), times ref, summed in channel order
__device__ __forceinline__ float combine(const floatx4 (&v)[4], const float (&w)[4], const float4& r4) {
  float acc = 0.f;
  acc = acc + fmaf(v[3][0], w[3], fmaf(v[2][0], w[2], fmaf(v[1][0], w[1], v[0][0] * w[0]))) * r4.x;
  acc = acc + fmaf(v[3][1], w[3], fmaf(v[2][1], w[2], fmaf(v[1][1], w[1], v[0][1] * w[0]))) * r4.y;
  acc = acc + fmaf(v[3][2], w[3], fmaf(v[2][2], w[2], fmaf(v[1][2], w[1], v[0][2] * w[0]))) * r4.z;
  acc = acc + fmaf(v[3][3], w[3], fmaf(v[2][3], w[2], fmaf(v[1][3], w[1], v[0][3] * w[0]))) * r4.w;
  return acc;
}

// Rounds R0..R0+N-1: in round t the whole group samples plane slot t (geometry broadcast from
// lane t), so each load instruction covers one contiguous C*4-byte row per group. Every
// round's (masked) loads are issued before any is consumed.
template <int C, bool REUSE, int R0, int N>
__device__ __forceinline__ void rounds(const __amdgpu_buffer_rsrc_t rsrc, unsigned vbase, unsigned rowb, int W,
                                       int H, const Geom& own, const float4& r4, Slots& S, float* part) {
  floatx4 v[N][4];
  float w[N][4];
#define TMVS_FETCH(I)                                                                          \
  if constexpr (REUSE)                                                                         \
    fetch_reuse<C>(rsrc, vbase, rowb, W, H, geom_bcast<C / 4, R0 + I>(own), S, v[I], w[I]); \
  else                                                                                         \
    fetch_full<C>(rsrc, vbase, rowb, W, H, geom_bcast<C / 4, R0 + I>(own), v[I], w[I]);
  TMVS_FETCH(0)
  if constexpr (N > 1) { TMVS_FETCH(1) }
  if constexpr (N > 2) { TMVS_FETCH(2) }
  if constexpr (N > 3) { TMVS_FETCH(3) }
#undef TMVS_FETCH
#pragma unroll
  for (int i = 0; i < N; ++i) part[R0 + i] = combine(v[i], w[i], r4);
}

// Full channel sum of this lane's own plane (slot k): LPS rounds, then a butterfly
// reduce-scatter over lane bits (xor 4, xor 2, xor 1). At each step a lane keeps the half of
// the planes whose slot bit matches its own lane bit and sends the other half to its partner;
// the sum for slot t ends in lane t: no dependent shuffle chains, LPS-1 exchanges.
template <int C, bool REUSE>
__device__ __forceinline__ float plane_corr(const __amdgpu_buffer_rsrc_t rsrc, unsigned vbase, unsigned rowb, int W,
                                            int H, const Geom& own, const float4& r4, int k, Slots& S) {
  constexpr int LPS = C / 4;
  float p[LPS];
  if constexpr (REUSE) {
    // batches of 2 rounds: the cached slots plus a batch's loads fit the VGPR budget
    rounds<C, true, 0, 2>(rsrc, vbase, rowb, W, H, own, r4, S, p);
    if constexpr (LPS >= 4) {
      __builtin_amdgcn_sched_barrier(0);
      rounds<C, true, 2, 2>(rsrc, vbase, rowb, W, H, own, r4, S, p);
    }
    if constexpr (LPS >= 8) {
      __builtin_amdgcn_sched_barrier(0);
      rounds<C, true, 4, 2>(rsrc, vbase, rowb, W, H, own, r4, S, p);
      __builtin_amdgcn_sched_barrier(0);
      rounds<C, true, 6, 2>(rsrc, vbase, rowb, W, H, own, r4, S, p);
    }
  } else if constexpr (LPS <= 4) {
    rounds<C, false, 0, LPS>(rsrc, vbase, rowb, W, H, own, r4, S, p);
  } else {
    rounds<C, false, 0, 4>(rsrc, vbase, rowb, W, H, own, r4, S, p);
    rounds<C, false, 4, 4>(rsrc, vbase, rowb, W, H, own, r4, S, p);
  }
  float q[LPS];
#pragma unroll
  for (int i = 0; i < LPS; ++i) q[i] = p[i];
  int n = LPS;
  if constexpr (LPS >= 8) {
    const bool hi = (k & 4) != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float keep = hi ? q[4 + i] : q[i], send = hi ? q[i] : q[4 + i];
      q[i] = keep + lane_xor_f<4>(send);
    }
    n = 4;
  }
  if constexpr (LPS >= 4) {
    const bool hi = (k & 2) != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = hi ? q[2 + i] : q[i], send = hi ? q[i] : q[2 + i];
      q[i] = keep + lane_xor_f<2>(send);
    }
    n = 2;
  }
  (void)n;
  if constexpr (LPS >= 2) {
    const bool hi = (k & 1) != 0;
    const float keep = hi ? q[1] : q[0], send = hi ? q[0] : q[1];
    q[0] = keep + lane_xor_f<1>(send);
  }
  return q[0];
}

// Views outer (a view's consecutive planes hit the same source lines: L1 reuse), planes inner
// and not unrolled: the plane's depth and running weighted sum live in this thread's LDS
// column, so the rounds' independent loads are the only large live set.
template <int C, int D, bool PW, bool PARTIAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void warp_corr_kernel(
    const float* __restrict__ ref, const float* __restrict__ src, const float* __restrict__ hyp,
    const float* __restrict__ vw_in, float* __restrict__ sim_out, float* __restrict__ wsum_out,
    float* __restrict__ vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total, WarpArgs args) {
  constexpr int LPS = C / 4;          // lanes per pixel
  constexpr int SPW = 64 / LPS;       // pixels per wave
  constexpr int PIX = 4 * SPW;        // pixels per block
  constexpr int DPT = D / LPS;        // depth planes owned per lane
  static_assert(D % LPS == 0, "D must be a multiple of C/4");
  // PixelwiseNet parameters in LDS (uniform-address reads broadcast); as kernel arguments
  // they would occupy ~200 SGPRs and spill
  __shared__ __attribute__((aligned(16))) float pw_lds[PW ? TMVS_PW_NPARAMS + 3 : 4];
  __shared__ float dep_lds[DPT][256];
  __shared__ float acc_lds[DPT][256];
  __shared__ float sim_lds[PW ? DPT : 1][PW ? 256 : 1];
  const int tid = threadIdx.x;
  if constexpr (PW) {
    if (tid < TMVS_PW_NPARAMS) pw_lds[tid] = args.pw[tid];
  }
  const int HW = H * W;
  const int nblk = (HW + PIX - 1) / PIX;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int lane = tid & 63;
  const int k = lane % LPS;
  int p = tile * PIX + (tid >> 6) * SPW + lane / LPS;
  const bool active = p < HW;
  if (!active) p = HW - 1;
  const int py = p / W, px = p - py * W;
  const float fxp = (float)px, fyp = (float)py;
  const float4 r4 = *reinterpret_cast<const float4*>(ref + (size_t)p * C + 4 * k);
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    dep_lds[j][tid] = hyp[(size_t)(j * LPS + k) * HW + p];
    acc_lds[j][tid] = 0.f;
  }
  if constexpr (PW) __syncthreads();  // pw_lds is shared; the columns are per thread
  const float halfw = (float)(W - 1) / 2.f;
  const float halfh = (float)(H - 1) / 2.f;
  float wsum = PARTIAL ? 0.f : 1e-5f;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, V * HW * C * 4, kRsrcWord3);
  const unsigned rowb = (unsigned)W * C * 4;
  const int Ws = W >> vw_shift, Hs = H >> vw_shift;

  for (int v = 0; v < V; ++v) {
    const float* R = args.proj[v];
    const float rx = rot_row(R, fxp, fyp, args.rot_plain);
    const float ry = rot_row(R + 4, fxp, fyp, args.rot_plain);
    const float rz = rot_row(R + 8, fxp, fyp, args.rot_plain);
    const unsigned vbase = (unsigned)(v * HW * C * 4 + 16 * k);
    float w = 0.f;
    if constexpr (!PW) w = vw_in[(size_t)(vw_offset + v) * Hs * Ws + (py >> vw_shift) * Ws + (px >> vw_shift)];
    float wm = 0.f;  // PW: running max of sigmoid (> 0, so 0 is neutral)
    Slots S;  // tap cache, valid within one view: planes j*LPS + t run in depth order
    slots_reset(S);
#pragma unroll 1
    for (int j = 0; j < DPT; ++j) {
      Geom own;
      project(rx, ry, rz, R[3], R[7], R[11], dep_lds[j][tid], halfw, halfh, own.x0, own.y0, own.fx, own.fy);
      const float sim = plane_corr<C, !PW>(rsrc, vbase, rowb, W, H, own, r4, k, S) * (1.f / (float)C);  // C = 2^n: == / C
      if constexpr (PW) {
        sim_lds[j][tid] = sim;
        int salt = 0;  // opaque offset: keeps the parameter reads from being hoisted into VGPRs
        asm volatile("" : "+v"(salt));
        const float lg = pixelwise_logit(sim, pw_lds + salt);
        wm = fmaxf(wm, 1.f / (1.f + expf(-lg)));
      } else {
        acc_lds[j][tid] = acc_lds[j][tid] + sim * w;
      }
    }
    if constexpr (PW) {
      w = group_max<LPS>(wm);
      if (active && k == 0) vw_out[(size_t)(vw_offset + v) * HW + p] = w;
#pragma unroll 4
      for (int j = 0; j < DPT; ++j) acc_lds[j][tid] = acc_lds[j][tid] + sim_lds[j][tid] * w;
    }
    wsum = wsum + w;
  }
  if (!active) return;
#pragma unroll 4
  for (int j = 0; j < DPT; ++j) {
    const size_t o = (size_t)(j * LPS + k) * HW + p;
    sim_out[o] = PARTIAL ? acc_lds[j][tid] : acc_lds[j][tid] / wsum;
  }
  if (PARTIAL && k == 0) wsum_out[p] = wsum;
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
  const float rx = rot_row(R, fx, fy, args.rot_plain);
  const float ry = rot_row(R + 4, fx, fy, args.rot_plain);
  const float rz = rot_row(R + 8, fx, fy, args.rot_plain);
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

// C = 8 with given view weights (stage 3): "row pair" lane layout. A pixel is served by 4
// lanes k = (tx, q): tx picks the tap column (x0 or x0+1), q the channel quad; in a round the
// group's 4 lanes load one contiguous 64-byte span per tap row (x0 and x0+1, all 8 channels)
// instead of two lanes loading 32-byte rows of different taps, so every lane quad of a load
// instruction stays on one span (measured with the C/4 layout: 48 address-unit cycles per
// instruction, stalled on the L1). Bilinear partial per lane: its column's two taps; the
// reduce-scatter over the 4 lanes then adds the columns and the channel quads.
// geometry of plane slot t (compile-time after unrolling) broadcast from lane t of the group
template <int LPS>
__device__ __forceinline__ Geom geom_round(const Geom& own, int t) {
  if (t == 0) return geom_bcast<LPS, 0>(own);
  if (t == 1) return geom_bcast<LPS, 1>(own);
  if constexpr (LPS > 2) {
    if (t == 2) return geom_bcast<LPS, 2>(own);
    if (t == 3) return geom_bcast<LPS, 3>(own);
  }
  if constexpr (LPS > 4) {
    if (t == 4) return geom_bcast<LPS, 4>(own);
    if (t == 5) return geom_bcast<LPS, 5>(own);
    if (t == 6) return geom_bcast<LPS, 6>(own);
    return geom_bcast<LPS, 7>(own);
  }
  return own;
}

// Row-pair rounds R0..R0+N-1 (see warp_pair_kernel): in round t the group samples plane t;
// this lane loads its tap column's two rows (one 16-byte channel quad each); all loads of the
// batch are issued before any is consumed.
template <int C, int R0, int N>
__device__ __forceinline__ void pair_rounds(const __amdgpu_buffer_rsrc_t rsrc, unsigned vbase, unsigned rowb, int W,
                                            int H, const Geom& own, const float4* r4, int tx, float* part) {
  constexpr int LPS = C / 2;
  floatx4 top[N], bot[N];
  float wt[N], wb[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const Geom g = geom_round<LPS>(own, R0 + i);
    const int X = g.x0 + tx;
    const unsigned ox = (unsigned)X < (unsigned)W ? (unsigned)X * (unsigned)(C * 4) : kAxisOut;
    const unsigned yrow = vbase + (unsigned)g.y0 * rowb;
    const unsigned oa = (unsigned)g.y0 < (unsigned)H ? yrow : kAxisOut;
    const unsigned ob = (unsigned)(g.y0 + 1) < (unsigned)H ? yrow + rowb : kAxisOut;
    top[i] = buf_load_f32x4(rsrc, oa + ox);
    bot[i] = buf_load_f32x4(rsrc, ob + ox);
    const float wx = tx ? g.fx : 1.f - g.fx;
    wt[i] = (1.f - g.fy) * wx;  // grid_sample: (y weight) * (x weight)
    wb[i] = g.fy * wx;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float4 r = r4[R0 + i];
    float acc = 0.f;
    acc = acc + fmaf(bot[i][0], wb[i], top[i][0] * wt[i]) * r.x;
    acc = acc + fmaf(bot[i][1], wb[i], top[i][1] * wt[i]) * r.y;
    acc = acc + fmaf(bot[i][2], wb[i], top[i][2] * wt[i]) * r.z;
    acc = acc + fmaf(bot[i][3], wb[i], top[i][3] * wt[i]) * r.w;
    part[R0 + i] = acc;
  }
}

// Butterfly reduce-scatter over a lane group (xor LPS/2 ... 1): lane k ends with slot k's sum.
template <int LPS>
__device__ __forceinline__ float reduce_scatter(const float* p, int k) {
  float q[LPS];
#pragma unroll
  for (int i = 0; i < LPS; ++i) q[i] = p[i];
  if constexpr (LPS >= 8) {
    const bool hi = (k & 4) != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float keep = hi ? q[4 + i] : q[i], send = hi ? q[i] : q[4 + i];
      q[i] = keep + lane_xor_f<4>(send);
    }
  }
  if constexpr (LPS >= 4) {
    const bool hi = (k & 2) != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = hi ? q[2 + i] : q[i], send = hi ? q[i] : q[2 + i];
      q[i] = keep + lane_xor_f<2>(send);
    }
  }
  if constexpr (LPS >= 2) {
    const bool hi = (k & 1) != 0;
    const float keep = hi ? q[1] : q[0], send = hi ? q[0] : q[1];
    q[0] = keep + lane_xor_f<1>(send);
  }
  return q[0];
}

// Which samples share a load instruction. Plane-major rounds (the original layout): in round t the
// wave's SPW groups sample SPW pixels at one plane each. Pixel-major rounds (TMVS_WARP_PMAJOR, used
// for C = 16): the SPW groups sample PPR = SPW/LPS pixels × LPS consecutive planes each (stage 2:
// 1 pixel × 8 planes), whose taps lie ≈0.7 px apart on one epipolar segment and so share cache lines.
// Group g's round-t sample is owned by its lane t (geometry broadcast as before), so lane (g, k) owns
// pixel k·PPR + g/LPS at planes j·LPS + g%LPS and holds the reference quads of the LPS pixels its
// rounds visit. Each sample's arithmetic (lane roles, channel order, reduce-scatter) is unchanged:
// the outputs are bit-identical either way. Measured (profiles/r13/warp_pmajor_ab.txt, two
// alternating reps in one box): stage 2 345.1 -> 323.3 us, stage 3 247.2 -> 252.1 us (the address
// unit is charged per 4-lane quad, so sharing lines between quads buys little); C = 8 keeps the
// plane-major rounds.
#ifndef TMVS_WARP_PMAJOR
#define TMVS_WARP_PMAJOR 1
#endif
#ifndef TMVS_WARP_PAD
#define TMVS_WARP_PAD 0
#endif

template <int C, int D, bool PARTIAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void warp_pair_kernel(
    const float* __restrict__ ref, const float* __restrict__ src, const float* __restrict__ hyp,
    const float* __restrict__ vw_in, float* __restrict__ sim_out, float* __restrict__ wsum_out, int V, int H, int W,
    int vw_shift, int vw_offset, WarpArgs args) {
  constexpr int NQ = C / 4;             // channel quads
  constexpr int LPS = 2 * NQ;           // lanes per pixel: (tap column, quad)
  constexpr int SPW = 64 / LPS, PIX = 4 * SPW, DPT = D / LPS;
  constexpr bool PM = TMVS_WARP_PMAJOR && C == 16;  // pixel-major rounds
  constexpr int PPR = PM ? SPW / LPS : SPW;          // pixels per round
  static_assert(C == 8 || C == 16, "row-pair layout for 8 or 16 channels");
  static_assert(D % LPS == 0, "D must be a multiple of the lanes per pixel");
  static_assert(!PM || PPR * LPS == SPW, "pixel-major rounds: LPS^2 must divide 64");
  __shared__ float dep_lds[DPT][256];
  __shared__ float acc_lds[DPT][256];
  const int tid = threadIdx.x;
  const int HW = H * W;
#if TMVS_WARP_PAD
  __shared__ float pad_lds[TMVS_WARP_PAD];  // A/B only: dead LDS that caps blocks per CU
  if (H < 0) pad_lds[tid] = 0.f;
#endif
  const int nblk = (HW + PIX - 1) / PIX;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int lane = tid & 63;
  const int k = lane % LPS, tx = k / NQ, q = k % NQ, g = lane / LPS;
  const int wbase = tile * PIX + (tid >> 6) * SPW;
  // owned samples: pixel `p`, planes j·LPS + dsub (pixel-major) or j·LPS + k (plane-major)
  const int pix_own = PM ? k * PPR + g / LPS : g;
  const int dsub = PM ? g % LPS : k;
  int p = wbase + pix_own;
  const bool active = p < HW;
  if (!active) p = HW - 1;
  const int py = p / W, px = p - py * W;
  const float fxp = (float)px, fyp = (float)py;
  float4 r4[LPS];  // reference quad q of the pixel round t samples
#pragma unroll
  for (int t = 0; t < LPS; ++t) {
    const int pt = PM ? min(wbase + t * PPR + g / LPS, HW - 1) : p;
    r4[t] = *reinterpret_cast<const float4*>(ref + (size_t)pt * C + 4 * q);
  }
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    dep_lds[j][tid] = hyp[(size_t)(j * LPS + dsub) * HW + p];
    acc_lds[j][tid] = 0.f;
  }
  const float halfw = (float)(W - 1) / 2.f;
  const float halfh = (float)(H - 1) / 2.f;
  const int Ws = W >> vw_shift, Hs = H >> vw_shift;
  const float* wv = vw_in + (size_t)vw_offset * Hs * Ws + (py >> vw_shift) * Ws + (px >> vw_shift);
  float wsum = PARTIAL ? 0.f : 1e-5f;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, V * HW * C * 4, kRsrcWord3);
  const unsigned rowb = (unsigned)W * C * 4;
  for (int v = 0; v < V; ++v) {
    const float* R = args.proj[v];
    const float rx = rot_row(R, fxp, fyp, args.rot_plain);
    const float ry = rot_row(R + 4, fxp, fyp, args.rot_plain);
    const float rz = rot_row(R + 8, fxp, fyp, args.rot_plain);
    const unsigned vbase = (unsigned)(v * HW * C * 4 + 16 * q);
    const float w = wv[(size_t)v * Hs * Ws];
#pragma unroll 1
    for (int j = 0; j < DPT; ++j) {
      Geom own;
      project(rx, ry, rz, R[3], R[7], R[11], dep_lds[j][tid], halfw, halfh, own.x0, own.y0, own.fx, own.fy);
      float part[LPS];
      pair_rounds<C, 0, (LPS < 4 ? LPS : 4)>(rsrc, vbase, rowb, W, H, own, r4, tx, part);
      if constexpr (LPS == 8) {
        __builtin_amdgcn_sched_barrier(0);
        pair_rounds<C, 4, 4>(rsrc, vbase, rowb, W, H, own, r4, tx, part);
      }
      float tot = reduce_scatter<LPS>(part, k);
      acc_lds[j][tid] = acc_lds[j][tid] + (tot * (1.f / (float)C)) * w;
    }
    wsum = wsum + w;
  }
  if (!active) return;
#pragma unroll 4
  for (int j = 0; j < DPT; ++j) {
    const size_t o = (size_t)(j * LPS + dsub) * HW + p;
    sim_out[o] = PARTIAL ? acc_lds[j][tid] : acc_lds[j][tid] / wsum;
  }
  if (PARTIAL && dsub == 0) wsum_out[p] = wsum;
}

template <int C, int D, bool PW, bool PARTIAL>
static int launch_warp(const float* ref, const float* src, const float* hyp, const float* vw_in, float* sim,
                       float* wsum, float* vw_out, int V, int H, int W, int vw_shift, int vw_offset, int vw_total,
                       const WarpArgs& args, hipStream_t st) {
  if constexpr ((C == 8 || C == 16) && !PW) {
    constexpr int PIXP = 4 * (64 / (C / 2));
    const int nblk = (H * W + PIXP - 1) / PIXP;
    hipLaunchKernelGGL((warp_pair_kernel<C, D, PARTIAL>), dim3(nblk), dim3(256), 0, st, ref, src, hyp, vw_in, sim,
                       wsum, V, H, W, vw_shift, vw_offset, args);
    TMVS_CHECK_LAUNCH();
    return TMVS_OK;
  }
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


// ---------------------------------------------------------------- backward (training, C5)
// Adjoint of the per-view similarity sim_v[d][p] = (1/C) sum_c ref[p][c] * bilinear(src_v, X(v,d,p))[c]
// (homo_warping + (warped * ref).mean(1), models/module.py:284-322, TransMVSNet.py:80), given
// dsim_v [V][D][H][W]:
//   dref[p][c]   = sum_v sum_d (dsim_v[d][p] / C) * bilinear_c         (gather: registers, no atomics)
//   dsrc_v[q][c] += w_tap * (dsim_v[d][p] / C) * ref[p][c]              (scatter to the 4 taps)
// The scatter is deterministic: contributions are rounded to fixed point and summed with 64-bit
// integer atomics (order-independent), then converted once. The fixed-point unit is chosen per call
// from max|dsim| and max|ref| (fix_shift): no texel can receive more than D*H*W contributions of at
// most max|dsim|/C * max|ref| each, so the unit 2^-k with k = 62 - ceil(log2(that product bound))
// keeps every texel's int64 sum in range whatever the gradient scale, and its resolution is
// 2^-40 or finer RELATIVE to the largest contribution (an absolute unit would flush the small
// gradients of a mean loss over a full-resolution stage to zero). Before that, the
// coefficients w_tap * g of a source pixel are summed in registers across the consecutive planes
// that hit it (one slot per tap parity class), so a pixel-view issues C atomics per UNIQUE tap. One thread per
// reference pixel walks the views and planes; coordinates come from project() (same rounding as
// the forward, incl. TMVS_WARP_ROT_PLAIN).
// max |x| over n floats -> atomicMax on its bit pattern (non-negative floats order as unsigned);
// a non-finite element sets the flag (the host raises: the gradient is unusable)
// (one atomic per block: per-wave atomics on one word serialise)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, long n, unsigned* __restrict__ out,
                                                     int* __restrict__ flag) {
  __shared__ float red[4];
  __shared__ int anybad;
  if (threadIdx.x == 0) anybad = 0;
  float m = 0.f;
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float a = fabsf(x[i]);
    bad |= !isfinite(a);
    m = fmaxf(m, a);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  if (bad) anybad = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicMax(out, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
    if (anybad) atomicOr(flag, 1);
  }
}

// the per-call fixed-point exponent: contributions are scaled by 2^k (see above)
__device__ inline int fix_shift(const unsigned* mx, int C, long count) {
  const double bound = (double)__uint_as_float(mx[0]) / (double)C * (double)__uint_as_float(mx[1]) * (double)count;
  if (!(bound > 0.0)) return 0;
  int e;
  frexp(bound, &e);  // bound < 2^e
  return 62 - e;
}

template <int C, bool SCATTER>
__global__ __launch_bounds__(256) void warp_corr_bwd_kernel(const float* __restrict__ ref,
                                                            const float* __restrict__ src,
                                                            const float* __restrict__ hyp,
                                                            const float* __restrict__ dsim, int V, int D, int H, int W,
                                                            int dchunk, WarpArgs args, float* __restrict__ dref_part,
                                                            unsigned long long* __restrict__ dsrc_fix,
                                                            const unsigned* __restrict__ absmax) {
  // one thread per (pixel, view blockIdx.y, chunk of dchunk planes blockIdx.z); d ref partial per (view, chunk).
  // Lanes past the image stay in the wave (inactive) because the scatter flushes are wave-cooperative.
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < HW;
  const int pc = live ? p : HW - 1;
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.y;
  const int d0 = blockIdx.z * dchunk, d1 = d0 + dchunk < D ? d0 + dchunk : D;
  const int py = pc / W, px = pc - py * W;
  const float fxp = (float)px, fyp = (float)py;
  float dr[C];
#pragma unroll
  for (int c = 0; c < C; ++c) dr[c] = 0.f;
  const float halfw = (float)(W - 1) / 2.f, halfh = (float)(H - 1) / 2.f;
  const int kfix = fix_shift(absmax, C, (long)D * HW);
  unsigned skey[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  float scoef[4] = {0.f, 0.f, 0.f, 0.f};
  unsigned long long* dv = dsrc_fix + (size_t)v * HW * C;
  // the block's reference rows in LDS (TMVS_WARP_BWD_SREF): a flush round reads its items' rows from
  // there, not from global memory -- one round is a chain of lane exchanges, the row read, the
  // fixed-point conversion and the atomic, and a global read had put a memory latency into every round
#ifndef TMVS_WARP_BWD_SREF
#define TMVS_WARP_BWD_SREF 1
#endif
  constexpr bool kSref = SCATTER && TMVS_WARP_BWD_SREF;
  __shared__ __attribute__((aligned(16))) float sref[kSref ? 256 * C : 4];
  if constexpr (kSref) {
    static_assert(C % 4 == 0, "float4 rows");
    const int p0 = blockIdx.x * blockDim.x;
    for (int i = threadIdx.x; i < 256 * C / 4; i += 256) {
      const int pp = p0 + i / (C / 4);
      reinterpret_cast<float4*>(sref)[i] =
          pp < HW ? reinterpret_cast<const float4*>(ref)[(size_t)pp * (C / 4) + i % (C / 4)] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
  }
  // Wave-cooperative flush: the pending (lane, slot) items are served 64/C at a time, lane c % C adding
  // channel c of item lane / C, so each atomic instruction covers whole C-channel rows (coalesced per
  // cache line) instead of 64 scattered rows. The added value per (texel, channel) is unchanged.
  constexpr int K = 64 / C;
  const int item = lane / C, ch = lane % C;
  auto flush = [&](int sl, bool need) {
    unsigned long long m = __ballot(need && skey[sl] != 0xFFFFFFFFu && scoef[sl] != 0.f);
    while (m) {
      int mine = -1;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int l = m ? __ffsll((long long)m) - 1 : -1;
        if (k == item) mine = l;
        if (m) m &= m - 1;
      }
      const int srcl = mine < 0 ? 0 : mine;
      const unsigned key = (unsigned)__shfl((int)skey[sl], srcl);
      const float coef = __shfl(scoef[sl], srcl);
      const int pp = kSref ? 0 : __shfl(pc, srcl);
      if (mine >= 0) {
        const float rv = kSref ? sref[((threadIdx.x & ~63) + srcl) * C + ch] : ref[(size_t)pp * C + ch];
        const float sc = ldexpf(coef * rv, kfix);
        if (sc != 0.f)
          atomicAdd(dv + ((size_t)(key >> 16) * W + (key & 0xFFFFu)) * C + ch,
                    (unsigned long long)(long long)llrintf(sc));
      }
    }
  };
  {
    const float* R = args.proj[v];
    const float rx = rot_row(R, fxp, fyp, args.rot_plain);
    const float ry = rot_row(R + 4, fxp, fyp, args.rot_plain);
    const float rz = rot_row(R + 8, fxp, fyp, args.rot_plain);
    const float* sv = src + (size_t)v * HW * C;
#pragma unroll 1
    for (int d = d0; d < d1; ++d) {
      const float g = live ? dsim[((size_t)v * D + d) * HW + pc] * (1.f / (float)C) : 0.f;  // C = 2^n: exact
      int x0, y0;
      float fx, fy;
      project(rx, ry, rz, R[3], R[7], R[11], hyp[(size_t)d * HW + pc], halfw, halfh, x0, y0, fx, fy);
      const float ea = 1.f - fx, s = 1.f - fy;
      const bool act = g != 0.f;
      if (act) {
        const float wt[4] = {s * ea, s * fx, fy * ea, fy * fx};  // nw, ne, sw, se (grid_sample)
        const int tx[4] = {x0, x0 + 1, x0, x0 + 1}, ty[4] = {y0, y0, y0 + 1, y0 + 1};
        bool in[4];
        const float* tp[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          in[t] = (unsigned)tx[t] < (unsigned)W && (unsigned)ty[t] < (unsigned)H;
          tp[t] = sv + ((size_t)(in[t] ? ty[t] : 0) * W + (in[t] ? tx[t] : 0)) * C;
        }
#pragma unroll
        for (int c4 = 0; c4 < C / 4; ++c4) {  // rows are 16-B aligned (C % 4 == 0): one float4 per tap quad
          // unconditional loads (an outside tap points at pixel 0, always valid), zeroed after: no
          // per-element branches around the loads
          const float4 a4 = *reinterpret_cast<const float4*>(tp[0] + 4 * c4);
          const float4 b4 = *reinterpret_cast<const float4*>(tp[1] + 4 * c4);
          const float4 c4v = *reinterpret_cast<const float4*>(tp[2] + 4 * c4);
          const float4 d4 = *reinterpret_cast<const float4*>(tp[3] + 4 * c4);
          const float av[4] = {in[0] ? a4.x : 0.f, in[0] ? a4.y : 0.f, in[0] ? a4.z : 0.f, in[0] ? a4.w : 0.f};
          const float bv[4] = {in[1] ? b4.x : 0.f, in[1] ? b4.y : 0.f, in[1] ? b4.z : 0.f, in[1] ? b4.w : 0.f};
          const float cv[4] = {in[2] ? c4v.x : 0.f, in[2] ? c4v.y : 0.f, in[2] ? c4v.z : 0.f, in[2] ? c4v.w : 0.f};
          const float dv4[4] = {in[3] ? d4.x : 0.f, in[3] ? d4.y : 0.f, in[3] ? d4.z : 0.f, in[3] ? d4.w : 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float val = fmaf(dv4[e], wt[3], fmaf(cv[e], wt[2], fmaf(bv[e], wt[1], av[e] * wt[0])));
            dr[4 * c4 + e] = fmaf(g, val, dr[4 * c4 + e]);
          }
        }
      }
      // scatter coefficients w_tap * g, summed per source pixel across consecutive planes: the 4 taps
      // of a plane occupy the 4 (x, y) parity classes, so slot (X&1, Y&1) holds the latest tap of its
      // class and its running coefficient; a slot is flushed (C atomics) only when its tap changes
      if constexpr (SCATTER)
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const int X = x0 + ((x0 ^ sl) & 1), Y = y0 + ((y0 ^ (sl >> 1)) & 1);
        const bool inside = (unsigned)X < (unsigned)W && (unsigned)Y < (unsigned)H;
        const float wgt = ((Y == y0) ? s : fy) * ((X == x0) ? ea : fx);
        const unsigned key = inside ? ((unsigned)Y << 16) | (unsigned)X : 0xFFFFFFFFu;
        const bool change = act && key != skey[sl];
        flush(sl, change);
        if (change) {
          skey[sl] = key;
          scoef[sl] = 0.f;
        }
        if (act && inside) scoef[sl] = fmaf(wgt, g, scoef[sl]);
      }
    }
    if constexpr (SCATTER)
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) flush(sl, true);
  }
  if (live) {
    float* dref = dref_part + ((size_t)(v * gridDim.z + blockIdx.z) * HW + p) * C;
#pragma unroll
    for (int c4 = 0; c4 < C / 4; ++c4)
      *reinterpret_cast<float4*>(dref + 4 * c4) =
          make_float4(dr[4 * c4], dr[4 * c4 + 1], dr[4 * c4 + 2], dr[4 * c4 + 3]);
  }
}

// d src as a GATHER, for fronto-parallel hypotheses (hyp[d][p] = hyp[d][0] for every p: stage 1's
// depth planes). On plane d the forward maps reference pixel p to X = A_d (p, 1) with
// A_d = z_d R + t e3^T (project(): ix = X/Z), a homography; source texel q is one of p's 4 bilinear
// taps iff ix(p) lies in [qx-1, qx+1) x [qy-1, qy+1). So q's contributors are the integer pixels in
// the preimage of that square under A_d: while the square is in front of the source camera (the
// third coordinate of A_d^-1 (c, 1), = 1/Z, positive at its 4 corners -- it is affine in c) that
// preimage is the quadrilateral of the 4 mapped corners; otherwise (the plane's horizon crosses the
// square) every pixel is a candidate. Each candidate is re-projected with project() -- the forward's
// own rounding -- and contributes w_tap * dsim/C * ref[p] exactly when the forward sampled q with
// weight w_tap, so no atomics and no fixed point: a texel's sum has a fixed order (planes ascending
// within each of the 4 waves' plane quarters, then (w0 + w1) + (w2 + w3)). The square is widened by
// 0.02 px before mapping to cover the difference between the exact and the forward-rounded ix.
// Block = 64 texels x 4 plane quarters (one wave each); a thread whose own hyp[d][q] differs from
// hyp[d][0] sets flag bit 2 (the hypotheses were not planes: the result is unusable).
constexpr int kPlanesMaxD = 64;
template <int C>
__global__ __launch_bounds__(256) void warp_bwd_src_planes_kernel(const float* __restrict__ ref,
                                                                  const float* __restrict__ hyp,
                                                                  const float* __restrict__ dsim, int D, int H, int W,
                                                                  WarpArgs args, float* __restrict__ dsrc,
                                                                  int* __restrict__ flag) {
  __shared__ float ainv[kPlanesMaxD][9];
  __shared__ float plane[kPlanesMaxD];
  __shared__ float red[3][64][C + 1];
  const int HW = H * W;
  const int v = blockIdx.y;
  const float* R = args.proj[v];
  if (threadIdx.x < D) {
    const double z = hyp[(size_t)threadIdx.x * HW];
    plane[threadIdx.x] = (float)z;
    const double a0 = z * R[0], a1 = z * R[1], a2 = z * R[2] + R[3];
    const double a3 = z * R[4], a4 = z * R[5], a5 = z * R[6] + R[7];
    const double a6 = z * R[8], a7 = z * R[9], a8 = z * R[10] + R[11];
    const double c0 = a4 * a8 - a5 * a7, c1 = a2 * a7 - a1 * a8, c2 = a1 * a5 - a2 * a4;
    const double det = a0 * c0 + a3 * c1 + a6 * c2;
    float* o = ainv[threadIdx.x];
    if (det != 0.0 && isfinite(det)) {
      const double r = 1.0 / det;
      o[0] = (float)(c0 * r);
      o[1] = (float)(c1 * r);
      o[2] = (float)(c2 * r);
      o[3] = (float)((a5 * a6 - a3 * a8) * r);
      o[4] = (float)((a0 * a8 - a2 * a6) * r);
      o[5] = (float)((a2 * a3 - a0 * a5) * r);
      o[6] = (float)((a3 * a7 - a4 * a6) * r);
      o[7] = (float)((a1 * a6 - a0 * a7) * r);
      o[8] = (float)((a0 * a4 - a1 * a3) * r);
    } else {
      for (int k = 0; k < 9; ++k) o[k] = 0.f;  // third coordinate 0: every pixel is a candidate
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = blockIdx.x * 64 + lane;
  const bool live = q < HW;
  const int qq = live ? q : HW - 1;
  const int qy = qq / W, qx = qq - qy * W;
  const float halfw = (float)(W - 1) / 2.f, halfh = (float)(H - 1) / 2.f;
  const float* dv = dsim + (size_t)v * D * HW;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  const int per = (D + 3) / 4, d0 = wv * per, d1 = d0 + per < D ? d0 + per : D;
  bool nonplanar = false;
  constexpr float kPad = 1.02f;
#pragma unroll 1
  for (int d = d0; d < d1; ++d) {
    const float dep = plane[d];
    nonplanar |= live && hyp[(size_t)d * HW + qq] != dep;
    const float* A = ainv[d];
    float mnx = 3.0e38f, mxx = -3.0e38f, mny = 3.0e38f, mxy = -3.0e38f;
    bool unb = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float cx = (float)qx + ((k & 1) ? kPad : -kPad), cy = (float)qy + ((k & 2) ? kPad : -kPad);
      const float hz = fmaf(A[6], cx, fmaf(A[7], cy, A[8]));
      if (!(hz > 0.f)) {
        unb = true;
      } else {
        const float px = fmaf(A[0], cx, fmaf(A[1], cy, A[2])) / hz;
        const float py = fmaf(A[3], cx, fmaf(A[4], cy, A[5])) / hz;
        mnx = fminf(mnx, px);
        mxx = fmaxf(mxx, px);
        mny = fminf(mny, py);
        mxy = fmaxf(mxy, py);
      }
    }
    int bx0 = 0, bx1 = W - 1, by0 = 0, by1 = H - 1;
    if (!unb) {  // clamp in float first (a far-away preimage must not overflow the int conversion)
      bx0 = (int)fminf(fmaxf(floorf(mnx), 0.f), (float)W);
      bx1 = (int)fmaxf(fminf(ceilf(mxx), (float)(W - 1)), -1.f);
      by0 = (int)fminf(fmaxf(floorf(mny), 0.f), (float)H);
      by1 = (int)fmaxf(fminf(ceilf(mxy), (float)(H - 1)), -1.f);
    }
    if (!live) bx1 = bx0 - 1;
    const float* gd = dv + (size_t)d * HW;
#pragma unroll 1
    for (int py = by0; py <= by1; ++py) {
      const float fyp = (float)py;
#pragma unroll 1
      for (int px = bx0; px <= bx1; ++px) {
        const float fxp = (float)px;
        const float rx = rot_row(R, fxp, fyp, args.rot_plain);
        const float ry = rot_row(R + 4, fxp, fyp, args.rot_plain);
        const float rz = rot_row(R + 8, fxp, fyp, args.rot_plain);
        int x0, y0;
        float fx, fy;
        project(rx, ry, rz, R[3], R[7], R[11], dep, halfw, halfh, x0, y0, fx, fy);
        const int dx = qx - x0, dy = qy - y0;
        if ((unsigned)dx > 1u || (unsigned)dy > 1u) continue;
        const int p = py * W + px;
        const float g = gd[p] * (1.f / (float)C);  // C = 2^n: exact
        const float wgt = (dy == 0 ? 1.f - fy : fy) * (dx == 0 ? 1.f - fx : fx);
        const float coef = wgt * g;
        const float* rp = ref + (size_t)p * C;
#pragma unroll
        for (int c4 = 0; c4 < C / 4; ++c4) {
          const float4 r4 = *reinterpret_cast<const float4*>(rp + 4 * c4);
          acc[4 * c4 + 0] = fmaf(coef, r4.x, acc[4 * c4 + 0]);
          acc[4 * c4 + 1] = fmaf(coef, r4.y, acc[4 * c4 + 1]);
          acc[4 * c4 + 2] = fmaf(coef, r4.z, acc[4 * c4 + 2]);
          acc[4 * c4 + 3] = fmaf(coef, r4.w, acc[4 * c4 + 3]);
        }
      }
    }
  }
  if (nonplanar) atomicOr(flag, 2);
  if (wv > 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) red[wv - 1][lane][c] = acc[c];
  }
  __syncthreads();
  if (wv == 0 && live) {
    float* o = dsrc + ((size_t)v * HW + q) * C;
#pragma unroll
    for (int c4 = 0; c4 < C / 4; ++c4) {
      float t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * c4 + e;
        t[e] = (acc[c] + red[0][lane][c]) + (red[1][lane][c] + red[2][lane][c]);
      }
      *reinterpret_cast<float4*>(o + 4 * c4) = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
}

// out[i] = sum over the nparts partials in part order (view-major, then plane chunk): fixed, reproducible
__global__ void sum_dref_parts_kernel(const float* __restrict__ part, int nparts, long n, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = part[i];
  for (int k = 1; k < nparts; ++k) s += part[(size_t)k * n + i];
  out[i] = s;
}

__global__ void fix_to_float_kernel(const unsigned long long* __restrict__ in, long n, const unsigned* __restrict__ absmax,
                                    int C, long count, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (float)ldexp((double)(long long)in[i], -fix_shift(absmax, C, count));
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
  // the kernel addresses one sample's source views with 32-bit byte offsets (< 2^30)
  if ((long long)n_src * height * width * channels * 4 >= (1LL << 30)) return TMVS_ERR_SHAPE;
  if (width > 32766 || height > 32766) return TMVS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const size_t HW = (size_t)height * width;
  for (int b = 0; b < batch; ++b) {
    WarpArgs a;
    a.rot_plain = (flags & TMVS_WARP_ROT_PLAIN) ? 1 : 0;
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
                                 int ndepth, int height, int width, int flags, float* out, void* stream) {
  if (!src_fea || !proj || !hyp || !out || batch <= 0 || channels <= 0 || ndepth <= 0 || height <= 0 || width <= 0)
    return TMVS_ERR_ARG;
  const size_t HW = (size_t)height * width;
  for (int b = 0; b < batch; ++b) {
    WarpArgs a = {};
    a.rot_plain = (flags & TMVS_WARP_ROT_PLAIN) ? 1 : 0;
    for (int k = 0; k < 12; ++k) a.proj[0][k] = proj[(size_t)b * 12 + k];
    const int n = ndepth * (int)HW;
    hipLaunchKernelGGL(homo_warping_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       src_fea + (size_t)b * channels * HW, hyp + (size_t)b * ndepth * HW,
                       out + (size_t)b * channels * ndepth * HW, channels, ndepth, height, width, a);
    TMVS_CHECK_LAUNCH();
  }
  return TMVS_OK;
}

static int bwd_dchunk(int ndepth) { return ndepth < 8 ? ndepth : 8; }

// [fixed-point d src: n_src*HW*C int64][flag int, max|dsim| u32, max|ref| u32, padded to 256 B]
// [d ref partials: n_src*chunks*HW*C fp32]
extern "C" size_t tmvs_warp_corr_backward_workspace(int n_src, int channels, int height, int width, int ndepth) {
  const size_t n = (size_t)n_src * height * width * channels;
  const int nch = (ndepth + bwd_dchunk(ndepth) - 1) / bwd_dchunk(ndepth);
  return n * sizeof(unsigned long long) + 256 + n * nch * sizeof(float);
}

extern "C" int tmvs_warp_corr_backward(const float* ref_fea, const float* src_fea, const float* proj, const float* hyp,
                                       const float* dsim, int n_src, int channels, int ndepth, int height, int width,
                                       int flags, void* workspace, size_t workspace_bytes, float* dref, float* dsrc,
                                       void* stream) {
  if (!ref_fea || !src_fea || !proj || !hyp || !dsim || !workspace || !dref || !dsrc) return TMVS_ERR_ARG;
  if (n_src <= 0 || n_src > TMVS_MAX_VIEWS || ndepth <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (width > 32766 || height > 32766) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_warp_corr_backward_workspace(n_src, channels, height, width, ndepth)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  WarpArgs a = {};
  a.rot_plain = (flags & TMVS_WARP_ROT_PLAIN) ? 1 : 0;
  for (int v = 0; v < n_src; ++v)
    for (int k = 0; k < 12; ++k) a.proj[v][k] = proj[(size_t)v * 12 + k];
  const long n = (long)n_src * height * width * channels;
  unsigned long long* fix = (unsigned long long*)workspace;
  int* ovf = (int*)((char*)workspace + (size_t)n * sizeof(unsigned long long));
  unsigned* absmax = (unsigned*)(ovf + 1);
  if ((flags & TMVS_WARP_BWD_PLANES) ? hipMemsetAsync(ovf, 0, 3 * sizeof(int), st) != hipSuccess
                                      : hipMemsetAsync(workspace, 0, (size_t)n * sizeof(unsigned long long) + 3 * sizeof(int),
                                                       st) != hipSuccess)
    return TMVS_ERR_HIP;
  const int HW = height * width;
  const long nd = (long)n_src * ndepth * HW, nr = (long)HW * channels;
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)std::min<long>(1024, (nd + 255) / 256)), dim3(256), 0, st, dsim, nd,
                     absmax, ovf);
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)std::min<long>(256, (nr + 255) / 256)), dim3(256), 0, st, ref_fea, nr,
                     absmax + 1, ovf);
  TMVS_CHECK_LAUNCH();
  const int dchunk = bwd_dchunk(ndepth), nch = (ndepth + dchunk - 1) / dchunk;
  float* part = (float*)((char*)workspace + (size_t)n * sizeof(unsigned long long) + 256);
  const dim3 grid((HW + 255) / 256, n_src, nch);
  const bool planes = (flags & TMVS_WARP_BWD_PLANES) != 0;
  if (planes && ndepth > kPlanesMaxD) return TMVS_ERR_SHAPE;
  const dim3 pgrid((HW + 63) / 64, n_src);
#define TMVS_BWD_CASE(CC)                                                                                              \
  case CC:                                                                                                             \
    if (planes) {                                                                                                      \
      hipLaunchKernelGGL((warp_corr_bwd_kernel<CC, false>), grid, dim3(256), 0, st, ref_fea, src_fea, hyp, dsim, n_src, \
                         ndepth, height, width, dchunk, a, part, fix, absmax);                                          \
      hipLaunchKernelGGL(warp_bwd_src_planes_kernel<CC>, pgrid, dim3(256), 0, st, ref_fea, hyp, dsim, ndepth, height,   \
                         width, a, dsrc, ovf);                                                                          \
    } else {                                                                                                           \
      hipLaunchKernelGGL((warp_corr_bwd_kernel<CC, true>), grid, dim3(256), 0, st, ref_fea, src_fea, hyp, dsim, n_src,  \
                         ndepth, height, width, dchunk, a, part, fix, absmax);                                          \
    }                                                                                                                  \
    break;
  switch (channels) {
    TMVS_BWD_CASE(8)
    TMVS_BWD_CASE(16)
    TMVS_BWD_CASE(32)
    default:
      return TMVS_ERR_SHAPE;
  }
#undef TMVS_BWD_CASE
  TMVS_CHECK_LAUNCH();
  const long nref = (long)HW * channels;
  hipLaunchKernelGGL(sum_dref_parts_kernel, dim3((unsigned)((nref + 255) / 256)), dim3(256), 0, st, (const float*)part,
                     n_src * nch, nref, dref);
  TMVS_CHECK_LAUNCH();
  if (!planes) {
    hipLaunchKernelGGL(fix_to_float_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const unsigned long long*)fix, n, (const unsigned*)absmax, channels, (long)ndepth * HW, dsrc);
    TMVS_CHECK_LAUNCH();
  }
  return TMVS_OK;
}
