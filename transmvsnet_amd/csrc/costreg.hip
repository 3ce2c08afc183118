// CostRegNet (models/module.py:425-456) on MI355X.
//
// Layout: NDHWC fp32 activations. Eval-mode BN is an (alpha, shift) epilogue,
// y = relu(fmaf(acc, alpha, shift)) (tmvs_bn_fold; the reference CPU kernel's exact form). The MFMA
// layers' epilogue is act(v, lo) = v > lo ? v : lo: lo = 0 is that ReLU; lo = -inf with alpha = 1,
// shift = 0 and no skip gives the raw convolution the training path runs them for
// (tmvs_conv3d_mfma: train-mode forward before BatchNorm, and the data gradients).
//
// Mid layers (conv1..conv6, deconv conv7/9/11) are LDS-staged implicit GEMMs on the exact-fp32 matrix
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

// Range-checked raw buffer over one tensor: a lane whose 32-bit byte offset is out of range reads
// zeros (the buffer unit's bound check), so padding taps need no exec-mask branch and no 64-bit
// address per load; the wave-uniform part of an offset goes in the scalar offset. Branch-free load
// streams keep the compiler's vmcnt waits exact (a branch per load made it wait vmcnt(0)).
struct Buf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Buf(const float* base, uint32_t nbytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)nbytes, 0x00020000)) {}
  static constexpr int kOOB = (int)0x80000000u;  // any offset >= the range reads zeros
  __device__ __forceinline__ float4 ld4(int voff, int soff = 0) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  }
  __device__ __forceinline__ float2 ld2(int voff, int soff = 0) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
  }
};
template <int N>
__device__ __forceinline__ void buf_load(VecN<N>& d, const Buf& b, int voff, int soff = 0);
template <>
__device__ __forceinline__ void buf_load<4>(VecN<4>& d, const Buf& b, int voff, int soff) {
  const float4 t = b.ld4(voff, soff);
  d.v[0] = t.x, d.v[1] = t.y, d.v[2] = t.z, d.v[3] = t.w;
}
template <>
__device__ __forceinline__ void buf_load<2>(VecN<2>& d, const Buf& b, int voff, int soff) {
  const float2 t = b.ld2(voff, soff);
  d.v[0] = t.x, d.v[1] = t.y;
}

struct Geo {
  int Di, Hi, Wi;  // input dims
  int Do, Ho, Wo;  // output dims
  float lo;        // epilogue floor: 0 = ReLU, -inf = none
};

__device__ __forceinline__ float act(float v, float lo) { return v > lo ? v : lo; }

// ---------------------------------------------------------------- conv3d k3 p1, stride S
// Workgroup tile: 16 output voxels along w x TH rows x TD depth slices, MBB blocks of 16
// output channels. Per CK-channel chunk the input tile (+halo) is staged once into LDS
// (voxel stride CK+4 floats: the 16 lanes of a row hit distinct banks), then each wave runs
// its NBW = TD*TH/4 rows through the 27 taps: A (weights) from global/L2, requested two taps
// ahead, B from LDS. The next chunk's tile is fetched into registers during the current
// chunk's MFMAs.
#ifndef TMVS_LDS_BPF
#define TMVS_LDS_BPF 1
#endif
#ifndef TMVS_LDS_ABL
#define TMVS_LDS_ABL 0  // timing ablations (scripts/gpu/r17f.sh): 1 no weight loads, 2 no next-chunk fetch,
#endif                  // 4 no chunk barriers / commit, 8 no MFMAs -- wrong results, never the product
#ifndef TMVS_LDS_SGB
#define TMVS_LDS_SGB 1
#endif
// TAPOUT: every channel chunk's tile is staged at once and the K walk runs taps outer, chunks inner --
// conv3d_direct_kernel's order (tap, chunk, lane channel), so the sums are that kernel's bit for bit; the
// default walks chunks outer (one chunk's tile in LDS at a time), which re-associates the K sum when
// CIN > 16. TAPOUT needs TD = 1 (the kd slices in the depth padding are skipped per workgroup, exact zeros).
template <int CIN, int COUT, int S, int TD, int TH, int MBB, int WS = 1, bool KDSKIP = false, bool TAPOUT = false>
#ifndef TMVS_LDS_WPE
#define TMVS_LDS_WPE 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TMVS_LDS_WPE, TMVS_LDS_WPE))) void conv3d_lds_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ shift, float* __restrict__ y,
                                                         Geo g) {
  constexpr int CK = CIN < 16 ? CIN : 16;
  constexpr int PL = CK / 4;
  constexpr int MB = (COUT + 15) / 16;
  constexpr int MG = MB / MBB;
  // WS: the 4 waves are WS block groups x 4/WS row groups; a wave runs NBW rows x MBW blocks (WS = 1:
  // every wave all MBB blocks of TD*TH/4 rows -- the 4 waves then request identical weight fragments)
  static_assert(WS == 1 || WS == 2 || WS == 4, "WS");
  static_assert(MBB % WS == 0 && (TD * TH * WS) % 4 == 0, "wave split");
  constexpr int NBW = TD * TH * WS / 4, MBW = MBB / WS;
  constexpr int LW = 15 * S + 3, LH = (TH - 1) * S + 3, LD = (TD - 1) * S + 3;
  // voxel stride / quad swizzle chosen so the 4 lane groups of every ds_read_b128 are
  // bank-conflict free (exhaustive search over the gfx950 b128 lane grouping)
  constexpr bool SWZ = (CK == 16);  // (stride 2 included: conv3's instance)
  constexpr int VST = SWZ ? 16 : CK + 4;
  constexpr int NVOX = LD * LH * LW;
  static_assert(MB % MBB == 0, "tile");
  static_assert(!TAPOUT || (TD == 1 && !KDSKIP), "TAPOUT: one output slice per workgroup, its own kd skip");
  __shared__ __attribute__((aligned(16))) float tile[(TAPOUT ? CIN / CK : 1) * NVOX * VST];

  const int nws = (g.Wo + 15) / 16, nhs = (g.Ho + TH - 1) / TH, nds = (g.Do + TD - 1) / TD;
  int t = xcd_remap(blockIdx.x, gridDim.x);  // contiguous tiles per XCD: halos share an L2
  const int mg = t % MG;
  t /= MG;
  const int ws = t % nws;
  t /= nws;
  const int hs = t % nhs;
  t /= nhs;
  const int ds = t % nds;
  const int n = t / nds;
  const int ow0 = ws * 16, oh0 = hs * TH, od0 = ds * TD;
  const int iw0 = ow0 * S - 1, ih0 = oh0 * S - 1, id0 = od0 * S - 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  const int rg = __builtin_amdgcn_readfirstlane(wv / WS), bg = __builtin_amdgcn_readfirstlane(wv % WS);
  const int mb0 = mg * MBB + bg * MBW;  // the wave's first 16-channel output block
  const size_t in_n = (size_t)n * g.Di * g.Hi * g.Wi;

  floatx4 acc[NBW][MBW];
#pragma unroll
  for (int r = 0; r < NBW; ++r)
#pragma unroll
    for (int m = 0; m < MBW; ++m) acc[r][m] = floatx4{0.f, 0.f, 0.f, 0.f};

  // channel chunk ch's tile: global -> registers (issued one chunk ahead) -> LDS
  constexpr int NCH = CIN / CK, NLD = (NVOX * PL + 255) / 256;
  const Buf xb(x + in_n * CIN, (uint32_t)g.Di * g.Hi * g.Wi * CIN * 4);  // this sample (host: < 2 GB)
  const Buf wb(wpk, 27u * COUT * CIN * 4);
  float4 pf[NLD];
  auto fetch_to = [&](int ch, float4(&dst)[NLD]) {
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int vox = idx / PL, q = idx - vox * PL;
      const int lw = vox % LW, rest = vox / LW, lh = rest % LH, ld = rest / LH;
      const int iw = iw0 + lw, ih = ih0 + lh, id = id0 + ld;
      // branch-free: padding lanes load x[0..3] and select zero, so the loads stay in one basic
      // block and the compiler's vmcnt waits count them exactly (a branch per load made it wait
      // vmcnt(0) every third tap, exposing the L2 latency of the two-tap-ahead weight loads)
      const bool ok = idx < NVOX * PL && iw >= 0 && iw < g.Wi && ih >= 0 && ih < g.Hi && id >= 0 && id < g.Di;
      dst[k] = xb.ld4(ok ? (((id * g.Hi + ih) * g.Wi + iw) * CIN + 4 * q) * 4 : Buf::kOOB, ch * CK * 4);
    }
  };
  auto fetch = [&](int ch) { fetch_to(ch, pf); };
  auto commit_from = [&](const float4(&src)[NLD], float* base) {
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int vox = idx / PL, q = idx - vox * PL;
      const int qs = SWZ ? (q ^ ((vox >> 1) & 3)) : q;
      if (idx < NVOX * PL) *reinterpret_cast<float4*>(base + vox * VST + 4 * qs) = src[k];
    }
  };
  auto commit = [&]() { commit_from(pf, tile); };
  // KDSKIP (launched only for output depth <= 2, where every wave has one): the kd slices whose
  // input plane lies wholly in the depth padding of the wave's output slice are not run (their
  // products are exact zeros). The taps then run as a loop over the kept slices (9 unrolled taps
  // each); the full-depth instance keeps the straight 27-tap schedule.
  static_assert(!KDSKIP || TH % NBW == 0, "KDSKIP needs one output slice per wave");
  int kd_lo = 0, kd_hi = 2;
  if constexpr (KDSKIP) {
    const int od = od0 + (rg * NBW) / TH;
    const int id_base = od * S - 1;  // input slice of kd = 0
    kd_lo = id_base < 0 ? -id_base : 0;
    kd_hi = g.Di - 1 - id_base < 2 ? g.Di - 1 - id_base : 2;
    if (od >= g.Do) kd_hi = -1;  // rows past the volume: nothing to compute
  }
  // A fragments (chunk ch, tap) from global/L2, requested two taps ahead of their MFMAs; the
  // chunk's last two taps request the next chunk's first two
  auto wload = [&](int ch, int tap, VecN<PL>(&a)[MBW]) {
#pragma unroll
    for (int m = 0; m < MBW; ++m) {
      const int co = (mb0 + m) * 16 + col;  // channels >= COUT read zeros
      if (TMVS_LDS_ABL & 1) {  // timing ablation only: no weight loads
#pragma unroll
        for (int i = 0; i < PL; ++i) a[m].v[i] = (float)(tap * PL + i + ch) * 1e-3f;
        continue;
      }
      buf_load(a[m], wb, (co < COUT ? co * CIN + kgrp * PL : Buf::kOOB / 4) * 4, (tap * COUT * CIN + ch * CK) * 4);
    }
  };
  VecN<PL> aw[3][MBW];
  // one tap: B fragments from the LDS tile, NBW x MBB x PL MFMAs
  // B fragments of one tap from the LDS tile
  auto bload_at = [&](const float* base, int kd, int kh, int kw, VecN<PL>(&b)[NBW]) {
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = rg * NBW + r;
      const int odl = rr / TH, ohl = rr - odl * TH;
      const int lvox = ((odl * S + kd) * LH + ohl * S + kh) * LW + col * S + kw;
      const int qs = SWZ ? (kgrp ^ ((lvox >> 1) & 3)) : kgrp;
      b[r].load(base + lvox * VST + qs * PL);
    }
  };
  auto bload = [&](int kd, int kh, int kw, VecN<PL>(&b)[NBW]) { bload_at(tile, kd, kh, kw, b); };
  // one tap: NBW x MBB x PL MFMAs on fragments already in registers
  auto tap_mfma = [&](const VecN<PL>* a, const VecN<PL>* b) {
    if (TMVS_LDS_ABL & 8) {  // timing ablation only: no MFMAs (one FMA keeps the loads live)
#pragma unroll
      for (int r = 0; r < NBW; ++r)
#pragma unroll
        for (int m = 0; m < MBW; ++m) acc[r][m][0] = fmaf(a[m].v[0], b[r].v[0], acc[r][m][0]);
      return;
    }
#pragma unroll
    for (int j = 0; j < PL; ++j)
#pragma unroll
      for (int r = 0; r < NBW; ++r)
#pragma unroll
        for (int m = 0; m < MBW; ++m)
          acc[r][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m].v[j], b[r].v[j], acc[r][m], 0, 0, 0);
    // one-MFMA schedule groups keep the accumulators' chains interleaved as written (the scheduler
    // otherwise issued each accumulator's PL dependent MFMAs back to back: 40-cycle dependent issue
    // against 32 for an independent one)
    if constexpr (TMVS_LDS_SGB)
#pragma unroll
      for (int i = 0; i < PL * NBW * MBW; ++i) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_barrier(0);  // keep the lookahead schedule (and the VGPR budget)
  };
  // B of tap t + 1 is read from LDS before tap t's MFMAs (TMVS_LDS_BPF; read right before its own
  // MFMAs its latency sat between every tap's MFMA groups)
  VecN<PL> bw[2][NBW];
  if constexpr (TAPOUT) {
    // all chunks staged (every chunk's loads in flight before the first commit), then per kept kd slice
    // 9 taps x NCH chunks as one step sequence with the same two-step weight / one-step B lookahead
    float4 pfc[NCH][NLD];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) fetch_to(ch, pfc[ch]);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) commit_from(pfc[ch], tile + ch * NVOX * VST);
    __syncthreads();
    const int id_base = od0 * S - 1;  // input slice of kd = 0 (workgroup-uniform: TD = 1)
    const int klo = id_base < 0 ? -id_base : 0;
    const int khi = od0 >= g.Do ? -1 : (g.Di - 1 - id_base < 2 ? g.Di - 1 - id_base : 2);
    constexpr int NS = 9 * NCH;  // steps per slice; a multiple of 3, so the weight ring lines up across slices
    auto wstep = [&](int kd, int s, VecN<PL>(&a)[MBW]) { wload(s % NCH, kd * 9 + s / NCH, a); };
    auto bstep = [&](int kd, int s, VecN<PL>(&b)[NBW]) {
      const int t9 = s / NCH;
      bload_at(tile + (s % NCH) * NVOX * VST, kd, t9 / 3, t9 % 3, b);
    };
    if (klo <= khi) {
      wstep(klo, 0, aw[0]);
      wstep(klo, 1, aw[1]);
    }
#pragma unroll 1
    for (int kd = klo; kd <= khi; ++kd) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s + 2 < NS)
          wstep(kd, s + 2, aw[(s + 2) % 3]);
        else if (kd < khi)  // uniform: the next slice's first two steps
          wstep(kd + 1, s + 2 - NS, aw[(s + 2) % 3]);
        if (s == 0) bstep(kd, 0, bw[0]);
        if (s + 1 < NS) bstep(kd, s + 1, bw[(s + 1) & 1]);
        tap_mfma(aw[s % 3], bw[s & 1]);
      }
    }
  } else {
  // The next chunk's tile is requested right after the chunk's last weight load (3 taps before
  // its end), not ahead of the chunk's first: vmcnt retires loads in issue order, so any weight
  // load issued behind the tile loads waits for them (fetching at the chunk's start measured the
  // same, r17a).
  fetch(0);
  commit();
  __syncthreads();
  if constexpr (KDSKIP) {
    if (kd_lo <= kd_hi) {
      wload(0, kd_lo * 9, aw[0]);
      wload(0, kd_lo * 9 + 1, aw[1]);
    }
  } else {
    wload(0, 0, aw[0]);
    wload(0, 1, aw[1]);
  }
  // one channel chunk; MORE (compile time, so no branch splits the load stream and the vmcnt
  // waits stay exact): the next chunk's first weights and tile are requested at its end
  auto chunk = [&](int ch, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value;
    if (MORE && KDSKIP && kd_lo > kd_hi) fetch(ch + 1);  // a wave with no slices still stages its share
    if constexpr (KDSKIP) {
#pragma unroll 1
      for (int kd = kd_lo; kd <= kd_hi; ++kd)
#pragma unroll
        for (int k9 = 0; k9 < 9; ++k9) {
          if (k9 + 2 < 9) {
            wload(ch, kd * 9 + k9 + 2, aw[(k9 + 2) % 3]);
          } else {  // uniform branch: the next slice's first taps, or the next chunk's
            if (kd < kd_hi)
              wload(ch, kd * 9 + k9 + 2, aw[(k9 + 2) % 3]);
            else if (MORE)
              wload(ch + 1, kd_lo * 9 + k9 - 7, aw[(k9 + 2) % 3]);
          }
          if (MORE && !(TMVS_LDS_ABL & 2) && k9 == 6 && kd == kd_hi) fetch(ch + 1);
          // B prefetch within the slice (9 taps: the parity would flip across the rolled kd loop)
          if (!TMVS_LDS_BPF || k9 == 0) bload(kd, k9 / 3, k9 % 3, bw[k9 & 1]);
          if (TMVS_LDS_BPF && k9 + 1 < 9) bload(kd, (k9 + 1) / 3, (k9 + 1) % 3, bw[(k9 + 1) & 1]);
          tap_mfma(aw[k9 % 3], bw[k9 & 1]);
        }
    } else {
#pragma unroll
      for (int tap = 0; tap < 27; ++tap) {
        if (tap + 2 < 27)
          wload(ch, tap + 2, aw[(tap + 2) % 3]);
        else if (MORE)
          wload(ch + 1, tap - 25, aw[(tap + 2) % 3]);
        if (MORE && !(TMVS_LDS_ABL & 2) && tap == 24) fetch(ch + 1);
        if (!TMVS_LDS_BPF || tap == 0) bload(tap / 9, (tap / 3) % 3, tap % 3, bw[tap & 1]);
        if (TMVS_LDS_BPF && tap + 1 < 27) bload((tap + 1) / 9, ((tap + 1) / 3) % 3, (tap + 1) % 3, bw[(tap + 1) & 1]);
        tap_mfma(aw[tap % 3], bw[tap & 1]);
      }
    }
    if (MORE && !(TMVS_LDS_ABL & 4)) {
      __syncthreads();
      commit();
      __syncthreads();
    }
  };
#pragma unroll 1
  for (int ch = 0; ch + 1 < NCH; ++ch) chunk(ch, std::true_type{});
  chunk(NCH - 1, std::false_type{});
  }
  const int ow = ow0 + col;
  if (ow >= g.Wo) return;
  const size_t out_n = (size_t)n * g.Do * g.Ho * g.Wo;
#pragma unroll
  for (int m = 0; m < MBW; ++m) {
    const int co = (mb0 + m) * 16 + kgrp * 4;
    if (co >= COUT) continue;
    const float4 al = *reinterpret_cast<const float4*>(alpha + co);
    const float4 sh = *reinterpret_cast<const float4*>(shift + co);
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = rg * NBW + r;
      const int od = od0 + rr / TH, oh = oh0 + rr % TH;
      if (od >= g.Do || oh >= g.Ho) continue;
      float4 o;
      o.x = act(fmaf(acc[r][m][0], al.x, sh.x), g.lo);
      o.y = act(fmaf(acc[r][m][1], al.y, sh.y), g.lo);
      o.z = act(fmaf(acc[r][m][2], al.z, sh.z), g.lo);
      o.w = act(fmaf(acc[r][m][3], al.w, sh.w), g.lo);
      *reinterpret_cast<float4*>(y + (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co) = o;
    }
  }
}

// ---------------------------------------------------------------- conv3d, direct (no LDS)
// Used for the stride-2 layers: no LDS footprint, high occupancy hides the per-tap L1/L2 latency.
// (Branch-free buffer loads with a one-step-ahead register prefetch measured the same, r17a.)
template <int CIN, int COUT, int S, int NBW, int MBW>
__global__ __launch_bounds__(256) void conv3d_direct_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                          const float* __restrict__ alpha,
                                                          const float* __restrict__ shift, float* __restrict__ y,
                                                          Geo g, int n_tasks) {
  constexpr int CK = CIN < 16 ? CIN : 16;  // channels per K chunk
  constexpr int PL = CK / 4;               // channels per lane per chunk (= MFMAs per chunk)
  constexpr int MB = (COUT + 15) / 16;     // 16-channel output blocks
  constexpr int MG = MB / MBW;             // wave groups along cout
  static_assert(MB % MBW == 0, "MBW must divide MB");
  const int lane = threadIdx.x & 63;
  const int task = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
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
      o.x = act(fmaf(acc[r][m][0], al.x, sh.x), g.lo);
      o.y = act(fmaf(acc[r][m][1], al.y, sh.y), g.lo);
      o.z = act(fmaf(acc[r][m][2], al.z, sh.z), g.lo);
      o.w = act(fmaf(acc[r][m][3], al.w, sh.w), g.lo);
      *reinterpret_cast<float4*>(y + (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co) = o;
    }
  }
}

// ---------------------------------------------------------------- ConvTranspose3d k3 s2 p1 op1
// output o = 2i - 1 + k: parity 0 -> (k=1, i=o/2); parity 1 -> (k=0, i=o/2+1), (k=2, i=o/2).
// Workgroup tile in input-grid coordinates: 16 columns x THI rows x TDI slices (outputs
// 32 x 2THI x 2TDI). Each wave owns TDI*THI/4 input-grid rows and all 8 output parity
// classes of them (a class = 16 outputs with one parity per dimension = one tap set of
// 1, 2, 4 or 8 taps), so the waves carry equal work. Input tile (+1 halo) staged in LDS.
#ifndef TMVS_DECONV_ABL
#define TMVS_DECONV_ABL 0  // timing ablations (wrong results): 1 no weight staging, 2 no tile staging, 4 no MFMAs
#endif
template <int CIN, int COUT, int TDI, int THI, int MBB>
__global__ __launch_bounds__(256) void deconv3d_lds_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ wpk,
                                                           const float* __restrict__ alpha,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ skip, float* __restrict__ y,
                                                           Geo g) {
  constexpr int CK = CIN < 16 ? CIN : 16;
  constexpr int PL = CK / 4;
  constexpr int MB = (COUT + 15) / 16;
  constexpr int MG = MB / MBB;
  constexpr int NBW = TDI * THI / 4;
  constexpr int LW = 17, LH = THI + 1, LD = TDI + 1;
  constexpr bool SWZ = (CK == 16);  // (stride 2 included: conv3's instance)  // conflict-free ds_read_b128 (see conv3d_lds_kernel)
  constexpr int VST = SWZ ? 16 : CK + 4;
  constexpr int NVOX = LD * LH * LW;
  static_assert(MB % MBB == 0 && (TDI * THI) % 4 == 0, "tile");
  static_assert(CK == 16 && MBB == 1, "LDS weight staging assumes 16-channel chunks, one 16-row block");
  // weights of the current channel chunk: [27 taps][RM rows][16 ch], quad-swizzled like the
  // tile so the A-fragment ds_read_b128 is bank-conflict free (a per-tap global load right
  // before its MFMAs exposed a full memory latency per tap: MFMA busy 35 %)
  constexpr int RM = COUT < 16 ? COUT : 16;
  __shared__ __attribute__((aligned(16))) float tile[NVOX * VST];
  __shared__ __attribute__((aligned(16))) float wts[27 * RM * 16];

  const int nws = (g.Wi + 15) / 16, nhs = (g.Hi + THI - 1) / THI, nds = (g.Di + TDI - 1) / TDI;
  int t = xcd_remap(blockIdx.x, gridDim.x);  // contiguous tiles per XCD: halos share an L2
  const int mg = t % MG;
  t /= MG;
  const int ws = t % nws;
  t /= nws;
  const int hs = t % nhs;
  t /= nhs;
  const int ds = t % nds;
  const int n = t / nds;
  const int mw0 = ws * 16, mh0 = hs * THI, md0 = ds * TDI;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  const size_t in_n = (size_t)n * g.Di * g.Hi * g.Wi;

  floatx4 acc[NBW][8][MBB];
#pragma unroll
  for (int r = 0; r < NBW; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int m = 0; m < MBB; ++m) acc[r][c][m] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int ch = 0; ch < CIN / CK; ++ch) {
    if (ch) __syncthreads();
    for (int idx = threadIdx.x; idx < ((TMVS_DECONV_ABL & 2) ? 0 : NVOX * PL); idx += 256) {
      const int vox = idx / PL, q = idx - vox * PL;
      const int lw = vox % LW, rest = vox / LW, lh = rest % LH, ld = rest / LH;
      const int iw = mw0 + lw, ih = mh0 + lh, id = md0 + ld;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (iw < g.Wi && ih < g.Hi && id < g.Di)
        v = *reinterpret_cast<const float4*>(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * CIN + ch * CK + 4 * q);
      const int qs = SWZ ? (q ^ ((vox >> 1) & 3)) : q;
      *reinterpret_cast<float4*>(tile + vox * VST + 4 * qs) = v;
    }
    for (int idx = threadIdx.x; idx < ((TMVS_DECONV_ABL & 1) ? 0 : 27 * RM * 4); idx += 256) {
      const int q = idx & 3, row = (idx >> 2) % RM, tap = (idx >> 2) / RM;
      const float4 v = *reinterpret_cast<const float4*>(wpk + ((size_t)tap * COUT + mg * 16 + row) * CIN + ch * CK + 4 * q);
      *reinterpret_cast<float4*>(wts + (tap * RM + row) * 16 + 4 * (q ^ ((row >> 1) & 3))) = v;
    }
    __syncthreads();
#pragma unroll
    for (int cls = 0; cls < 8; ++cls) {
      const int pd = cls >> 2, ph = (cls >> 1) & 1, pw = cls & 1;
#pragma unroll
      for (int td = 0; td < 1 + pd; ++td)
#pragma unroll
        for (int th = 0; th < 1 + ph; ++th)
#pragma unroll
          for (int tw = 0; tw < 1 + pw; ++tw) {
            const int kd = pd ? (td ? 2 : 0) : 1, od_off = (pd && !td) ? 1 : 0;
            const int kh = ph ? (th ? 2 : 0) : 1, oh_off = (ph && !th) ? 1 : 0;
            const int kw = pw ? (tw ? 2 : 0) : 1, ow_off = (pw && !tw) ? 1 : 0;
            const int tap = kd * 9 + kh * 3 + kw;
            VecN<PL> a[MBB];
            if (col < RM)
              a[0].load(wts + (tap * RM + col) * 16 + 4 * (kgrp ^ ((col >> 1) & 3)));
            else
              a[0].zero();
#pragma unroll
            for (int r = 0; r < NBW; ++r) {
              const int rr = wv * NBW + r;
              const int mdl = rr / THI, mhl = rr - mdl * THI;
              VecN<PL> b;
              const int lvox = ((mdl + od_off) * LH + mhl + oh_off) * LW + col + ow_off;
              const int qs = SWZ ? (kgrp ^ ((lvox >> 1) & 3)) : kgrp;
              b.load(tile + lvox * VST + qs * PL);
#pragma unroll
              for (int j = 0; j < PL; ++j)
#pragma unroll
                for (int m = 0; m < MBB; ++m) {
                  if (TMVS_DECONV_ABL & 4)  // timing ablation: no MFMAs (one FMA keeps the reads live)
                    acc[r][cls][m][0] = fmaf(a[m].v[j], b.v[j], acc[r][cls][m][0]);
                  else
                    acc[r][cls][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m].v[j], b.v[j], acc[r][cls][m], 0, 0, 0);
                }
            }
          }
    }
  }
  const size_t out_n = (size_t)n * g.Do * g.Ho * g.Wo;
  if constexpr (COUT == 8) {
    // 8-channel output (conv11, full resolution): the 32 output voxels of one (od, oh) row
    // segment are exchanged through LDS so the skip read and the output store are single
    // contiguous 1 KiB accesses (each 4-lane quad on 64 consecutive bytes) instead of 16-byte
    // pieces at a 64-byte stride.
    __shared__ __attribute__((aligned(16))) float ep[4][32 * 8];
    float* eb = ep[wv];
    const int co = kgrp * 4;
    float4 al = make_float4(0.f, 0.f, 0.f, 0.f), sh = al;
    if (kgrp < 2) {
      al = *reinterpret_cast<const float4*>(alpha + co);
      sh = *reinterpret_cast<const float4*>(shift + co);
    }
    const int ow = 2 * mw0 + (lane >> 1);  // voxel this lane stores (half lane & 1)
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = wv * NBW + r;
      const int md = md0 + rr / THI, mh = mh0 + rr % THI;
#pragma unroll
      for (int pdh = 0; pdh < 4; ++pdh) {
        if (kgrp < 2) {
#pragma unroll
          for (int pw = 0; pw < 2; ++pw) {
            const floatx4 a = acc[r][pdh * 2 + pw][0];
            *reinterpret_cast<float4*>(eb + (2 * col + pw) * 8 + co) =
                make_float4(act(fmaf(a[0], al.x, sh.x), g.lo), act(fmaf(a[1], al.y, sh.y), g.lo),
                            act(fmaf(a[2], al.z, sh.z), g.lo), act(fmaf(a[3], al.w, sh.w), g.lo));
          }
        }
        __builtin_amdgcn_wave_barrier();
        const float4 v = *reinterpret_cast<const float4*>(eb + lane * 4);
        __builtin_amdgcn_wave_barrier();
        const int od = 2 * md + (pdh >> 1), oh = 2 * mh + (pdh & 1);
        if (md < g.Di && mh < g.Hi && ow < 2 * g.Wi) {
          const size_t o = (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * 8 + (lane & 1) * 4;
          const float4 s = skip ? *reinterpret_cast<const float4*>(skip + o) : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(y + o) = make_float4(s.x + v.x, s.y + v.y, s.z + v.z, s.w + v.w);
        }
      }
    }
    return;
  }
  const int mw = mw0 + col;
  if (mw >= g.Wi) return;
#pragma unroll
  for (int m = 0; m < MBB; ++m) {
    const int co = (mg * MBB + m) * 16 + kgrp * 4;
    if (co >= COUT) continue;
    const float4 al = *reinterpret_cast<const float4*>(alpha + co);
    const float4 sh = *reinterpret_cast<const float4*>(shift + co);
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = wv * NBW + r;
      const int md = md0 + rr / THI, mh = mh0 + rr % THI;
      if (md >= g.Di || mh >= g.Hi) continue;
#pragma unroll
      for (int cls = 0; cls < 8; ++cls) {
        const int od = 2 * md + (cls >> 2), oh = 2 * mh + ((cls >> 1) & 1), ow = 2 * mw + (cls & 1);
        const size_t o = (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co;
        const float4 s = skip ? *reinterpret_cast<const float4*>(skip + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 v;
        v.x = s.x + act(fmaf(acc[r][cls][m][0], al.x, sh.x), g.lo);
        v.y = s.y + act(fmaf(acc[r][cls][m][1], al.y, sh.y), g.lo);
        v.z = s.z + act(fmaf(acc[r][cls][m][2], al.z, sh.z), g.lo);
        v.w = s.w + act(fmaf(acc[r][cls][m][3], al.w, sh.w), g.lo);
        *reinterpret_cast<float4*>(y + o) = v;
      }
    }
  }
}

constexpr int kDChunk = 8;  // depth planes per thread in the full-resolution VALU convs

// ---------------------------------------------------------------- conv0: Cin=1 -> 8, VALU
// Same row-segment layout as prob_kernel below: a wave owns 62 output columns of one row, lane l
// column w0 + l - 1 (lanes 0 / 63 are the kw halo). Each input row is one coalesced dword per
// lane; kw neighbours come by DPP. The thread walks D with a 3-plane ring of its 3x3 windows;
// the next plane's raw rows are in flight while an output plane is computed.
// The 8 output channels are 4 packed pairs: one v_pk_fma per (tap, pair) with the weight pair
// {W[t][2cp], W[t][2cp+1]} (packing [27][Co]) and the tap value broadcast, the 4 chains
// interleaved (a dependent v_pk_fma issued back to back stalls a cycle). Every output still
// sees its taps in (kd, kh, kw) order. A lane stores its voxel's 8 channels (32 bytes): staging
// them through LDS for lane-contiguous stores measured slower here.
constexpr int kProbCols = 62;
typedef float float2_v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lane_from_left(float v) {  // lane l <- lane l-1 (wave_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_from_right(float v) {  // lane l <- lane l+1 (wave_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, false));
}

__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ x, float* __restrict__ y, int D, int H,
                                                    int W, const float* __restrict__ wt,
                                                    const float* __restrict__ alpha,
                                                    const float* __restrict__ shift, float lo) {
  const int HW = H * W;
  const int nseg = (W + kProbCols - 1) / kProbCols, nrow = (H + 3) / 4, ndc = (D + kDChunk - 1) / kDChunk;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = lb % nseg;
  lb /= nseg;
  const int rowb = lb % nrow;
  lb /= nrow;
  const int dc = lb % ndc;
  const int n = lb / ndc;
  const int lane = threadIdx.x & 63;
  const int h = rowb * 4 + (threadIdx.x >> 6);
  if (h >= H) return;  // whole wave
  const int w = seg * kProbCols + lane - 1;
  const bool writes = lane >= 1 && lane <= kProbCols && w < W;
  const int d0 = dc * kDChunk, d1 = min(D, d0 + kDChunk);
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)n * D * HW, (unsigned)(D * HW * 4));
  float* yp = y + ((size_t)n * D * HW + (size_t)h * W + w) * 8;
  const unsigned offw = (unsigned)w < (unsigned)W ? (unsigned)w * 4u : kOffOut;
  unsigned offh[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) offh[k] = (unsigned)(h - 1 + k) < (unsigned)H ? (unsigned)((h - 1 + k) * W) * 4u : kOffOut;
  auto load_raw = [&](int d, float (&o)[3]) {
    const unsigned offd = (unsigned)d < (unsigned)D ? (unsigned)d * (unsigned)HW * 4u : kOffOut;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const unsigned off = offd | offh[kh] | offw;  // any out-of-range term keeps the top bit
      o[kh] = buf_load_f32(rx, (offd + offh[kh] + offw) | (off & kOffOut));
    }
  };
  auto expand = [&](const float (&r)[3], float (&o)[3][3]) {
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      o[kh][0] = lane_from_left(r[kh]);
      o[kh][1] = r[kh];
      o[kh][2] = lane_from_right(r[kh]);
    }
  };
  float al[8], sh[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    al[c] = alpha[c];
    sh[c] = shift[c];
  }
  float win[3][3][3];
  // one output plane; `raw` holds plane d+1's rows and is refilled with plane d+2's
  auto step = [&](int d, float (&raw)[3]) {
    expand(raw, win[2]);
    load_raw(d + 2, raw);
    const float* wk = wt;
    float2_v a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int t = 0; t < 27; ++t) {
      const float xv = win[t / 9][(t / 3) % 3][t % 3];
#pragma unroll
      for (int cp = 0; cp < 4; ++cp)
        a[cp] = __builtin_elementwise_fma(*reinterpret_cast<const float2_v*>(wk + t * 8 + 2 * cp), float2_v{xv, xv},
                                          a[cp]);
    }
    float o[8];
#pragma unroll
    for (int cp = 0; cp < 4; ++cp) {
      o[2 * cp] = act(fmaf(a[cp].x, al[2 * cp], sh[2 * cp]), lo);
      o[2 * cp + 1] = act(fmaf(a[cp].y, al[2 * cp + 1], sh[2 * cp + 1]), lo);
    }
    if (writes) {
      float4* q = reinterpret_cast<float4*>(yp + (size_t)d * HW * 8);
      q[0] = make_float4(o[0], o[1], o[2], o[3]);
      q[1] = make_float4(o[4], o[5], o[6], o[7]);
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        win[0][kh][k] = win[1][kh][k];
        win[1][kh][k] = win[2][kh][k];
      }
  };
  float ra[3];
  load_raw(d0 - 1, ra);
  expand(ra, win[0]);
  load_raw(d0, ra);
  expand(ra, win[1]);
  load_raw(d0 + 1, ra);
  for (int d = d0; d < d1; ++d) step(d, ra);
}

// ---------------------------------------------------------------- prob: 8 -> 1, VALU
// A wave owns one (h) row segment of 62 output columns; lane l holds column w0 + l - 1 (lanes
// 0 and 63 are the kw halo and write nothing). Every input row is one coalesced 32-byte load
// per lane (the segment's 64 pixels are 2 KB contiguous); the kw = 0 / 2 neighbours come from
// lanes l -+ 1 by wave-wide DPP shifts instead of re-gathering them (the 3x re-read of the
// 1-pixel-per-thread form made this kernel address-unit bound). The thread walks kDChunk output
// planes (prob_walk).

// The D walk both prob kernels run: input plane i (3 rows x 3 taps x 8 channels) feeds outputs
// i+1 (kd=0), i (kd=1) and i-1 (kd=2), each output's FMA chain in (kd, kh, kw, c) order:
// c12 = {output i (kd=0 done, adds kd=1), output i-1 (kd=0,1 done, adds kd=2)}, one packed FMA per
// (tap, channel) with the weight pair {W[kd=1], W[kd=2]} (an aligned SGPR pair, see the host
// packing in include/transmvs.h) and x broadcast; acc_next (output i+1, kd=0) is scalar.
// Planes d0-1 .. d0+8 (kDChunk + 2), double-buffered: plane i+1's three rows are in flight while
// plane i is consumed (with one row of lookahead a wave had a single load outstanding and the
// kernels ran at 2.3-2.5 TB/s). emit(d, logit) for d = d0 .. d0+7 (the caller bounds d by D).
// the same for prob_walk's plane loop (prob_kernel, stage 1: 38.6 -> 37.2 us, bitwise the same, r18z2)
#ifndef TMVS_PROB1_UNIFORM
#define TMVS_PROB1_UNIFORM 1
#endif
template <typename Emit>
__device__ __forceinline__ void prob_walk(__amdgpu_buffer_rsrc_t rx, int w, int h, int D, int H, int W, int d0,
                                          const float* __restrict__ wt, Emit emit) {
  const unsigned offw = (unsigned)w < (unsigned)W ? (unsigned)w * 32u : kOffOut;
  auto load_plane = [&](int i, float4 (&o)[3][2]) {
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = h - 1 + kh;
      const unsigned offr = ((unsigned)i < (unsigned)D && (unsigned)ih < (unsigned)H)
                                ? ((unsigned)i * (unsigned)H + (unsigned)ih) * (unsigned)W * 32u
                                : kOffOut;
      const unsigned off = (offr + offw) | ((offr | offw) & kOffOut);
      const floatx4 u = buf_load_f32x4(rx, off);
      const floatx4 v = buf_load_f32x4(rx, off + 16u);
      o[kh][0] = make_float4(u[0], u[1], u[2], u[3]);
      o[kh][1] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  float2_v c12 = {0.f, 0.f};
  auto plane = [&](int i, const float4 (&p)[3][2]) {
    float acc_next = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const float xc[8] = {p[kh][0].x, p[kh][0].y, p[kh][0].z, p[kh][0].w,
                           p[kh][1].x, p[kh][1].y, p[kh][1].z, p[kh][1].w};
      // the row's 72 weights through an opaque (uniform) offset: loaded where the row is consumed
      // instead of all 216 hoisted out of the plane loop into SGPRs (spills)
      int wo = kh * 72;
      asm volatile("" : "+s"(wo));
      const float* wk = wt + __builtin_amdgcn_readfirstlane(wo);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float xv = kw == 0 ? lane_from_left(xc[c]) : kw == 1 ? xc[c] : lane_from_right(xc[c]);
          const float2_v wp = *reinterpret_cast<const float2_v*>(wk + 2 * (kw * 8 + c));
          acc_next = fmaf(wk[48 + kw * 8 + c], xv, acc_next);
          c12 = __builtin_elementwise_fma(wp, float2_v{xv, xv}, c12);
        }
      }
      // both chains complete per row (no FMA sunk past the row: its shifted taps die here)
      asm volatile("" : "+v"(acc_next), "+v"(c12));
    }
    if (i - 1 >= d0) emit(i - 1, c12.y);  // output i-1 complete
    c12 = float2_v{acc_next, c12.x};
  };
  float4 pa[3][2], pb[3][2];
#if TMVS_PROB1_UNIFORM
  d0 = __builtin_amdgcn_readfirstlane(d0);  // as in prob_walk_rows (TMVS_PROB_UNIFORM)
#endif
  load_plane(d0 - 1, pa);
#if TMVS_PROB1_UNIFORM
#pragma unroll
  for (int j = 0; j < kDChunk + 2; j += 2) {
    const int i = d0 - 1 + j;
#else
#pragma unroll 1
  for (int i = d0 - 1; i < d0 + kDChunk + 1; i += 2) {  // planes i (in pa) and i + 1 (in pb)
#endif
    load_plane(i + 1, pb);
    plane(i, pa);
    load_plane(i + 2, pa);  // (past the last plane: rows the next chunk reads anyway)
    plane(i + 1, pb);
  }
}

// prob_walk_rows' plane loop: 0 = divergent loop on the per-lane d0 (the latch copied the prefetched
// plane between buffers after a vmcnt(0)), 1 = d0 made wave-uniform, 2 = uniform and fully unrolled
// (r18z, bitwise the same: stage 3 89.6 -> 86.0 us, stage 2 94.7 -> 93.5 us; 1 alone 89.8 / 96.3; the
// same build re-run on another box in r18z2: 89.2 / 93.0 -- box-to-box spread of about 3 %)
#ifndef TMVS_PROB_UNIFORM
#define TMVS_PROB_UNIFORM 2
#endif
// prob_walk for NR consecutive output rows h .. h+NR-1 per wave: input plane i's rows h-1 .. h+NR are
// loaded once (NR+2 row loads per plane instead of 3 NR: the row re-reads had the kernels address-unit
// bound) and each row feeds the outputs it borders. Every output keeps prob_walk's FMA chains and
// order (kd, kh, kw, c), so the logits are bitwise prob_walk's. emit(r, d, logit).
template <int NR, typename Emit>
__device__ __forceinline__ void prob_walk_rows(__amdgpu_buffer_rsrc_t rx, int w, int h, int D, int H, int W, int d0,
                                               const float* __restrict__ wt, Emit emit) {
  constexpr int NL = NR + 2;
#if TMVS_PROB_UNIFORM
  // d0 is the wave's depth chunk: wave-uniform, but derived from threadIdx.x, so without this the plane
  // loop is a divergent (exec-mask) loop whose latch waits vmcnt(0) for the prefetched plane
  d0 = __builtin_amdgcn_readfirstlane(d0);
#endif
  const unsigned offw = (unsigned)w < (unsigned)W ? (unsigned)w * 32u : kOffOut;
  auto load_plane = [&](int i, float4 (&o)[NL][2]) {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int ih = h - 1 + j;
      const unsigned offr = ((unsigned)i < (unsigned)D && (unsigned)ih < (unsigned)H)
                                ? ((unsigned)i * (unsigned)H + (unsigned)ih) * (unsigned)W * 32u
                                : kOffOut;
      const unsigned off = (offr + offw) | ((offr | offw) & kOffOut);
      const floatx4 u = buf_load_f32x4(rx, off);
      const floatx4 v = buf_load_f32x4(rx, off + 16u);
      o[j][0] = make_float4(u[0], u[1], u[2], u[3]);
      o[j][1] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  float2_v c12[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) c12[r] = float2_v{0.f, 0.f};
  auto plane = [&](int i, const float4 (&p)[NL][2]) {
    float acc_next[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc_next[r] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      int wo = kh * 72;
      asm volatile("" : "+s"(wo));
      const float* wk = wt + __builtin_amdgcn_readfirstlane(wo);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int j = r + kh;  // input row h-1+j feeds output row h+r through weight row kh
        const float xc[8] = {p[j][0].x, p[j][0].y, p[j][0].z, p[j][0].w, p[j][1].x, p[j][1].y, p[j][1].z, p[j][1].w};
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float xv = kw == 0 ? lane_from_left(xc[c]) : kw == 1 ? xc[c] : lane_from_right(xc[c]);
            const float2_v wp = *reinterpret_cast<const float2_v*>(wk + 2 * (kw * 8 + c));
            acc_next[r] = fmaf(wk[48 + kw * 8 + c], xv, acc_next[r]);
            c12[r] = __builtin_elementwise_fma(wp, float2_v{xv, xv}, c12[r]);
          }
        }
        asm volatile("" : "+v"(acc_next[r]), "+v"(c12[r]));
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (i - 1 >= d0) emit(r, i - 1, c12[r].y);
      c12[r] = float2_v{acc_next[r], c12[r].x};
    }
  };
  float4 pa[NL][2], pb[NL][2];
  load_plane(d0 - 1, pa);
#if TMVS_PROB_UNIFORM >= 2
  // unrolled: no loop-carried plane buffers, whose register copies at the latch waited vmcnt(0)
#pragma unroll
  for (int j = 0; j < kDChunk + 2; j += 2) {
    const int i = d0 - 1 + j;
#else
#pragma unroll 1
  for (int i = d0 - 1; i < d0 + kDChunk + 1; i += 2) {
#endif
    load_plane(i + 1, pb);
    plane(i, pa);
    load_plane(i + 2, pa);
    plane(i + 1, pb);
  }
}

// rows per wave of the raw prob walk (prob_kernel: 1; the 2-row form measured 42.3 -> 44.9 us at stage 1's
// D = 48, 96.0 -> 92.1 / 90.9 -> 87.8 at stages 2 / 3, r16c) and of the fused prob + softmax/WTA kernel
// (stages 2 / 3)
#ifndef TMVS_PROB_ROWS
#define TMVS_PROB_ROWS 1
#endif
#ifndef TMVS_PROB_WTA_ROWS
#define TMVS_PROB_WTA_ROWS 2
#endif

// prob_kernel with NR output rows per wave (4 waves: 4 NR rows per workgroup)
template <int NR>
__global__ __launch_bounds__(256) void prob_rows_kernel(const float* __restrict__ x, float* __restrict__ y, int D, int H,
                                                        int W, const float* __restrict__ wt) {
  const int HW = H * W;
  const int nseg = (W + kProbCols - 1) / kProbCols, nrow = (H + 4 * NR - 1) / (4 * NR), ndc = (D + kDChunk - 1) / kDChunk;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = lb % nseg;
  lb /= nseg;
  const int rowb = lb % nrow;
  lb /= nrow;
  const int dc = lb % ndc;
  const int n = lb / ndc;
  const int lane = threadIdx.x & 63;
  const int h = (rowb * 4 + (threadIdx.x >> 6)) * NR;
  if (h >= H) return;  // whole wave
  const int w = seg * kProbCols + lane - 1;
  const bool writes = lane >= 1 && lane <= kProbCols && w < W;
  const int d0 = dc * kDChunk, d1 = min(D, d0 + kDChunk);
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)n * D * HW * 8, (unsigned)(D * HW * 32));
  float* yn = y + (size_t)n * D * HW + (size_t)h * W + w;
  prob_walk_rows<NR>(rx, w, h, D, H, W, d0, wt, [&](int r, int d, float v) {
    if (d < d1 && writes && h + r < H) yn[(size_t)d * HW + (size_t)r * W] = v;
  });
}

// prob_wta_kernel with NR rows per workgroup: wave k walks depth chunk k of all NR rows; after the
// barrier the first waves run the softmax / WTA of one row each (wave 0 of all rows when D = 8)
template <int D, int NR>
__global__ __launch_bounds__(64 * (D / kDChunk)) void prob_wta_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ hyp, int H, int W, float lo,
    float hi, float* __restrict__ prob, float* __restrict__ depth, float* __restrict__ depth_raw,
    float* __restrict__ conf) {
  constexpr int NW = D / kDChunk;
  __shared__ float lg[NR][D * 64];
  const int HW = H * W;
  const int nseg = (W + kProbCols - 1) / kProbCols, nrow = (H + NR - 1) / NR;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = lb % nseg;
  lb /= nseg;
  const int h0 = (lb % nrow) * NR;
  const int n = lb / nrow;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d0 = wv * kDChunk;
  const int w = seg * kProbCols + lane - 1;
  const bool writes = lane >= 1 && lane <= kProbCols && w < W;
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)n * D * HW * 8, (unsigned)(D * HW * 32));
  prob_walk_rows<NR>(rx, w, h0, D, H, W, d0, wt, [&](int r, int d, float v) { lg[r][d * 64 + lane] = v; });
  __syncthreads();
  if (!writes) return;
  for (int r = wv; r < NR; r += NW) {
    const int h = h0 + r;
    if (h >= H) break;
    float xl[D];
#pragma unroll
    for (int d = 0; d < D; ++d) xl[d] = lg[r][d * 64 + lane];
    const size_t base = (size_t)n * D * HW + (size_t)h * W + w;
    float best;
    const int bi = softmax_first_max<D>(xl, [&](int d, float pr) { prob[base + (size_t)d * HW] = pr; }, best);
    const size_t o = (size_t)n * HW + (size_t)h * W + w;
    const float dr = hyp[base + (size_t)bi * HW];
    depth_raw[o] = dr;
    depth[o] = fminf(fmaxf(dr, lo), hi);
    conf[o] = best;
  }
}

__global__ __launch_bounds__(256) void prob_kernel(const float* __restrict__ x, float* __restrict__ y, int D, int H,
                                                   int W, const float* __restrict__ wt) {
  const int HW = H * W;
  const int nseg = (W + kProbCols - 1) / kProbCols, nrow = (H + 3) / 4, ndc = (D + kDChunk - 1) / kDChunk;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = lb % nseg;
  lb /= nseg;
  const int rowb = lb % nrow;
  lb /= nrow;
  const int dc = lb % ndc;
  const int n = lb / ndc;
  const int lane = threadIdx.x & 63;
  const int h = rowb * 4 + (threadIdx.x >> 6);
  if (h >= H) return;  // whole wave
  const int w = seg * kProbCols + lane - 1;
  const bool writes = lane >= 1 && lane <= kProbCols && w < W;
  const int d0 = dc * kDChunk, d1 = min(D, d0 + kDChunk);
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)n * D * HW * 8, (unsigned)(D * HW * 32));
  float* yn = y + (size_t)n * D * HW + (size_t)h * W + w;
  prob_walk(rx, w, h, D, H, W, d0, wt, [&](int d, float v) {
    if (d < d1 && writes) yn[(size_t)d * HW] = v;
  });
}

// ---------------------------------------------------------------- prob + softmax / WTA, fused
// prob_kernel's row-segment D walk with the D / 8 depth chunks of one row segment as the waves of
// one workgroup (wave k walks planes 8k-1 .. 8k+8, exactly prob_kernel's chunk k); each wave parks
// its 8 logits per column in LDS ([D][64]) instead of HBM, and after one barrier wave 0 runs
// softmax_first_max (common.h, the code softmax_wta_kernel runs) per column and gathers the
// winning hypothesis (models/TransMVSNet.py:97-103,217-221). Same FMA chains as prob_kernel, so
// prob / depth / conf equal prob_kernel + softmax_wta_kernel bit for bit, without the logits'
// 8·D bytes per pixel of HBM traffic and one launch; same wave count as prob_kernel.
template <int D>
__global__ __launch_bounds__(64 * (D / kDChunk)) void prob_wta_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ hyp, int H, int W, float lo,
    float hi, float* __restrict__ prob, float* __restrict__ depth, float* __restrict__ depth_raw,
    float* __restrict__ conf) {
  __shared__ float lg[D * 64];
  const int HW = H * W;
  const int nseg = (W + kProbCols - 1) / kProbCols;
  int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = lb % nseg;
  lb /= nseg;
  const int h = lb % H;
  const int n = lb / H;
  const int lane = threadIdx.x & 63;
  const int d0 = (threadIdx.x >> 6) * kDChunk;
  const int w = seg * kProbCols + lane - 1;
  const bool writes = lane >= 1 && lane <= kProbCols && w < W;
  const __amdgpu_buffer_rsrc_t rx = raw_rsrc(x + (size_t)n * D * HW * 8, (unsigned)(D * HW * 32));
  prob_walk(rx, w, h, D, H, W, d0, wt, [&](int d, float v) { lg[d * 64 + lane] = v; });
  __syncthreads();
  if (threadIdx.x >= 64 || !writes) return;
  float xl[D];
#pragma unroll
  for (int d = 0; d < D; ++d) xl[d] = lg[d * 64 + lane];
  const size_t base = (size_t)n * D * HW + (size_t)h * W + w;
  float best;
  const int bi = softmax_first_max<D>(xl, [&](int d, float pr) { prob[base + (size_t)d * HW] = pr; }, best);
  const size_t o = (size_t)n * HW + (size_t)h * W + w;
  const float dr = hyp[base + (size_t)bi * HW];
  depth_raw[o] = dr;
  depth[o] = fminf(fmaxf(dr, lo), hi);
  conf[o] = best;
}


// ---------------------------------------------------------------- conv 16 -> 16, stride 1 (conv2)
// Persistent form of conv3d_lds_kernel for the one stride-1 layer whose weights fit in LDS next
// to a tile (27 x 16 x 16 fp32 = 27 KB): a workgroup stages them once, then walks its share of
// 2x4x16-voxel output tiles; the next tile's input is fetched into registers while the
// current tile's 27 taps run on the MFMAs, and committed to LDS between two barriers.
// Same fragment layouts, tap order and epilogue as conv3d_lds_kernel.
// NWV waves per workgroup (4, or 8 = two workgroups' rows in one: the staged weights shared by twice
// the waves, 4 waves/SIMD at <= 128 VGPRs instead of 2 workgroups x 4 waves at 2 waves/SIMD)
template <int TD, int TH, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(NWV == 8 ? 4 : 2))) void conv3d_c16_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ shift, float* __restrict__ y, Geo g,
                                                         int ntiles) {
  constexpr int C = 16, PL = 4, NBW = TD * TH / NWV, NTH = NWV * 64;
  static_assert(TD * TH % NWV == 0, "rows split evenly over the waves");
  constexpr int LW = 18, LH = TH + 2, LD = TD + 2, VST = 16;
  constexpr int NVOX = LD * LH * LW;
  constexpr int NLD = (NVOX * 4 + NTH - 1) / NTH;
  __shared__ __attribute__((aligned(16))) float tile[NVOX * VST];
  __shared__ __attribute__((aligned(16))) float wts[27 * 16 * 16];
  const int nws = (g.Wo + 15) / 16, nhs = (g.Ho + TH - 1) / TH, nds = (g.Do + TD - 1) / TD;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  const int nxcd = gridDim.x >= 8 ? 8 : 1, per_xcd = gridDim.x / nxcd;
  const int xcd = blockIdx.x % nxcd, kx = blockIdx.x / nxcd;
  const int t_lo = (int)((long)ntiles * xcd / nxcd), t_hi = (int)((long)ntiles * (xcd + 1) / nxcd);
  if (kx >= per_xcd) return;
  struct TileCoord {
    int n, od0, oh0, ow0;
  };
  auto coord = [&](int t) {
    TileCoord c;
    c.ow0 = (t % nws) * 16;
    t /= nws;
    c.oh0 = (t % nhs) * TH;
    t /= nhs;
    c.od0 = (t % nds) * TD;
    c.n = t / nds;
    return c;
  };
  float4 pf[NLD];
  auto fetch = [&](int t) {
    const TileCoord c = coord(t);
    const size_t in_n = (size_t)c.n * g.Di * g.Hi * g.Wi;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + NTH * k;
      const int vox = idx >> 2, q = idx & 3;
      const int lw = vox % LW, rest = vox / LW, lh = rest % LH, ld = rest / LH;
      const int iw = c.ow0 - 1 + lw, ih = c.oh0 - 1 + lh, id = c.od0 - 1 + ld;
      pf[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vox < NVOX && (unsigned)iw < (unsigned)g.Wi && (unsigned)ih < (unsigned)g.Hi && (unsigned)id < (unsigned)g.Di)
        pf[k] = *reinterpret_cast<const float4*>(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * C + 4 * q);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + NTH * k;
      const int vox = idx >> 2, q = idx & 3;
      if (vox < NVOX) *reinterpret_cast<float4*>(tile + vox * VST + 4 * (q ^ ((vox >> 1) & 3))) = pf[k];
    }
  };
  for (int idx = threadIdx.x; idx < 27 * 16 * 4; idx += NTH) {
    const int q = idx & 3, row = (idx >> 2) & 15, tap = idx >> 6;
    const float4 v = *reinterpret_cast<const float4*>(wpk + ((size_t)tap * C + row) * C + 4 * q);
    *reinterpret_cast<float4*>(wts + (tap * 16 + row) * 16 + 4 * (q ^ ((row >> 1) & 3))) = v;
  }
  const float4 al = *reinterpret_cast<const float4*>(alpha + kgrp * 4);
  const float4 sh = *reinterpret_cast<const float4*>(shift + kgrp * 4);
  int t = t_lo + kx;
  if (t < t_hi) {
    fetch(t);
    commit();
  }
  __syncthreads();
  for (; t < t_hi; t += per_xcd) {
    const TileCoord c = coord(t);
    const int tn = t + per_xcd;
    if (tn < t_hi) fetch(tn);
    floatx4 acc[NBW];
#pragma unroll
    for (int r = 0; r < NBW; ++r) acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 27; ++tap) {
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      VecN<PL> a;
      a.load(wts + (tap * 16 + col) * 16 + 4 * (kgrp ^ ((col >> 1) & 3)));
      VecN<PL> b[NBW];
#pragma unroll
      for (int r = 0; r < NBW; ++r) {
        const int rr = wv * NBW + r;
        const int odl = rr / TH, ohl = rr - odl * TH;
        const int lvox = ((odl + kd) * LH + ohl + kh) * LW + col + kw;
        b[r].load(tile + lvox * VST + 4 * (kgrp ^ ((lvox >> 1) & 3)));
      }
#pragma unroll
      for (int j = 0; j < PL; ++j)
#pragma unroll
        for (int r = 0; r < NBW; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b[r].v[j], acc[r], 0, 0, 0);
      if (tap % (NBW > 2 ? 3 : 9) == (NBW > 2 ? 2 : 8)) __builtin_amdgcn_sched_barrier(0);  // bound the fragments in flight
    }
    const int ow = c.ow0 + col;
    const size_t out_n = (size_t)c.n * g.Do * g.Ho * g.Wo;
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = wv * NBW + r;
      const int od = c.od0 + rr / TH, oh = c.oh0 + rr % TH;
      if (ow >= g.Wo || od >= g.Do || oh >= g.Ho) continue;
      float4 o;
      o.x = act(fmaf(acc[r][0], al.x, sh.x), g.lo);
      o.y = act(fmaf(acc[r][1], al.y, sh.y), g.lo);
      o.z = act(fmaf(acc[r][2], al.z, sh.z), g.lo);
      o.w = act(fmaf(acc[r][3], al.w, sh.w), g.lo);
      *reinterpret_cast<float4*>(y + (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * C + kgrp * 4) = o;
    }
    __syncthreads();  // every wave is done with the tile
    if (tn < t_hi) commit();
    __syncthreads();
  }
}

// residency of a persistent kernel: resident workgroups per CU x CUs (queried once per kernel)
template <typename K>
static int persistent_grid(K kernel, long ntiles, int block = 256) {
  struct Entry {
    const void* fn;
    int dev, cap;
  };
  static Entry cache[16];
  static int used = 0;
  int dev = 0;
  hipGetDevice(&dev);
  for (int i = 0; i < used; ++i)
    if (cache[i].fn == (const void*)kernel && cache[i].dev == dev) return (int)std::min<long>(ntiles, cache[i].cap);
  int cus = 0, per = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0);
  const int cap = std::max(8, cus * std::max(per, 1));
  if (used < 16) cache[used++] = Entry{(const void*)kernel, dev, cap};
  return (int)std::min<long>(ntiles, cap);
}

#ifndef TMVS_C16_NWV
#define TMVS_C16_NWV 4
#endif
template <int TD, int TH>
static int launch_conv_c16(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                           const Geo& g, hipStream_t st) {
  constexpr int NWV = TMVS_C16_NWV;
  const long ntiles = (long)B * ((g.Do + TD - 1) / TD) * ((g.Ho + TH - 1) / TH) * ((g.Wo + 15) / 16);
  const int grid = persistent_grid(conv3d_c16_kernel<TD, TH, NWV>, ntiles, NWV * 64);
  hipLaunchKernelGGL((conv3d_c16_kernel<TD, TH, NWV>), dim3(grid), dim3(NWV * 64), 0, st, x, w, al, sh, y, g,
                     (int)ntiles);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// ---------------------------------------------------------------- conv1: 8 -> 16, stride 2, persistent
// A persistent workgroup keeps the 13.8 KB of
// weights in LDS and walks 2x4x16-output tiles; a tile's 5x9x33-voxel input footprint (8
// channels, 32 B per voxel) is staged with W split by parity -- [d][h][w&1][w>>1][8] -- so the
// stride-2 taps of 16 consecutive outputs read 16 consecutive voxels (kw 0/1/2 -> parity
// 0/1/0, index col + kw/2): conflict-free ds_read_b128 with no address-unit waste. The next
// tile is fetched into registers during the current tile's MFMAs.
// Tap pairs: with 8 input channels a per-tap B fragment would be 2 channels per lane. The 27
// taps are taken in pairs (a, b): lanes kgrp 0/1 read channel quads 0/1 of tap a, lanes 2/3
// of tap b, one 16-byte read each; MFMA j contracts k = (tap, quad) over channel j of each
// quad, and the A fragments are laid out to match (the 14th pair is half empty).
template <int TD, int TH, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(NWV == 8 ? 4 : 1))) void conv3d_s2c8_tile_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ wpk,
                                                               const float* __restrict__ alpha,
                                                               const float* __restrict__ shift, float* __restrict__ y,
                                                               Geo g, int ntiles) {
  constexpr int CIN = 8, COUT = 16, NBW = TD * TH / NWV, NTH = NWV * 64;
  static_assert(TD * TH % NWV == 0, "rows split evenly over the waves");
  // (SW = 20, which offsets the staging writes' odd-column voxels by 32 banks, measured the same: r16g)
  constexpr int LW = 33, LH = 2 * TH + 1, LD = 2 * TD + 1, SW = 17;
  constexpr int NROW = LD * LH, NQ = NROW * LW * 2;  // float4 quads per tile
  constexpr int NLD = (NQ + NTH - 1) / NTH;
  __shared__ __attribute__((aligned(16))) float tile[NROW * 2 * SW * 8];
  __shared__ __attribute__((aligned(16))) float wts[28 * 16 * 8];
  const int nws = (g.Wo + 15) / 16, nhs = (g.Ho + TH - 1) / TH, nds = (g.Do + TD - 1) / TD;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  const int half = kgrp & 1, side = kgrp >> 1;
  const int nxcd = gridDim.x >= 8 ? 8 : 1, per_xcd = gridDim.x / nxcd;
  const int xcd = blockIdx.x % nxcd, kx = blockIdx.x / nxcd;
  const int t_lo = (int)((long)ntiles * xcd / nxcd), t_hi = (int)((long)ntiles * (xcd + 1) / nxcd);
  if (kx >= per_xcd) return;
  struct TileCoord {
    int n, od0, oh0, ow0;
  };
  auto coord = [&](int t) {
    TileCoord c;
    c.ow0 = (t % nws) * 16;
    t /= nws;
    c.oh0 = (t % nhs) * TH;
    t /= nhs;
    c.od0 = (t % nds) * TD;
    c.n = t / nds;
    return c;
  };
  float4 pf[NLD];
  auto fetch = [&](int t) {
    const TileCoord c = coord(t);
    const size_t in_n = (size_t)c.n * g.Di * g.Hi * g.Wi;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + NTH * k;
      const int q = idx & 1, v = idx >> 1;
      const int lw = v % LW, row = v / LW, lh = row % LH, ld = row / LH;
      const int iw = 2 * c.ow0 - 1 + lw, ih = 2 * c.oh0 - 1 + lh, id = 2 * c.od0 - 1 + ld;
      pf[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < NQ && (unsigned)iw < (unsigned)g.Wi && (unsigned)ih < (unsigned)g.Hi && (unsigned)id < (unsigned)g.Di)
        pf[k] = *reinterpret_cast<const float4*>(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * CIN + 4 * q);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + NTH * k;
      const int q = idx & 1, v = idx >> 1;
      const int lw = v % LW, row = v / LW;
      if (idx < NQ) *reinterpret_cast<float4*>(tile + ((row * 2 + (lw & 1)) * SW + (lw >> 1)) * 8 + 4 * q) = pf[k];
    }
  };
  for (int idx = threadIdx.x; idx < 28 * 16 * 2; idx += NTH) {  // tap 27: zero (the empty half of pair 13)
    const int q = idx & 1, row = (idx >> 1) & 15, tap = idx >> 5;
    const float4 v = tap < 27 ? *reinterpret_cast<const float4*>(wpk + ((size_t)tap * COUT + row) * CIN + 4 * q)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(wts + (tap * 16 + row) * 8 + 4 * q) = v;
  }
  const int co = kgrp * 4;
  const float4 al = *reinterpret_cast<const float4*>(alpha + co);
  const float4 sh = *reinterpret_cast<const float4*>(shift + co);
  int t = t_lo + kx;
  if (t < t_hi) {
    fetch(t);
    commit();
  }
  __syncthreads();
  for (; t < t_hi; t += per_xcd) {
    const TileCoord c = coord(t);
    const int tn = t + per_xcd;
    if (tn < t_hi) fetch(tn);
    floatx4 acc[NBW];
#pragma unroll
    for (int r = 0; r < NBW; ++r) acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pr = 0; pr < 14; ++pr) {
      const int tap = 2 * pr + side;
      const int tp = tap < 27 ? tap : 26;  // the empty tap reads a real voxel against zero weights
      const int kd = tp / 9, kh = (tp / 3) % 3, kw = tp % 3;
      const float4 a = *reinterpret_cast<const float4*>(wts + (tap * 16 + col) * 8 + 4 * half);
      float4 b[NBW];
#pragma unroll
      for (int r = 0; r < NBW; ++r) {
        const int rr = wv * NBW + r;
        const int odl = rr / TH, ohl = rr - odl * TH;
        const int row = (2 * odl + kd) * LH + 2 * ohl + kh;
        b[r] = *reinterpret_cast<const float4*>(tile + ((row * 2 + (kw & 1)) * SW + col + (kw >> 1)) * 8 + 4 * half);
      }
      // component-major: consecutive MFMAs alternate accumulators (no back-to-back dependence)
#pragma unroll
      for (int r = 0; r < NBW; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[r].x, acc[r], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < NBW; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[r].y, acc[r], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < NBW; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[r].z, acc[r], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < NBW; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[r].w, acc[r], 0, 0, 0);
    }
    const int ow = c.ow0 + col;
    const size_t out_n = (size_t)c.n * g.Do * g.Ho * g.Wo;
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = wv * NBW + r;
      const int od = c.od0 + rr / TH, oh = c.oh0 + rr % TH;
      if (ow >= g.Wo || od >= g.Do || oh >= g.Ho) continue;
      float4 o;
      o.x = act(fmaf(acc[r][0], al.x, sh.x), g.lo);
      o.y = act(fmaf(acc[r][1], al.y, sh.y), g.lo);
      o.z = act(fmaf(acc[r][2], al.z, sh.z), g.lo);
      o.w = act(fmaf(acc[r][3], al.w, sh.w), g.lo);
      *reinterpret_cast<float4*>(y + (out_n + ((size_t)od * g.Ho + oh) * g.Wo + ow) * COUT + co) = o;
    }
    __syncthreads();
    if (tn < t_hi) commit();
    __syncthreads();
  }
}

#ifndef TMVS_S2C8_NWV
#define TMVS_S2C8_NWV 4
#endif
template <int TD, int TH>
static int launch_conv_s2c8_tile(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                                 const Geo& g, hipStream_t st) {
  const long ntiles = (long)B * ((g.Do + TD - 1) / TD) * ((g.Ho + TH - 1) / TH) * ((g.Wo + 15) / 16);
  constexpr int NWV = TMVS_S2C8_NWV;
  const int grid = persistent_grid(conv3d_s2c8_tile_kernel<TD, TH, NWV>, ntiles, NWV * 64);
  hipLaunchKernelGGL((conv3d_s2c8_tile_kernel<TD, TH, NWV>), dim3(grid), dim3(NWV * 64), 0, st, x, w, al, sh, y, g,
                     (int)ntiles);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// ---------------------------------------------------------------- launchers
#ifndef TMVS_KDSKIP_MAX_DO
#define TMVS_KDSKIP_MAX_DO 2
#endif
template <int CIN, int COUT, int S, int TD, int TH, int MBB, int WS = 1>
static int launch_conv(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                       const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBB;
  const long nblk = (long)B * ((g.Do + TD - 1) / TD) * ((g.Ho + TH - 1) / TH) * ((g.Wo + 15) / 16) * MG;
  // output depth <= 2 (the coarse levels of a D = 8 stage): every wave has a depth-padding kd slice
  if (g.Do <= TMVS_KDSKIP_MAX_DO)
    hipLaunchKernelGGL((conv3d_lds_kernel<CIN, COUT, S, TD, TH, MBB, WS, true>), dim3((unsigned)nblk), dim3(256), 0, st,
                       x, w, al, sh, y, g);
  else
    hipLaunchKernelGGL((conv3d_lds_kernel<CIN, COUT, S, TD, TH, MBB, WS>), dim3((unsigned)nblk), dim3(256), 0, st, x, w,
                       al, sh, y, g);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int CIN, int COUT, int S, int TD, int TH, int MBB, int WS>
static int launch_conv_tapout(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                              const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBB;
  const long nblk = (long)B * ((g.Do + TD - 1) / TD) * ((g.Ho + TH - 1) / TH) * ((g.Wo + 15) / 16) * MG;
  hipLaunchKernelGGL((conv3d_lds_kernel<CIN, COUT, S, TD, TH, MBB, WS, false, true>), dim3((unsigned)nblk), dim3(256), 0,
                     st, x, w, al, sh, y, g);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int CIN, int COUT, int S, int NBW, int MBW>
static int launch_conv_direct(const float* x, const float* w, const float* al, const float* sh, float* y, int B,
                              const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBW;
  const long n_tasks = (long)B * g.Do * ((g.Ho + NBW - 1) / NBW) * ((g.Wo + 15) / 16) * MG;
  const int nblk = (int)((n_tasks + 3) / 4);
  hipLaunchKernelGGL((conv3d_direct_kernel<CIN, COUT, S, NBW, MBW>), dim3(nblk), dim3(256), 0, st, x, w, al, sh, y, g,
                     (int)n_tasks);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// ---------------------------------------------------------------- deconv 16 -> 8 (conv11)
// With 8 output channels a 16-row MFMA block would be half empty. Here rows 0-7 and 8-15 hold
// the two W-parity outputs 2m and 2m+1 of one input column m: for each (d, h) tap the first
// MFMA group applies kw=1 (rows 0-7) and kw=2 (rows 8-15) to input column m, the second
// applies kw=0 (rows 8-15 only) to column m+1 -- 8 instead of 12 MFMAs per (d, h) tap and all
// 64 lanes carry output.
// Persistent: a workgroup stages the 13.8 KB of weights in LDS once and then walks its share
// of the tiles (restaging them per 4-row tile moved as many bytes as the input itself). Input
// tiles are double-buffered in LDS -- the next tile's global loads are issued before the
// current tile's MFMAs and land in the other buffer after them -- and the skip (conv0) rows
// are requested before the MFMAs too, so neither latency sits between MFMA phases.
// Tiles are dealt out XCD-contiguously (an XCD's workgroups share one L2: neighbouring tiles
// share their halo voxels).
template <int TDI, int THI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void deconv3d_c8_kernel(const float* __restrict__ x, const float* __restrict__ wpk,
                                                          const float* __restrict__ alpha,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ skip, float* __restrict__ y,
                                                          Geo g, int ntiles) {
  constexpr int CIN = 16, COUT = 8, PL = 4;
  constexpr int NBW = TDI * THI / 4;
  constexpr int LW = 17, LH = THI + 1, LD = TDI + 1, VST = 16;
  constexpr int NVOX = LD * LH * LW;
  constexpr int NLD = (NVOX * 4 + 255) / 256;  // float4 staging loads per thread and tile
  static_assert((TDI * THI) % 4 == 0, "tile");
  __shared__ __attribute__((aligned(16))) float tile[2][NVOX * VST];
  __shared__ __attribute__((aligned(16))) float wts[27 * 8 * 16];
  __shared__ __attribute__((aligned(16))) float ep[4][32 * 8];

  const int nws = (g.Wi + 15) / 16, nhs = (g.Hi + THI - 1) / THI, nds = (g.Di + TDI - 1) / TDI;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kgrp = lane >> 4;
  // XCD-contiguous tile ranges: workgroup b runs on XCD b % 8 (round-robin dispatch)
  const int nxcd = gridDim.x >= 8 ? 8 : 1, per_xcd = gridDim.x / nxcd;
  const int xcd = blockIdx.x % nxcd, kx = blockIdx.x / nxcd;
  const int t_lo = (int)((long)ntiles * xcd / nxcd), t_hi = (int)((long)ntiles * (xcd + 1) / nxcd);
  if (kx >= per_xcd) return;  // grid not a multiple of 8: the remainder idles

  struct TileCoord {
    int n, md0, mh0, mw0;
  };
  auto coord = [&](int t) {
    TileCoord c;
    c.mw0 = (t % nws) * 16;
    t /= nws;
    c.mh0 = (t % nhs) * THI;
    t /= nhs;
    c.md0 = (t % nds) * TDI;
    c.n = t / nds;
    return c;
  };
  float4 pf[NLD];
  auto fetch = [&](int t) {  // global -> registers
    const TileCoord c = coord(t);
    const size_t in_n = (size_t)c.n * g.Di * g.Hi * g.Wi;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int vox = idx >> 2, q = idx & 3;
      const int lw = vox % LW, rest = vox / LW, lh = rest % LH, ld = rest / LH;
      const int iw = c.mw0 + lw, ih = c.mh0 + lh, id = c.md0 + ld;
      pf[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vox < NVOX && iw < g.Wi && ih < g.Hi && id < g.Di)
        pf[k] = *reinterpret_cast<const float4*>(x + (in_n + ((size_t)id * g.Hi + ih) * g.Wi + iw) * CIN + 4 * q);
    }
  };
  auto commit = [&](float* buf) {  // registers -> LDS (quad-swizzled voxels)
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int vox = idx >> 2, q = idx & 3;
      if (vox < NVOX) *reinterpret_cast<float4*>(buf + vox * VST + 4 * (q ^ ((vox >> 1) & 3))) = pf[k];
    }
  };

  for (int idx = threadIdx.x; idx < 27 * 8 * 4; idx += 256) {
    const int q = idx & 3, row = (idx >> 2) & 7, tap = idx >> 5;
    const float4 v = *reinterpret_cast<const float4*>(wpk + ((size_t)tap * COUT + row) * CIN + 4 * q);
    *reinterpret_cast<float4*>(wts + (tap * 8 + row) * 16 + 4 * (q ^ ((row >> 1) & 3))) = v;
  }
  const int co = col & 7;    // A row -> output channel
  const bool hi = col >= 8;  // rows 8-15: the odd-w output
  float* eb = ep[wv];
  const int cq = 4 * (kgrp & 1);
  const float4 al = *reinterpret_cast<const float4*>(alpha + cq);
  const float4 sh = *reinterpret_cast<const float4*>(shift + cq);
  auto wfrag = [&](int tap, VecN<PL>& a) { a.load(wts + (tap * 8 + co) * 16 + 4 * (kgrp ^ ((co >> 1) & 3))); };

  int t = t_lo + kx;
  if (t < t_hi) {
    fetch(t);
    commit(tile[0]);
  }
  __syncthreads();
  for (int it = 0; t < t_hi; t += per_xcd, ++it) {
    const float* cur = tile[it & 1];
    const TileCoord c = coord(t);
    const int tn = t + per_xcd;
    if (tn < t_hi) fetch(tn);
    // skip rows of this tile: lane (pair) j of a 1 KiB output row, as the epilogue stores it (storing each
    // lane's own MFMA outputs without the exchange measured 110.2 -> 112.6 us in the step, r16g)
    const size_t out_n = (size_t)c.n * g.Do * g.Ho * g.Wo;
    const int ow = 2 * c.mw0 + (lane >> 1);
    const size_t plane = (size_t)g.Ho * g.Wo * 8, row = (size_t)g.Wo * 8;  // output strides (floats)
    float4 sk[NBW][4];
    size_t oo[NBW];
    bool ok[NBW];
#pragma unroll
    for (int r = 0; r < NBW; ++r) {
      const int rr = wv * NBW + r;
      const int md = c.md0 + rr / THI, mh = c.mh0 + rr % THI;
      ok[r] = md < g.Di && mh < g.Hi && ow < 2 * g.Wi;
      oo[r] = (out_n + ((size_t)(2 * md) * g.Ho + 2 * mh) * g.Wo + ow) * 8 + (lane & 1) * 4;
#pragma unroll
      for (int pdh = 0; pdh < 4; ++pdh)
        sk[r][pdh] = (ok[r] && skip) ? *reinterpret_cast<const float4*>(skip + oo[r] + (pdh >> 1) * plane + (pdh & 1) * row)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    floatx4 acc[NBW][4];
#pragma unroll
    for (int r = 0; r < NBW; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[r][q] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pdh = 0; pdh < 4; ++pdh) {
      const int pd = pdh >> 1, ph = pdh & 1;
#pragma unroll
      for (int td = 0; td < 1 + pd; ++td)
#pragma unroll
        for (int th = 0; th < 1 + ph; ++th) {
          const int kd = pd ? (td ? 2 : 0) : 1, od_off = (pd && !td) ? 1 : 0;
          const int kh = ph ? (th ? 2 : 0) : 1, oh_off = (ph && !th) ? 1 : 0;
          const int tap_base = kd * 9 + kh * 3;
          VecN<PL> a1, a2;
          wfrag(tap_base + (hi ? 2 : 1), a1);  // rows 0-7: kw=1, rows 8-15: kw=2 (input column m)
          if (hi)
            wfrag(tap_base + 0, a2);           // rows 8-15: kw=0 (input column m+1)
          else
            a2.zero();
#pragma unroll
          for (int r = 0; r < NBW; ++r) {
            const int rr = wv * NBW + r;
            const int mdl = rr / THI, mhl = rr - mdl * THI;
            const int lv = ((mdl + od_off) * LH + mhl + oh_off) * LW + col;
            VecN<PL> b1, b2;
            b1.load(cur + lv * VST + 4 * (kgrp ^ ((lv >> 1) & 3)));
            b2.load(cur + (lv + 1) * VST + 4 * (kgrp ^ (((lv + 1) >> 1) & 3)));
#pragma unroll
            for (int j = 0; j < PL; ++j)
              acc[r][pdh] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.v[j], b1.v[j], acc[r][pdh], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < PL; ++j)
              acc[r][pdh] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2.v[j], b2.v[j], acc[r][pdh], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);  // one tap's fragments live at a time (VGPR budget)
        }
    }
    // epilogue: lane (col, kgrp) holds channels 4*(kgrp&1).. of output w 2*(mw0+col) + (kgrp>>1);
    // exchanged through LDS so the skip read and the store are contiguous 1 KiB rows
#pragma unroll
    for (int r = 0; r < NBW; ++r)
#pragma unroll
      for (int pdh = 0; pdh < 4; ++pdh) {
        const floatx4 a = acc[r][pdh];
        *reinterpret_cast<float4*>(eb + (2 * col + (kgrp >> 1)) * 8 + cq) =
            make_float4(act(fmaf(a[0], al.x, sh.x), g.lo), act(fmaf(a[1], al.y, sh.y), g.lo), act(fmaf(a[2], al.z, sh.z), g.lo),
                        act(fmaf(a[3], al.w, sh.w), g.lo));
        __builtin_amdgcn_wave_barrier();
        const float4 v = *reinterpret_cast<const float4*>(eb + lane * 4);
        __builtin_amdgcn_wave_barrier();
        const float4 sv = sk[r][pdh];
        if (ok[r])
          *reinterpret_cast<float4*>(y + oo[r] + (pdh >> 1) * plane + (pdh & 1) * row) =
              make_float4(sv.x + v.x, sv.y + v.y, sv.z + v.z, sv.w + v.w);
      }
    if (tn < t_hi) commit(tile[(it + 1) & 1]);
    __syncthreads();
  }
}

template <int TDI, int THI>
static int launch_deconv_c8(const float* x, const float* w, const float* al, const float* sh, const float* skip,
                            float* y, int B, const Geo& g, hipStream_t st) {
  const long ntiles = (long)B * ((g.Di + TDI - 1) / TDI) * ((g.Hi + THI - 1) / THI) * ((g.Wi + 15) / 16);
  const long grid = persistent_grid(deconv3d_c8_kernel<TDI, THI>, ntiles);
  hipLaunchKernelGGL((deconv3d_c8_kernel<TDI, THI>), dim3((unsigned)grid), dim3(256), 0, st, x, w, al, sh, skip, y, g,
                     (int)ntiles);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

template <int CIN, int COUT, int TDI, int THI, int MBB>
static int launch_deconv(const float* x, const float* w, const float* al, const float* sh, const float* skip,
                         float* y, int B, const Geo& g, hipStream_t st) {
  constexpr int MG = ((COUT + 15) / 16) / MBB;
  const long nblk = (long)B * ((g.Di + TDI - 1) / TDI) * ((g.Hi + THI - 1) / THI) * ((g.Wi + 15) / 16) * MG;
  hipLaunchKernelGGL((deconv3d_lds_kernel<CIN, COUT, TDI, THI, MBB>), dim3((unsigned)nblk), dim3(256), 0, st, x, w,
                     al, sh, skip, y, g);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

static int conv_dispatch(const float* x, int B, int cin, int d, int h, int w, const float* wpk, const float* al,
                         const float* sh, int cout, int stride, float* y, hipStream_t st, float lo = 0.f) {
  Geo g;
  g.lo = lo;
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
  // the MFMA kernels address one sample's input through a buffer with 32-bit byte offsets
  if ((long long)d * h * w * cin * 4 >= (1LL << 31)) return TMVS_ERR_SHAPE;
  // stride 1: LDS-staged tiles, one output depth slice x 8 rows x 16 columns per workgroup
#define TMVS_CONV_LDS(CI, CO, ...)                                                              \
  if (cin == CI && cout == CO && stride == 1) {                                               \
    return launch_conv<CI, CO, 1, __VA_ARGS__>(x, wpk, al, sh, y, B, g, st);                 \
  }
#ifndef TMVS_C16_TD
#define TMVS_C16_TD 2
#define TMVS_C16_TH 4
#endif
#ifdef TMVS_C16_LDS  // A/B: conv2 through the general LDS kernel (weights from L2) with this (TD, TH, MBB, WS)
  TMVS_CONV_LDS(16, 16, TMVS_C16_LDS)
#endif
  if (cin == 16 && cout == 16 && stride == 1)
    return launch_conv_c16<TMVS_C16_TD, TMVS_C16_TH>(x, wpk, al, sh, y, B, g, st);
#ifndef TMVS_C4_CFG
#define TMVS_C4_CFG 2, 2, 2, 2     // (TD, TH, MBB, WS) of conv4 (32 -> 32); output depth > 2 (r17h)
#endif
#ifndef TMVS_C4_CFG_KD
#define TMVS_C4_CFG_KD 2, 4, 2, 1  // output depth <= 2 (the depth-padding-skipping instance)
#endif
  if (cin == 32 && cout == 32 && stride == 1 && g.Do <= TMVS_KDSKIP_MAX_DO)
    return launch_conv<32, 32, 1, TMVS_C4_CFG_KD>(x, wpk, al, sh, y, B, g, st);
#ifndef TMVS_C6_CFG
#define TMVS_C6_CFG 1, 2, 4, 4  // and of conv6 (64 -> 64): each wave one output block (r17g)
#endif
#ifndef TMVS_C3_CFG
#define TMVS_C3_CFG 2, 2, 2, 2  // and of conv3 (16 -> 32, stride 2): 50.4 -> 46.0 us at stage 3 (r17n)
#endif
  TMVS_CONV_LDS(32, 32, TMVS_C4_CFG)
  TMVS_CONV_LDS(64, 64, TMVS_C6_CFG)
#undef TMVS_CONV_LDS
  // stride 2, 8 -> 16 (full-resolution input): tap pairs, 16-byte loads
#ifndef TMVS_S2C8_TD
#define TMVS_S2C8_TD 2  // 2x2 tiles: 3 workgroups per CU (41.5 KB LDS); 2x4 measured 103 vs 97-98 us (r12e)
#define TMVS_S2C8_TH 2
#endif
  if (cin == 8 && cout == 16 && stride == 2)
    return launch_conv_s2c8_tile<TMVS_S2C8_TD, TMVS_S2C8_TH>(x, wpk, al, sh, y, B, g, st);
#ifndef TMVS_S2_LDS
#define TMVS_S2_LDS 1
#endif
#if TMVS_S2_LDS
  // conv3 (16 -> 32, stride 2, one 16-channel chunk): the LDS-staged kernel -- each input voxel is
  // fetched once per tile instead of once per tap that reads it (the direct form's stride-2 lane
  // pattern half-fills every cache line it touches); same accumulation order as the direct kernel.
  // 63.8 -> 54.2 us per stage-2/3 call (r12k). (conv5 through the LDS kernel measured no faster
  // before the wave split, 58.0 vs 56.9 us, r12k; with it, below, it is.)
  if (cin == 16 && cout == 32 && stride == 2) return launch_conv<16, 32, 2, TMVS_C3_CFG>(x, wpk, al, sh, y, B, g, st);
#endif
  // stride 2: direct
#define TMVS_CONV_DIRECT(CI, CO, NBW, MBW) \
  if (cin == CI && cout == CO && stride == 2) return launch_conv_direct<CI, CO, 2, NBW, MBW>(x, wpk, al, sh, y, B, g, st);
  TMVS_CONV_DIRECT(8, 16, 4, 1)
  TMVS_CONV_DIRECT(16, 32, 4, 1)
#ifndef TMVS_C5_LDS
#define TMVS_C5_LDS 1, 2, 4, 4  // conv5 (32 -> 64, stride 2) through the LDS-tiled kernel, (TD, TH, MBB, WS)
#endif
  // conv5 through the wave-split LDS kernel: 52.6 -> 30.4 / 24.0 -> 15.5 / 24.2 -> 19.1 us (stages 2 / 1 / 3)
  // against the direct kernel's best tilings (2 rows x 2 blocks per wave on the stage-2/3 grids, 2 x 1 on
  // stage 1; r12r, r12s, r17j). TMVS_C5_MODE 2 (default): both 16-channel chunks staged, taps outer -- the
  // direct kernel's K order, so its sums bit for bit (round 6); 1: chunk-outer (round 5: re-associated
  // sums, one stage-2 near-tie flip at C2 cascading into 23 stage-3 pixels); 0: the direct kernel.
#ifndef TMVS_C5_MODE
#define TMVS_C5_MODE 2
#endif
  if (cin == 32 && cout == 64 && stride == 2) {
    if constexpr (TMVS_C5_MODE == 2) return launch_conv_tapout<32, 64, 2, TMVS_C5_LDS>(x, wpk, al, sh, y, B, g, st);
    if constexpr (TMVS_C5_MODE == 1) return launch_conv<32, 64, 2, TMVS_C5_LDS>(x, wpk, al, sh, y, B, g, st);
  }
  TMVS_CONV_DIRECT(32, 64, 2, 1)
#undef TMVS_CONV_DIRECT
  return TMVS_ERR_SHAPE;
}

static int deconv_dispatch(const float* x, int B, int cin, int d, int h, int w, const float* wpk, const float* al,
                           const float* sh, int cout, const float* skip, float* y, hipStream_t st, float lo = 0.f) {
  Geo g;
  g.lo = lo;
  g.Di = d;
  g.Hi = h;
  g.Wi = w;
  g.Do = 2 * d;
  g.Ho = 2 * h;
  g.Wo = 2 * w;
#ifndef TMVS_DECONV_EVEN
#define TMVS_DECONV_EVEN 2, 2  // (TDI, THI) input tile for an even input depth
#define TMVS_DECONV_ODD 1, 4   // and for an odd one
#endif
#define TMVS_DECONV_CASE(CI, CO, MBB)                                                                       \
  if (cin == CI && cout == CO) {                                                                           \
    if (g.Di % 2 == 0) return launch_deconv<CI, CO, TMVS_DECONV_EVEN, MBB>(x, wpk, al, sh, skip, y, B, g, st); \
    return launch_deconv<CI, CO, TMVS_DECONV_ODD, MBB>(x, wpk, al, sh, skip, y, B, g, st);                  \
  }
  TMVS_DECONV_CASE(64, 32, 1)
  TMVS_DECONV_CASE(32, 16, 1)
  if (cin == 16 && cout == 8) {  // W-parity outputs packed into the 16 MFMA rows
    if (g.Di % 2 == 0) return launch_deconv_c8<2, 2>(x, wpk, al, sh, skip, y, B, g, st);
    return launch_deconv_c8<1, 4>(x, wpk, al, sh, skip, y, B, g, st);
  }
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

static dim3 prob_grid(int batch, int D, int H, int W, int dchunk) {
  return dim3((unsigned)(((W + kProbCols - 1) / kProbCols) * ((H + 3) / 4) * batch * ((D + dchunk - 1) / dchunk)));
}

// prob (8 -> 1) raw logits: one row per wave (prob_kernel) or TMVS_PROB_ROWS rows per wave
static int launch_prob(const float* x, float* y, int batch, int D, int H, int W, const float* wt, hipStream_t st) {
  if constexpr (TMVS_PROB_ROWS > 1) {
    constexpr int NR = TMVS_PROB_ROWS;
    const dim3 grid((unsigned)(((W + kProbCols - 1) / kProbCols) * ((H + 4 * NR - 1) / (4 * NR)) * batch *
                               ((D + kDChunk - 1) / kDChunk)));
    hipLaunchKernelGGL(prob_rows_kernel<NR>, grid, dim3(256), 0, st, x, y, D, H, W, wt);
  } else {
    hipLaunchKernelGGL(prob_kernel, prob_grid(batch, D, H, W, kDChunk), dim3(256), 0, st, x, y, D, H, W, wt);
  }
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// alpha = 1, shift = 0 for the raw (training) form of the MFMA layers (64 = the widest layer)
__device__ float kUnitAlpha[64] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                   1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                   1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                   1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
__device__ float kZeroShift[64];

extern "C" int tmvs_conv3d_mfma(const float* x, int batch, int cin, int d, int h, int w, const float* wpk, int cout,
                                int stride, int transposed, const float* skip, float* y, void* stream) {
  if (!x || !wpk || !y || batch <= 0 || d <= 0 || h <= 0 || w <= 0) return TMVS_ERR_ARG;
  if (transposed ? stride != 2 : (stride != 1 && stride != 2)) return TMVS_ERR_ARG;
  if (skip && !transposed) return TMVS_ERR_ARG;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return TMVS_ERR_HIP;
  static const float* unit[64][2];  // per device: the symbols' addresses
  if (!unit[dev][0]) {
    void *a, *b;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(kUnitAlpha)) != hipSuccess ||
        hipGetSymbolAddress(&b, HIP_SYMBOL(kZeroShift)) != hipSuccess)
      return TMVS_ERR_HIP;
    unit[dev][1] = (const float*)b;
    unit[dev][0] = (const float*)a;
  }
  const float *al = unit[dev][0], *sh = unit[dev][1];
  const float lo = -__builtin_huge_valf();
  hipStream_t st = (hipStream_t)stream;
  if (!transposed && stride == 1 && cin == 1 && cout == 8) {  // conv0's VALU kernel, raw epilogue
    if ((long long)d * h * w * 32 >= (1LL << 31)) return TMVS_ERR_SHAPE;
    const dim3 grid((unsigned)(((w + kProbCols - 1) / kProbCols) * ((h + 3) / 4) * batch * ((d + kDChunk - 1) / kDChunk)));
    hipLaunchKernelGGL(conv0_kernel, grid, dim3(256), 0, st, x, y, d, h, w, wpk, al, sh, lo);
    TMVS_CHECK_LAUNCH();
    return TMVS_OK;
  }
  if (!transposed && stride == 1 && cin == 8 && cout == 1) {  // prob's VALU kernel (prob packing)
    if ((long long)d * h * w * 32 >= (1LL << 31)) return TMVS_ERR_SHAPE;
    return launch_prob(x, y, batch, d, h, w, wpk, st);
  }
  if (transposed) return deconv_dispatch(x, batch, cin, d, h, w, wpk, al, sh, cout, skip, y, st, lo);
  return conv_dispatch(x, batch, cin, d, h, w, wpk, al, sh, cout, stride, y, st, lo);
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

// CostRegNet up to conv11 + skip (models/module.py:447-455); *x11_out = the 8-channel
// full-resolution NDHWC volume the prob conv reads, *c0_out = conv0's (dead once x11 exists).
static int costregnet_trunk(const float* x, int batch, int depth, int height, int width, const TmvsCostRegWeights* w,
                            void* workspace, size_t workspace_bytes, hipStream_t st, float** x11_out,
                            float** c0_out) {
  if (!x || !w || !workspace || batch <= 0) return TMVS_ERR_ARG;
  if (depth % 8 || height % 8 || width % 8) return TMVS_ERR_SHAPE;
  if (w->base_ch != 8) return TMVS_ERR_SHAPE;
  // conv0 / prob address one sample's 8-channel full-resolution volume with 32-bit offsets
  if ((long long)depth * height * width * 32 >= (1LL << 31)) return TMVS_ERR_SHAPE;
  for (int i = 0; i < 11; ++i)
    if (!w->w[i]) return TMVS_ERR_ARG;
  for (int i = 0; i < 10; ++i)
    if (!w->alpha[i] || !w->shift[i]) return TMVS_ERR_ARG;
  if (workspace_bytes < tmvs_costregnet_workspace(batch, depth, height, width, w->base_ch)) return TMVS_ERR_ARG;
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
  const dim3 g0x((unsigned)(((W0 + kProbCols - 1) / kProbCols) * ((H0 + 3) / 4) * batch * ((D0 + kDChunk - 1) / kDChunk)));
  hipLaunchKernelGGL(conv0_kernel, g0x, dim3(256), 0, st, x, c0, D0, H0, W0, w->w[0], w->alpha[0], w->shift[0],
                     0.f);
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
  *x11_out = x11;
  *c0_out = c0;
  return TMVS_OK;
}

extern "C" int tmvs_costregnet(const float* x, int batch, int depth, int height, int width,
                               const TmvsCostRegWeights* w, void* workspace, size_t workspace_bytes, float* logits,
                               void* stream) {
  if (!logits) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  float *x11, *c0;
  int rc;
  if ((rc = costregnet_trunk(x, batch, depth, height, width, w, workspace, workspace_bytes, st, &x11, &c0))) return rc;
  return launch_prob(x11, logits, batch, depth, height, width, w->w[10], st);
}

extern "C" int tmvs_costregnet_wta(const float* x, const float* hyp, int batch, int depth, int height, int width,
                                   const TmvsCostRegWeights* w, void* workspace, size_t workspace_bytes,
                                   float clamp_lo, float clamp_hi, float* prob, float* depth_out, float* depth_raw,
                                   float* conf, void* stream) {
  if (!hyp || !prob || !depth_out || !depth_raw || !conf) return TMVS_ERR_ARG;
  switch (depth) {  // the D values tmvs_softmax_wta takes that CostRegNet's depth % 8 rule admits
    case 8: case 16: case 24: case 32: case 48: case 64: break;
    default: return TMVS_ERR_SHAPE;
  }
  hipStream_t st = (hipStream_t)stream;
  float *x11, *c0;
  int rc;
  if ((rc = costregnet_trunk(x, batch, depth, height, width, w, workspace, workspace_bytes, st, &x11, &c0))) return rc;
  if (depth > 32) {
    // D = 48 (stage 1) fused measured 53.8 us vs 40.1 + 10.3 us split (r07d vs r07b): few columns
    // and a 48-deep softmax tail behind the barrier. Split: the depth-chunked prob kernel, its
    // logits in conv0's buffer (dead once conv11 has consumed it as its skip), then the softmax kernel
    if ((rc = launch_prob(x11, c0, batch, depth, height, width, w->w[10], st))) return rc;
    return tmvs_softmax_wta(c0, hyp, batch, depth, height, width, clamp_lo, clamp_hi, prob, depth_out, depth_raw,
                            conf, stream);
  }
  // D <= 32: one workgroup per (sample, row, 62-column segment), its D/8 waves prob_kernel's depth
  // chunks. Measured (r07d vs r07b): D = 32 114.0 vs 108.4 + 15.7 us, D = 8 104.3 vs 90.9 + 18.6 us
  constexpr int NR = TMVS_PROB_WTA_ROWS;
  const dim3 gf((unsigned)(((width + kProbCols - 1) / kProbCols) * ((height + NR - 1) / NR) * batch));
  const dim3 bf((unsigned)(64 * (depth / kDChunk)));
#define TMVS_PW_CASE(DD)                                                                                      \
  case DD:                                                                                                    \
    if constexpr (NR > 1)                                                                                     \
      hipLaunchKernelGGL((prob_wta_rows_kernel<DD, NR>), gf, bf, 0, st, x11, w->w[10], hyp, height, width,    \
                         clamp_lo, clamp_hi, prob, depth_out, depth_raw, conf);                               \
    else                                                                                                      \
      hipLaunchKernelGGL(prob_wta_kernel<DD>, gf, bf, 0, st, x11, w->w[10], hyp, height, width, clamp_lo,     \
                         clamp_hi, prob, depth_out, depth_raw, conf);                                         \
    break;
  switch (depth) {
    TMVS_PW_CASE(8)
    TMVS_PW_CASE(16)
    TMVS_PW_CASE(24)
    TMVS_PW_CASE(32)
  }
#undef TMVS_PW_CASE
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
