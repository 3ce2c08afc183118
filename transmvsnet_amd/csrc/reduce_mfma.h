// Block-level reduction sum_p a[p][i] * b[p][j] on the fp32 matrix cores, shared by the weight-gradient
// kernels of costreg_train.hip and featurenet_train.hip (256-thread blocks).
#pragma once
#include "common.h"

namespace tmvs {

// sum_p a[p][i] b[p][j] over the block's rows [v0, v1) (A, BC multiples of 4): per 64-row chunk,
// D[a][b] += sum_r sa[r][a] sb[r][b] as v_mfma_f32_16x16x4f32 chains (A operand: lane l reads
// sa[4s + (l >> 4)][16 ma + (l & 15)], B operand sb[4s + (l >> 4)][16 nb + (l & 15)]; row strides
// A + 16 / BC + 16 floats put the 4 row groups of a read in disjoint bank ranges). The (A/16) x (BC/16)
// output tiles are dealt to the 4 waves; with fewer than 4 tiles, KS = 4 / tiles waves split each
// chunk's rows and are added in wave order at the end. fp32 within a chunk, fp64 across chunks.
// load_a(v, q) / load_b(v, q): float4 q of row v (zeros where a gathered tap is outside); out: the
// block's A x BC partial, fp64. The next chunk's rows are loaded into registers while this chunk's MFMAs run.
typedef float floatx4_t __attribute__((ext_vector_type(4)));
// BROW: thread t stages B quads 2(t&3), 2(t&3)+1 of row t>>2 (BC = 32) with one loader call
// load_b(v, q0, float4 (&)[2]) instead of quad t&7 of rows t>>3 and t>>3 + 32: a gathered B row whose
// loader derives per-row state (the DCN sample geometry) derives it once for both quads. Same LDS
// contents, same sums.
template <int A, int BC, bool BROW = false, typename LoadA, typename LoadB>
__device__ __forceinline__ void tile_reduce_mfma(long v0, long v1, LoadA load_a, LoadB load_b,
                                                 double* __restrict__ out) {
  // A or BC of 8 are zero-padded to 16 (half the matrix-core rows idle, still far above the VALU form)
  constexpr int AP = (A + 15) / 16 * 16, BP = (BC + 15) / 16 * 16;
  constexpr int CH = 64, SA = AP + 16, SB = BP + 16;
  constexpr int NT = (AP / 16) * (BP / 16);
  constexpr int TPW = NT >= 4 ? NT / 4 : 1;  // tiles per wave
  constexpr int KS = NT >= 4 ? 1 : 4 / NT;   // waves per tile (row split)
  static_assert(A % 4 == 0 && BC % 4 == 0 && (NT % 4 == 0 || 4 % NT == 0), "tile");
  constexpr int LA = CH * AP / 4 / 256, LB = CH * BP / 4 / 256;  // float4 loads per thread and chunk
  static_assert(CH * AP / 4 % 256 == 0 && CH * BP / 4 % 256 == 0, "staging");
  static_assert(!BROW || (BP == 32 && LB == 2), "BROW: 64 rows x 8 quads, 2 per thread");
  __shared__ __attribute__((aligned(16))) float lds[CH * (SA + SB)];
  __shared__ double cmb[KS > 1 ? (KS - 1) * NT * 256 : 1];
  float* sa = lds;
  float* sb = lds + CH * SA;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, kg = lane >> 4;
  const int ks = wv % KS;  // this wave's row slice
  double acc[TPW][4];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[t][r] = 0.0;
  float4 pa[LA], pb[LB];
  auto fetch = [&](long vb) {
#pragma unroll
    for (int k = 0; k < LA; ++k) {
      const int i = threadIdx.x + 256 * k, r = i / (AP / 4), q = i % (AP / 4);
      pa[k] = (vb + r < v1 && q < A / 4) ? load_a(vb + r, q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (BROW) {  // load_b(v, q0, float4 (&)[2]): quads q0, q0 + 1 of row v
      const int r = (int)threadIdx.x >> 2;
      pb[0] = pb[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vb + r < v1) load_b(vb + r, 2 * (int)(threadIdx.x & 3), pb);
    } else {
#pragma unroll
      for (int k = 0; k < LB; ++k) {
        const int i = threadIdx.x + 256 * k, r = i / (BP / 4), q = i % (BP / 4);
        pb[k] = (vb + r < v1 && q < BC / 4) ? load_b(vb + r, q) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < LA; ++k) {
      const int i = threadIdx.x + 256 * k, r = i / (AP / 4), q = i % (AP / 4);
      *reinterpret_cast<float4*>(sa + r * SA + 4 * q) = pa[k];
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int r = BROW ? (int)threadIdx.x >> 2 : i / (BP / 4), q = BROW ? 2 * (threadIdx.x & 3) + k : i % (BP / 4);
      *reinterpret_cast<float4*>(sb + r * SB + 4 * q) = pb[k];
    }
  };
  if (v0 < v1) fetch(v0);
#pragma unroll 1
  for (long vb = v0; vb < v1; vb += CH) {
    __syncthreads();
    commit();
    __syncthreads();
    if (vb + CH < v1) fetch(vb + CH);  // lands during this chunk's MFMAs
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = KS > 1 ? wv / KS : wv * TPW + t;
      const int ma = tile / (BP / 16), nb = tile % (BP / 16);
      floatx4_t d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = ks; s < CH / 4; s += KS) {
        const int r = 4 * s + kg;
        d = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[r * SA + 16 * ma + col], sb[r * SB + 16 * nb + col], d, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] += (double)d[r];
    }
  }
  // lane (col, kg) of tile (ma, nb) holds D[16 ma + 4 kg + r][16 nb + col]
  if (KS > 1) {
    __syncthreads();
    if (ks > 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) cmb[(((ks - 1) * NT + wv / KS) * 64 + lane) * 4 + r] = acc[0][r];
    __syncthreads();
    if (ks == 0)
#pragma unroll 1
      for (int k = 1; k < KS; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[0][r] += cmb[(((k - 1) * NT + wv / KS) * 64 + lane) * 4 + r];
  }
  if (ks == 0)
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = KS > 1 ? wv / KS : wv * TPW + t;
      const int ma = tile / (BP / 16), nb = tile % (BP / 16);
      const int b = 16 * nb + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = 16 * ma + 4 * kg + r;
        if (a < A && b < BC) out[a * BC + b] = acc[t][r];
      }
    }
}

}  // namespace tmvs
