// Depth-map fusion: the fusibile kernel of gipuma (gipuma/fusibile/fusibile.cu:89-173; SURVEY.md 8f
// rank 4, the output side). For every pixel of the reference camera whose depth exceeds 425.001,
// back-project to 3D, project into every other camera (in camera order, stopping once 2 x
// consistent_threshold views agree), sample that camera's (B, G, R, depth) image, and accept the
// view when the two depths agree as disparities (|f b / d - f b / d'| < depth_threshold). With at
// least consistent_threshold agreeing views the averaged 3D point and colour are written; other
// pixels keep the buffer's previous contents (the reference reuses one point buffer across cameras).
//
// Arithmetic follows the reference's float formulas with the FMA contractions nvcc applies by
// default (-fmad=true) written out as fmaf. Texture fetches (main.cpp:30-66: cudaFilterModeLinear,
// unnormalised coordinates -> CUDA clamps whatever address mode is requested) are done in software
// as CUDA documents linear filtering: texel centres at i + 0.5, weights with 8 fractional bits.
//
// One thread per pixel, 256-thread blocks of 64 x 4 pixels: a wave covers 64 consecutive pixels
// of one row, so the reference-view load is one coalesced 1 KB float4 row and the projected
// gathers of neighbouring lanes land on neighbouring texels.
#include "common.h"

namespace tmvs {

namespace fz {
constexpr int CAM = 32;  // floats per packed camera: P[12], RK_inv[9], C4[3], fx, pad
constexpr float kDepthFloor = 425.001f;
}  // namespace fz

__device__ __forceinline__ float4 fz_load(const float4* __restrict__ img, int W, int x, int y) {
  return img[(size_t)y * W + x];
}

// tex2D<float4>(tex, x, y), cudaFilterModeLinear, unnormalised coordinates, clamp addressing
__device__ __forceinline__ float4 fz_tex_linear(const float4* __restrict__ img, int H, int W, float x, float y) {
  const float xb = x - 0.5f, yb = y - 0.5f;
  const float fi = floorf(xb), fj = floorf(yb);
  const float a = rintf((xb - fi) * 256.f) * (1.f / 256.f), b = rintf((yb - fj) * 256.f) * (1.f / 256.f);
  const int i0 = (int)fi, j0 = (int)fj;
  const int ic0 = min(max(i0, 0), W - 1), ic1 = min(max(i0 + 1, 0), W - 1);
  const int jc0 = min(max(j0, 0), H - 1), jc1 = min(max(j0 + 1, 0), H - 1);
  const float4 t00 = fz_load(img, W, ic0, jc0), t10 = fz_load(img, W, ic1, jc0);
  const float4 t01 = fz_load(img, W, ic0, jc1), t11 = fz_load(img, W, ic1, jc1);
  const float w00 = (1.f - a) * (1.f - b), w10 = a * (1.f - b), w01 = (1.f - a) * b, w11 = a * b;
  float4 r;
  r.x = fmaf(w11, t11.x, fmaf(w01, t01.x, fmaf(w10, t10.x, w00 * t00.x)));
  r.y = fmaf(w11, t11.y, fmaf(w01, t01.y, fmaf(w10, t10.y, w00 * t00.y)));
  r.z = fmaf(w11, t11.z, fmaf(w01, t01.z, fmaf(w10, t10.z, w00 * t00.z)));
  r.w = fmaf(w11, t11.w, fmaf(w01, t01.w, fmaf(w10, t10.w, w00 * t00.w)));
  return r;
}

// get_3dpoint_cu (fusibile.cu:54-68)
__device__ __forceinline__ void fz_3dpoint(const float* __restrict__ cam, float px, float py, float d, float* X) {
  const float* P = cam;
  const float* M = cam + 12;
  const float vx = fmaf(d, px, -P[3]), vy = fmaf(d, py, -P[7]), vz = d - P[11];
  X[0] = fmaf(M[2], vz, fmaf(M[1], vy, M[0] * vx));
  X[1] = fmaf(M[5], vz, fmaf(M[4], vy, M[3] * vx));
  X[2] = fmaf(M[8], vz, fmaf(M[7], vy, M[6] * vx));
}

__global__ __launch_bounds__(256) void fusibile_kernel(const float4* __restrict__ rgbd, const float* __restrict__ cams,
                                                       int V, int H, int W, int ref, int consistent_threshold,
                                                       float depth_threshold, float4* __restrict__ coord,
                                                       float4* __restrict__ tex) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= W || y >= H) return;
  const size_t HW = (size_t)H * W;
  float4 sum_t = rgbd[ref * HW + (size_t)y * W + x];
  if (!(sum_t.w > fz::kDepthFloor)) return;  // fusibile.cu:116 (depth <= 425.001 -> return)
  const float* cr = cams + ref * fz::CAM;
  float X[3];
  fz_3dpoint(cr, (float)x, (float)y, sum_t.w, X);
  float sx = X[0], sy = X[1], sz = X[2];
  const float f = cr[24];
  int count = 0;
  for (int i = 0; i < V && count < 2 * consistent_threshold; ++i) {
    if (i == ref) continue;
    const float* ci = cams + i * fz::CAM;
    const float* P = ci;
    const float tx = fmaf(P[2], X[2], fmaf(P[1], X[1], P[0] * X[0])) + P[3];
    const float ty = fmaf(P[6], X[2], fmaf(P[5], X[1], P[4] * X[0])) + P[7];
    const float tz = fmaf(P[10], X[2], fmaf(P[9], X[1], P[8] * X[0])) + P[11];
    const float ptx = tx / tz, pty = ty / tz, depth = tz;
    if (!(ptx >= 0.f && ptx < (float)W && pty >= 0.f && pty < (float)H)) continue;  // also rejects NaN
    const float4 t = fz_tex_linear(rgbd + i * HW, H, W, ptx + 0.5f, pty + 0.5f);
    if (!(t.w > fz::kDepthFloor)) continue;
    const float bx = cr[21] - ci[21], by = cr[22] - ci[22], bz = cr[23] - ci[23];
    const float base = sqrtf(fmaf(bz, bz, fmaf(by, by, bx * bx)));
    const float ddisp = (f * base) / depth, tdisp = (f * base) / t.w;
    if (fabsf(ddisp - tdisp) < depth_threshold) {
      float Xi[3];
      fz_3dpoint(ci, (float)(int)ptx, (float)(int)pty, t.w, Xi);
      sx = sx + Xi[0];
      sy = sy + Xi[1];
      sz = sz + Xi[2];
      sum_t.x = sum_t.x + t.x;
      sum_t.y = sum_t.y + t.y;
      sum_t.z = sum_t.z + t.z;
      ++count;
    }
  }
  if (count >= consistent_threshold) {
    const float n = (float)count + 1.f;
    const size_t o = (size_t)y * W + x;
    coord[o] = make_float4(sx / n, sy / n, sz / n, 0.f);           // operator/ zeroes .w
    tex[o] = make_float4(sum_t.x / n, sum_t.y / n, sum_t.z / n, 0.f);
  }
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_fusibile(const float* rgbd, const float* cams, int n_views, int height, int width, int ref_view,
                             int consistent_threshold, float depth_threshold, float* coord, float* texture,
                             void* stream) {
  if (!rgbd || !cams || !coord || !texture || n_views <= 0 || height <= 0 || width <= 0) return TMVS_ERR_ARG;
  if (ref_view < 0 || ref_view >= n_views || consistent_threshold < 0) return TMVS_ERR_ARG;
  const dim3 grid((width + 63) / 64, (height + 3) / 4);
  hipLaunchKernelGGL(fusibile_kernel, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<const float4*>(rgbd),
                     cams, n_views, height, width, ref_view, consistent_threshold, depth_threshold,
                     reinterpret_cast<float4*>(coord), reinterpret_cast<float4*>(texture));
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
