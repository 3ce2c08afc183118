// Training-side losses: entropy_loss / trans_mvsnet_loss / focal_loss_bld
// (models/module.py:495-592) over one stage's probability volume, fused with the backward of
// the cross-entropy through the stage's softmax, so the first backward step of training -- the
// gradient of the total loss w.r.t. CostRegNet's logits -- comes out of the same pass.
//
// Per pixel (one thread, walking D): the ground-truth hypothesis index (first argmin of
// |depth_value - gt|, module.py:508; 0 where the mask is off, :510-511), the winner-take-all
// index (first argmax of prob, :524-525), CE = -log(prob[gt] + 1e-6) (:517), the smooth-L1 term
// of trans_mvsnet_loss's depth_loss (:545) and, with grad_logits, the softmax backward of
// L = scale * mean_b(sum_pix m * CE / valid_b):
//   dL/dlogit_d = scale / (B * valid_b) * m * p_gt / (p_gt + 1e-6) * (p_d - [d == gt]).
// Sums are per-block fp32 partials, combined in a fixed order in fp64 by one finalize block
// (deterministic); the per-batch valid-pixel counts are integer atomics (order-free).
#include "common.h"

namespace tmvs {

constexpr int kLossBlock = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wv = threadIdx.x >> 6;
  __syncthreads();  // red reuse
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < kLossBlock / 64; ++k) t += red[k];
  return t;  // valid in thread 0
}

__global__ __launch_bounds__(kLossBlock) void mask_count_kernel(const float* __restrict__ mask, int HW,
                                                                int* __restrict__ counts) {
  __shared__ float red[kLossBlock / 64];
  const int b = blockIdx.y;
  float c = 0.f;
  for (int p = blockIdx.x * kLossBlock + threadIdx.x; p < HW; p += gridDim.x * kLossBlock)
    c += mask[(size_t)b * HW + p] > 0.5f ? 1.f : 0.f;
  const float t = block_sum(c, red);  // <= 2^24 per block: exact
  if (threadIdx.x == 0 && t > 0.f) atomicAdd(counts + b, (int)t);
}

__global__ __launch_bounds__(kLossBlock) void entropy_loss_kernel(
    const float* __restrict__ prob, const float* __restrict__ dv, int dv_per_pixel, const float* __restrict__ gt,
    const float* __restrict__ mask, int D, int HW, const int* __restrict__ counts, float grad_scale, int batch,
    float* __restrict__ wta, float* __restrict__ conf, float* __restrict__ grad, float* __restrict__ partial) {
  __shared__ float red[kLossBlock / 64];
  const int b = blockIdx.y;
  const int p = blockIdx.x * kLossBlock + threadIdx.x;
  float ce = 0.f, sl1 = 0.f;
  if (p < HW) {
    const size_t base = (size_t)b * D * HW + p;
    const float* pv = prob + base;
    const float* hv = dv_per_pixel ? dv + base : dv + (size_t)b * D;
    const size_t hs = dv_per_pixel ? (size_t)HW : 1;
    const float g = gt[(size_t)b * HW + p];
    const bool m = mask[(size_t)b * HW + p] > 0.5f;
    float dbest = fabsf(hv[0] - g), pbest = pv[0];
    int gi = 0, wi = 0;
    for (int d = 1; d < D; ++d) {
      const float e = fabsf(hv[(size_t)d * hs] - g);
      const float pd = pv[(size_t)d * HW];
      if (e < dbest) {  // strict: first minimum, as torch.argmin
        dbest = e;
        gi = d;
      }
      if (pd > pbest) {  // first maximum, as torch.argmax
        pbest = pd;
        wi = d;
      }
    }
    if (!m) gi = 0;
    const float pg = pv[(size_t)gi * HW];
    const float wd = hv[(size_t)wi * hs];
    if (wta) wta[(size_t)b * HW + p] = wd;
    if (conf) conf[(size_t)b * HW + p] = pbest;
    if (m) {
      ce = -logf(pg + 1e-6f);
      const float x = fabsf(wd - g);
      sl1 = x < 1.f ? 0.5f * x * x : x - 0.5f;
    }
    if (grad) {
      float* gv = grad + base;
      if (m) {
        const float valid = (float)counts[b] + 1e-6f;
        const float k = grad_scale / ((float)batch * valid) * (pg / (pg + 1e-6f));
        for (int d = 0; d < D; ++d) gv[(size_t)d * HW] = k * (pv[(size_t)d * HW] - (d == gi ? 1.f : 0.f));
      } else {
        for (int d = 0; d < D; ++d) gv[(size_t)d * HW] = 0.f;
      }
    }
  }
  const float s_ce = block_sum(ce, red);
  const float s_sl1 = block_sum(sl1, red);
  if (threadIdx.x == 0) {
    float* o = partial + ((size_t)b * gridDim.x + blockIdx.x) * 2;
    o[0] = s_ce;
    o[1] = s_sl1;
  }
}

// out[0] = mean_b(ce_b / (valid_b + 1e-6)) (module.py:520-522); out[1] = sum sl1 / sum valid
// (smooth_l1_loss over the masked pixels of all batches, :545; NaN for an empty mask, as torch)
__global__ __launch_bounds__(kLossBlock) void entropy_finalize_kernel(const float* __restrict__ partial, int nblk,
                                                                      int batch, const int* __restrict__ counts,
                                                                      float* __restrict__ out) {
  __shared__ double red[2][kLossBlock];
  float loss = 0.f;
  double sl1_all = 0.0;
  long cnt_all = 0;
  for (int b = 0; b < batch; ++b) {
    double a = 0.0, c = 0.0;
    for (int k = threadIdx.x; k < nblk; k += kLossBlock) {
      a += partial[((size_t)b * nblk + k) * 2];
      c += partial[((size_t)b * nblk + k) * 2 + 1];
    }
    red[0][threadIdx.x] = a;
    red[1][threadIdx.x] = c;
    __syncthreads();
    for (int s = kLossBlock / 2; s > 0; s >>= 1) {
      if (threadIdx.x < s) {
        red[0][threadIdx.x] += red[0][threadIdx.x + s];
        red[1][threadIdx.x] += red[1][threadIdx.x + s];
      }
      __syncthreads();
    }
    const float valid = (float)counts[b] + 1e-6f;
    loss += (float)red[0][0] / valid;
    sl1_all += red[1][0];
    cnt_all += counts[b];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = loss / (float)batch;
    out[1] = (float)(sl1_all / (double)cnt_all);  // 0/0 = NaN
  }
}

// focal_loss_bld's stage-3 metrics (module.py:581-587): |gt - depth| / (interval * 192 / 128) over
// the masked pixels: out = {epe (mean), less1, less3 (fractions)}
__global__ __launch_bounds__(kLossBlock) void depth_metrics_kernel(const float* __restrict__ depth,
                                                                   const float* __restrict__ gt,
                                                                   const float* __restrict__ mask, int n, float scale,
                                                                   float* __restrict__ partial) {
  __shared__ float red[kLossBlock / 64];
  float e = 0.f, l1 = 0.f, l3 = 0.f, c = 0.f;
  for (int i = blockIdx.x * kLossBlock + threadIdx.x; i < n; i += gridDim.x * kLossBlock) {
    if (mask[i] > 0.5f) {
      const float x = fabsf(gt[i] - depth[i]) / scale;
      e += x;
      l1 += x < 1.f ? 1.f : 0.f;
      l3 += x < 3.f ? 1.f : 0.f;
      c += 1.f;
    }
  }
  const float se = block_sum(e, red), s1 = block_sum(l1, red), s3 = block_sum(l3, red), sc = block_sum(c, red);
  if (threadIdx.x == 0) {
    float* o = partial + (size_t)blockIdx.x * 4;
    o[0] = se;
    o[1] = s1;
    o[2] = s3;
    o[3] = sc;
  }
}

__global__ __launch_bounds__(kLossBlock) void depth_metrics_finalize_kernel(const float* __restrict__ partial,
                                                                            int nblk, float* __restrict__ out) {
  __shared__ double red[4][kLossBlock];
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  for (int k = threadIdx.x; k < nblk; k += kLossBlock)
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] += partial[(size_t)k * 4 + j];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[j][threadIdx.x] = a[j];
  __syncthreads();
  for (int s = kLossBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double c = red[3][0];
    out[0] = (float)(red[0][0] / c);
    out[1] = (float)(red[1][0] / c);
    out[2] = (float)(red[2][0] / c);
  }
}

constexpr int kMetricsBlocks = 1024;

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
static int loss_nblk(int HW) { return (HW + kLossBlock - 1) / kLossBlock; }

}  // namespace tmvs

using namespace tmvs;

extern "C" size_t tmvs_entropy_loss_workspace(int batch, int height, int width) {
  if (batch <= 0 || height <= 0 || width <= 0) return 0;
  return align256((size_t)batch * sizeof(int)) + (size_t)batch * loss_nblk(height * width) * 2 * sizeof(float);
}

extern "C" int tmvs_entropy_loss(const float* prob, const float* depth_values, int dv_per_pixel, const float* depth_gt,
                                 const float* mask, int batch, int ndepth, int height, int width, float grad_scale,
                                 void* workspace, size_t workspace_bytes, float* out, float* wta_depth,
                                 float* photo_conf, float* grad_logits, void* stream) {
  if (!prob || !depth_values || !depth_gt || !mask || !workspace || !out) return TMVS_ERR_ARG;
  if (batch <= 0 || ndepth <= 0 || height <= 0 || width <= 0) return TMVS_ERR_SHAPE;
  if ((long)height * width >= (1L << 31) / kLossBlock) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_entropy_loss_workspace(batch, height, width)) return TMVS_ERR_ARG;
  const int HW = height * width, nblk = loss_nblk(HW);
  hipStream_t st = (hipStream_t)stream;
  int* counts = (int*)workspace;
  float* partial = (float*)((char*)workspace + align256((size_t)batch * sizeof(int)));
  if (hipMemsetAsync(counts, 0, (size_t)batch * sizeof(int), st) != hipSuccess) return TMVS_ERR_HIP;
  hipLaunchKernelGGL(mask_count_kernel, dim3(nblk < 512 ? nblk : 512, batch), dim3(kLossBlock), 0, st, mask, HW,
                     counts);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(entropy_loss_kernel, dim3(nblk, batch), dim3(kLossBlock), 0, st, prob, depth_values,
                     dv_per_pixel, depth_gt, mask, ndepth, HW, (const int*)counts, grad_scale, batch, wta_depth,
                     photo_conf, grad_logits, partial);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(entropy_finalize_kernel, dim3(1), dim3(kLossBlock), 0, st, (const float*)partial, nblk, batch,
                     (const int*)counts, out);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

extern "C" size_t tmvs_depth_metrics_workspace(int n) {
  (void)n;
  return (size_t)kMetricsBlocks * 4 * sizeof(float);
}

extern "C" int tmvs_depth_metrics(const float* depth, const float* depth_gt, const float* mask, int n,
                                  float depth_interval, void* workspace, size_t workspace_bytes, float* out,
                                  void* stream) {
  if (!depth || !depth_gt || !mask || !workspace || !out) return TMVS_ERR_ARG;
  if (n <= 0) return TMVS_ERR_SHAPE;
  if (workspace_bytes < tmvs_depth_metrics_workspace(n)) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int nblk0 = (n + kLossBlock - 1) / kLossBlock;
  const int nblk = nblk0 < kMetricsBlocks ? nblk0 : kMetricsBlocks;
  const float scale = depth_interval * 192.f / 128.f;  // module.py:582, left to right in fp32
  hipLaunchKernelGGL(depth_metrics_kernel, dim3(nblk), dim3(kLossBlock), 0, st, depth, depth_gt, mask, n, scale,
                     (float*)workspace);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(depth_metrics_finalize_kernel, dim3(1), dim3(kLossBlock), 0, st, (const float*)workspace, nblk,
                     out);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
