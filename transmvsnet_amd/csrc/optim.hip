// Adam for the training path (config C5: finetune.py:324, torch.optim.Adam(lr, betas=(0.9, 0.999),
// weight_decay=wd), L2 weight decay, no amsgrad), over one flat fp32 parameter buffer: every
// parameter of the model is a view of it (transmvsnet_amd.train.FlatAdam), so a step is one launch.
// Per element, in torch's single-tensor order (torch/optim/adam.py _single_tensor_adam):
//   g = grad + wd * p;  m = lerp(m, g, 1 - b1);  v = b2 * v + (1 - b2) * g * g
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound: 4 streams read (p, g, m, v), 3 written (p, m, v): 28 B per parameter.
#include "common.h"

namespace tmvs {

// The scalars arrive as the fp32 values torch's scalar arguments become: the complements 1 - beta are
// formed in double from the double betas (as Python does) and only then rounded to fp32.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n, float omb1,
                                                   float beta2, float omb2, float eps, float wd, float step_size,
                                                   float bc2_sqrt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float pv = p[i];
  const float gr = wd != 0.f ? fmaf(wd, pv, g[i]) : g[i];
  const float mv = m[i];
  const float mn = fmaf(omb1, gr - mv, mv);  // torch.lerp (weight < 0.5): start + weight * (end - start)
  const float vn = fmaf(omb2, gr * gr, beta2 * v[i]);
  const float denom = sqrtf(vn) / bc2_sqrt + eps;
  m[i] = mn;
  v[i] = vn;
  p[i] = fmaf(-step_size, mn / denom, pv);
}

}  // namespace tmvs

using namespace tmvs;

extern "C" int tmvs_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, double lr,
                              double beta1, double beta2, double eps, double weight_decay, int step, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || n <= 0 || step <= 0) return TMVS_ERR_ARG;
  const double bc1 = 1.0 - pow(beta1, (double)step), bc2 = 1.0 - pow(beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, param, grad,
                     exp_avg, exp_avg_sq, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     (float)weight_decay, (float)(lr / bc1), (float)sqrt(bc2));
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}

// The same step with the step counter on the device (HIP-graph replays): a one-thread kernel advances
// *step and writes lr / (1 - beta1^step) and sqrt(1 - beta2^step) (double, as the host form) into
// scal[0..1], which adam_kernel_dev reads. lr_dev (ABI 8): when non-null the learning rate is read from
// that device double at run time, so a replayed graph follows the caller's schedule (finetune.py:58-72
// steps WarmupMultiStepLR every iteration) instead of the lr in effect at capture.
__global__ void adam_prep_kernel(int* __restrict__ step, float* __restrict__ scal, double lr,
                                 const double* __restrict__ lr_dev, double beta1, double beta2) {
  const int s = ++step[0];
  if (lr_dev) lr = lr_dev[0];
  scal[0] = (float)(lr / (1.0 - pow(beta1, (double)s)));
  scal[1] = (float)sqrt(1.0 - pow(beta2, (double)s));
}

__global__ __launch_bounds__(256) void adam_kernel_dev(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, long n, float omb1,
                                                       float beta2, float omb2, float eps, float wd,
                                                       const float* __restrict__ scal) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float step_size = scal[0], bc2_sqrt = scal[1];
  const float pv = p[i];
  const float gr = wd != 0.f ? fmaf(wd, pv, g[i]) : g[i];
  const float mv = m[i];
  const float mn = fmaf(omb1, gr - mv, mv);
  const float vn = fmaf(omb2, gr * gr, beta2 * v[i]);
  const float denom = sqrtf(vn) / bc2_sqrt + eps;
  m[i] = mn;
  v[i] = vn;
  p[i] = fmaf(-step_size, mn / denom, pv);
}

extern "C" int tmvs_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n,
                                  double lr, const double* lr_dev, double beta1, double beta2, double eps,
                                  double weight_decay, int* step_counter, float* scalars, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step_counter || !scalars || n <= 0) return TMVS_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, st, step_counter, scalars, lr, lr_dev, beta1, beta2);
  TMVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(adam_kernel_dev, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, param, grad, exp_avg,
                     exp_avg_sq, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     (float)weight_decay, (const float*)scalars);
  TMVS_CHECK_LAUNCH();
  return TMVS_OK;
}
