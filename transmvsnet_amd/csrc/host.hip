// Host-side helpers of the C-ABI (no device code).
#include <cmath>

#include "common.h"

extern "C" int tmvs_abi_version(void) { return TMVS_ABI_VERSION; }

extern "C" const char* tmvs_status_string(int status) {
  switch (status) {
    case TMVS_OK:
      return "ok";
    case TMVS_ERR_ARG:
      return "bad argument";
    case TMVS_ERR_SHAPE:
      return "unsupported shape";
    case TMVS_ERR_HIP:
      return "HIP launch error";
    default:
      return "unknown status";
  }
}

// batch_norm_cpu_collect_linear_and_constant_terms semantics (fp32, fused multiply-add)
extern "C" int tmvs_bn_fold(const float* gamma, const float* beta, const float* mean, const float* var, int n,
                            float eps, float* alpha, float* shift) {
  if (!gamma || !beta || !mean || !var || !alpha || !shift || n <= 0) return TMVS_ERR_ARG;
  for (int c = 0; c < n; ++c) {
    const float invstd = 1.0f / std::sqrt(var[c] + eps);
    alpha[c] = invstd * gamma[c];
    shift[c] = std::fmaf(-mean[c], alpha[c], beta[c]);
  }
  return TMVS_OK;
}
