// BatchNorm statistics finalize of one channel (bn.hip's stats_finalize_raw_kernel; the fused
// in-launch finalize that shared it was retired in round 5, tools/retired/): raw fp64 sums (sum y,
// sum y^2) over M rows -> mean, biased var, running stats, and the coefficients the consumers
// apply on load, coef = [alpha | shift | mean | invstd] (alpha = gamma invstd, shift = beta -
// mean alpha).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace avc {

__device__ __forceinline__ void bn_finalize_channel(int64_t M, int C, int c, double a, double b,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float eps, float* __restrict__ mean, float* __restrict__ var,
                                                    float* __restrict__ coef, float* __restrict__ run_mean,
                                                    float* __restrict__ run_var, float momentum) {
  const double n = (double)M;
  const double mu = a / n;
  double v = b / n - mu * mu;
  if (v < 0.0) v = 0.0;
  const float muf = (float)mu, vf = (float)v;
  mean[c] = muf;
  var[c] = vf;
  const float invstd = 1.0f / sqrtf(vf + eps);
  const float alpha = invstd * (gamma ? gamma[c] : 1.f);
  coef[c] = alpha;
  coef[C + c] = (beta ? beta[c] : 0.f) - muf * alpha;
  coef[2 * C + c] = muf;
  coef[3 * C + c] = invstd;
  if (run_mean) run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
  if (run_var) run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * v * n / (n > 1.0 ? n - 1.0 : 1.0));
}

}  // namespace avc
