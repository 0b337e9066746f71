// BatchNorm1d (+ ReLU / tanh / identity) for NTC activations, train and eval mode.
//
// Reference: nn.BatchNorm1d(C) after every ConvNorm (model_vc_mel.py:57,100,140,151,160)
// followed by F.relu (encoder/decoder, :69,:115) or torch.tanh (postnet :165) or nothing
// (last postnet layer :167).  Train mode: batch statistics over (B, T) per channel,
// biased variance for normalisation, unbiased for running_var, momentum 0.1, eps 1e-5,
// num_batches_tracked += 1.
//
// Channel statistics are a column reduction of the (M = B*T, C) activation: a partial
// kernel (grid = column tiles x row splits, coalesced 256 B row segments per wave,
// double accumulators about a per-channel shift = row 0) and a finalize kernel that
// sums the partials in a fixed order -> deterministic, no atomics.
#include <algorithm>

#include "common.h"
#include "bn_finalize.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int kRowSplits = 128;

enum Act { kNone = 0, kRelu = 1, kTanh = 2 };

__device__ __forceinline__ float act_fwd(float v, int act) {
  return act == kRelu ? fmaxf(v, 0.f) : (act == kTanh ? tanhf(v) : v);
}

// derivative of the activation expressed through its OUTPUT z
__device__ __forceinline__ float act_grad(float dz, float z, int act) {
  return act == kRelu ? (z > 0.f ? dz : 0.f) : (act == kTanh ? dz * (1.f - z * z) : dz);
}

// ---- statistics: partial[rs][c] = (sum (x - x0), sum (x - x0)^2) ------------------
__global__ __launch_bounds__(256) void stats_partial_kernel(int64_t M, int C, const float* __restrict__ y, int64_t ld,
                                                           double* __restrict__ part) {
  __shared__ double red[4][64][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rs = blockIdx.y, RS = gridDim.y;
  const int64_t r0 = M * rs / RS, r1 = M * (rs + 1) / RS;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const double x0 = y[c];
#pragma unroll 4
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const double d = (double)y[r * ld + c] - x0;
      s1 += d;
      s2 += d * d;
    }
  }
  red[w][lane][0] = s1;
  red[w][lane][1] = s2;
  __syncthreads();
  if (w == 0 && c < C) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < 4; ++q) { a += red[q][lane][0]; b += red[q][lane][1]; }
    part[((int64_t)rs * C + c) * 2 + 0] = a;
    part[((int64_t)rs * C + c) * 2 + 1] = b;
  }
}

// The finalize kernels sum RS partial rows per channel.  Block = 16 row groups x 16
// channels (lanes t & 15 of a group read one 256 B row segment of (s1, s2) pairs as
// double2), each group sums every 16th row, then lanes t < 16 add the 16 group sums in
// group order: fixed order (deterministic), RS/16 loads in flight per thread instead of a
// serial RS/4-long chain, and C/16 blocks instead of C/64.
constexpr int kFinCh = 16;

// returns true on the lanes that own a finished channel sum (threadIdx.x < 16, c < C)
__device__ __forceinline__ bool sum_partials(const double* __restrict__ part, int RS, int C, int c, double& a,
                                             double& b) {
  __shared__ double red[16][kFinCh][2];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
#pragma unroll 4
    for (int rs = g; rs < RS; rs += 16) {
      const double2 v = *reinterpret_cast<const double2*>(part + ((int64_t)rs * C + c) * 2);
      s1 += v.x;
      s2 += v.y;
    }
  red[g][cl][0] = s1;
  red[g][cl][1] = s2;
  __syncthreads();
  a = 0.0;
  b = 0.0;
  if (threadIdx.x >= 16) return false;
  for (int q = 0; q < 16; ++q) {
    a += red[q][cl][0];
    b += red[q][cl][1];
  }
  return c < C;
}

__device__ __forceinline__ int fin_channel() { return blockIdx.x * kFinCh + (threadIdx.x & 15); }

// grid = ceil(C/16), block 256
__global__ __launch_bounds__(256) void stats_finalize_kernel(int64_t M, int C, const float* __restrict__ y,
                                                            const double* __restrict__ part, int RS,
                                                            float* __restrict__ mean, float* __restrict__ var,
                                                            float* __restrict__ run_mean, float* __restrict__ run_var,
                                                            float momentum, int64_t* __restrict__ nbt) {
  const int c = fin_channel();
  double a, b;
  const bool own = sum_partials(part, RS, C, c, a, b);
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (!own) return;
  const double n = (double)M;
  const double mu_s = a / n;
  double v = b / n - mu_s * mu_s;
  if (v < 0.0) v = 0.0;
  const double mu = (double)y[c] + mu_s;
  mean[c] = (float)mu;
  var[c] = (float)v;
  if (run_mean) run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
  if (run_var) run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * v * n / (n > 1.0 ? n - 1.0 : 1.0));
}

// ---- apply: z = act(y * alpha + beta') (+ residual), alpha = gamma/sqrt(var+eps) -------
// 2-D launch: blockIdx.x * 64 + lane = channel, (blockIdx.y, wave) stride the rows, so the
// per-channel coefficients are computed once per thread and no 64-bit divide is needed.
__global__ __launch_bounds__(256) void apply_kernel(int64_t M, int C, const float* __restrict__ y, int64_t ldy,
                                                   const float* __restrict__ mean, const float* __restrict__ var,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float eps, int act, const float* __restrict__ res, int64_t ldr,
                                                   float* __restrict__ z, int64_t ldz) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(var[c] + eps);
  const float alpha = invstd * (gamma ? gamma[c] : 1.f);
  const float b = (beta ? beta[c] : 0.f) - mean[c] * alpha;
  const int64_t rstep = (int64_t)gridDim.y * 4;
#pragma unroll 4
  for (int64_t m = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6); m < M; m += rstep) {
    float v = act_fwd(fmaf(y[m * ldy + c], alpha, b), act);
    if (res) v += res[m * ldr + c];
    z[m * ldz + c] = v;
  }
}

// ---- backward reduce: partial sums of dy_act and dy_act * xhat ----------------------
__global__ __launch_bounds__(256) void bwd_partial_kernel(int64_t M, int C, const float* __restrict__ dz, int64_t lddz,
                                                         const float* __restrict__ z, int64_t ldz,
                                                         const float* __restrict__ y, int64_t ldy,
                                                         const float* __restrict__ mean, int act,
                                                         double* __restrict__ part) {
  __shared__ double red[4][64][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rs = blockIdx.y, RS = gridDim.y;
  const int64_t r0 = M * rs / RS, r1 = M * (rs + 1) / RS;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const float mu = mean[c];
#pragma unroll 4
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const float g = act_grad(dz[r * lddz + c], act == kNone ? 0.f : z[r * ldz + c], act);
      s1 += (double)g;
      s2 += (double)g * (double)(y[r * ldy + c] - mu);
    }
  }
  red[w][lane][0] = s1;
  red[w][lane][1] = s2;
  __syncthreads();
  if (w == 0 && c < C) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < 4; ++q) { a += red[q][lane][0]; b += red[q][lane][1]; }
    part[((int64_t)rs * C + c) * 2 + 0] = a;
    part[((int64_t)rs * C + c) * 2 + 1] = b;
  }
}

// sums -> dbeta = sum dy_act, dgamma = sum dy_act * xhat ; keeps the raw sums for apply
__device__ __forceinline__ void bwd_finalize_body(int blk, int C, const double* __restrict__ part, int RS,
                                                  const float* __restrict__ var, float eps, float* __restrict__ sums,
                                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                  int accumulate) {
  const int c = blk * kFinCh + (threadIdx.x & 15);
  double a, b;
  if (!sum_partials(part, RS, C, c, a, b)) return;
  const float invstd = 1.0f / sqrtf(var[c] + eps);
  const float sdy = (float)a, sdyx = (float)(b * (double)invstd);
  sums[2 * c] = sdy;
  sums[2 * c + 1] = sdyx;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + sdy : sdy;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + sdyx : sdyx;
}

__global__ __launch_bounds__(256) void bwd_finalize_kernel(int C, const double* __restrict__ part, int RS,
                                                          const float* __restrict__ var, float eps,
                                                          float* __restrict__ sums, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta, int accumulate) {
  bwd_finalize_body(blockIdx.x, C, part, RS, var, eps, sums, dgamma, dbeta, accumulate);
}

// dy = (dy_act - sdy/M - xhat * sdyx/M) * invstd * gamma   (2-D launch as apply_kernel)
__global__ __launch_bounds__(256) void bwd_apply_kernel(int64_t M, int C, const float* __restrict__ dz, int64_t lddz,
                                                       const float* __restrict__ z, int64_t ldz,
                                                       const float* __restrict__ y, int64_t ldy,
                                                       const float* __restrict__ mean, const float* __restrict__ var,
                                                       const float* __restrict__ gamma, float eps, int act,
                                                       const float* __restrict__ sums, float* __restrict__ dy,
                                                       int64_t lddy) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (c >= C) return;
  const float inv_m = 1.0f / (float)M;
  const float invstd = 1.0f / sqrtf(var[c] + eps);
  const float mu = mean[c], s0 = sums[2 * c] * inv_m, s1 = sums[2 * c + 1] * inv_m;
  const float gsc = invstd * (gamma ? gamma[c] : 1.f);
  const int64_t rstep = (int64_t)gridDim.y * 4;
#pragma unroll 4
  for (int64_t m = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6); m < M; m += rstep) {
    const float g = act_grad(dz[m * lddz + c], act == kNone ? 0.f : z[m * ldz + c], act);
    const float xhat = (y[m * ldy + c] - mu) * invstd;
    dy[m * lddy + c] = (g - s0 - xhat * s1) * gsc;
  }
}

// ---- fused Conv-BN chain (winograd.hip's wino_output_stats_kernel partials) ----------
// raw fp64 sums (sum y, sum y^2) of RS row blocks -> mean, biased var, running stats, and
// the coefficients the consumers apply on load: coef = [alpha | shift | mean | invstd],
// alpha = gamma invstd, shift = beta - mean alpha (apply_kernel's arithmetic)
__global__ __launch_bounds__(256) void stats_finalize_raw_kernel(int64_t M, int C, const double* __restrict__ part,
                                                                int RS, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps,
                                                                float* __restrict__ mean, float* __restrict__ var,
                                                                float* __restrict__ coef, float* __restrict__ run_mean,
                                                                float* __restrict__ run_var, float momentum,
                                                                int64_t* __restrict__ nbt) {
  const int c = fin_channel();
  double a, b;
  const bool own = sum_partials(part, RS, C, c, a, b);
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (!own) return;
  avc::bn_finalize_channel(M, C, c, a, b, gamma, beta, eps, mean, var, coef, run_mean, run_var, momentum);
}

// eval mode: the same coefficients from the running statistics
__global__ void coef_kernel(int C, const float* __restrict__ mean, const float* __restrict__ var,
                            const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                            float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(var[c] + eps);
  const float alpha = invstd * (gamma ? gamma[c] : 1.f);
  coef[c] = alpha;
  coef[C + c] = (beta ? beta[c] : 0.f) - mean[c] * alpha;
  coef[2 * C + c] = mean[c];
  coef[3 * C + c] = invstd;
}

// column sums of RS fp64 partial rows (the fused conv bias gradient), fixed order
__device__ __forceinline__ void colsum_f64_body(int blk, int C, int RS, const double* __restrict__ part,
                                                float* __restrict__ out, int accumulate) {
  __shared__ double red[16][kFinCh];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blk * kFinCh + cl;
  double s = 0.0;
  if (c < C)
#pragma unroll 8
    for (int rs = g; rs < RS; rs += 16) s += part[(int64_t)rs * C + c];
  red[g][cl] = s;
  __syncthreads();
  if (threadIdx.x >= 16 || c >= C) return;
  double t = 0.0;
  for (int q = 0; q < 16; ++q) t += red[q][cl];
  const float v = (float)t;
  out[c] = accumulate ? out[c] + v : v;
}

__global__ __launch_bounds__(256) void colsum_f64_finalize_kernel(int C, int RS, const double* __restrict__ part,
                                                                 float* __restrict__ out, int accumulate) {
  colsum_f64_body(blockIdx.x, C, RS, part, out, accumulate);
}

// One launch for two independent finalizes of the Conv-BN stack backward: blocks [0, nb_bn)
// finish this layer's BatchNorm-backward sums, the rest the previous (deeper) layer's conv
// bias sums, which no kernel in between reads.
__global__ __launch_bounds__(256) void bwd_finalize_bias_kernel(int C, const double* __restrict__ part, int RS,
                                                               const float* __restrict__ var, float eps,
                                                               float* __restrict__ sums, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, int accumulate, int nb_bn,
                                                               int Cb, int RSb, const double* __restrict__ bpart,
                                                               float* __restrict__ db, int acc_b) {
  if ((int)blockIdx.x < nb_bn) bwd_finalize_body(blockIdx.x, C, part, RS, var, eps, sums, dgamma, dbeta, accumulate);
  else colsum_f64_body(blockIdx.x - nb_bn, Cb, RSb, bpart, db, acc_b);
}

// ---- fused Conv-BN stacks under bf16 (gemm.hip autovc_bnconv_*): the BatchNorm +
// activation backward of one layer and its conv bias sums in one pass:
//   g = act'(pre) dz, pre = alpha y + shift (relu' from pre > 0, tanh' = 1 - avc_tanh_fast(pre)^2
//   as the stack's GEMMs computed it), dy = (g - sums0 / M - xhat sums1 / M) alpha,
//   xhat = (y - mean) invstd (bwd_apply_kernel's arithmetic; coef = [alpha|shift|mean|invstd]),
//   bpart[rs][c] = sum of dy over row block rs (double, fixed order) for the conv bias.
// dy is written as fp32 (dy) and / or as the bf16 copy the stack's GEMMs read (dyh).
// grid (ceil(C/64), RS): 4 waves stride the rows of block rs.
template <int ACT>
__global__ __launch_bounds__(256) void bn_dy_kernel(int64_t M, int C, const float* __restrict__ dz,
                                                   const float* __restrict__ y, const float* __restrict__ coef,
                                                   const float* __restrict__ sums, float* __restrict__ dy,
                                                   __bf16* __restrict__ dyh, double* __restrict__ bpart) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rs = blockIdx.y, RS = gridDim.y;
  const int64_t r0 = M * rs / RS, r1 = M * (rs + 1) / RS;
  double sb = 0.0;
  if (c < C) {
    const float inv_m = 1.0f / (float)M;
    const float a = coef[c], sh = coef[C + c], mu = coef[2 * C + c], invstd = coef[3 * C + c];
    const float s0 = sums[2 * c] * inv_m, s1 = sums[2 * c + 1] * inv_m;
#pragma unroll 4
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const float yv = y[r * C + c], d = dz[r * C + c];
      const float pre = fmaf(yv, a, sh);
      float g = d;
      if (ACT == kRelu) g = pre > 0.f ? d : 0.f;
      else if (ACT == kTanh) { const float z = avc_tanh_fast(pre); g = d * (1.f - z * z); }
      const float xhat = (yv - mu) * invstd;
      const float v = (g - s0 - xhat * s1) * a;
      if (dy) dy[r * C + c] = v;
      if (dyh) dyh[r * C + c] = (__bf16)v;
      sb += (double)v;
    }
  }
  red[w][lane] = sb;
  __syncthreads();
  if (w == 0 && c < C) bpart[(int64_t)rs * C + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// z = bf16(act(y alpha + shift)) — the bf16 copy of a stack layer's output that the next
// layer's bf16 conv GEMMs (forward and weight gradient) read; tanh as the stack's backward
// recomputes it.  4 channels per thread (C % 4 == 0), grid-stride over the (M, C/4) elements.
template <int ACT>
__global__ __launch_bounds__(256) void apply_bf16_kernel(int64_t n4, int C4, const float* __restrict__ y,
                                                        const float* __restrict__ coef, __bf16* __restrict__ z) {
  const int C = 4 * C4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = 4 * (int)(e % C4);
    const float4 v = reinterpret_cast<const float4*>(y)[e];
    const float4 a = *reinterpret_cast<const float4*>(coef + c), sh = *reinterpret_cast<const float4*>(coef + C + c);
    float o[4] = {fmaf(v.x, a.x, sh.x), fmaf(v.y, a.y, sh.y), fmaf(v.z, a.z, sh.z), fmaf(v.w, a.w, sh.w)};
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ACT == kRelu ? fmaxf(o[j], 0.f) : (ACT == kTanh ? avc_tanh_fast(o[j]) : o[j]);
    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
    reinterpret_cast<bf16x4_t*>(z)[e] = bf16x4_t{(__bf16)o[0], (__bf16)o[1], (__bf16)o[2], (__bf16)o[3]};
  }
}

// 2-D grid of the apply kernels: 64-channel column tiles x row groups (~8 rows per thread)
dim3 grid2d(int64_t M, int C) {
  const int64_t ry = std::max<int64_t>(1, std::min<int64_t>((M + 31) / 32, 4096));
  return dim3((C + 63) / 64, (unsigned)ry);
}

}  // namespace

extern "C" int64_t autovc_bn_workspace_bytes(int C) {
  return (int64_t)kRowSplits * C * 2 * sizeof(double) + (int64_t)2 * C * sizeof(float);
}

extern "C" int autovc_bn_stats_f32(int64_t M, int C, const float* y, int64_t ldy, float* mean, float* var,
                                   float* running_mean, float* running_var, float momentum, int64_t* num_batches,
                                   void* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0, "autovc_bn_stats_f32: bad dims");
  AVC_CHECK_ARG(y && mean && var && workspace, "autovc_bn_stats_f32: null pointer");
  double* part = reinterpret_cast<double*>(workspace);
  const int RS = (int)std::min<int64_t>(kRowSplits, M);
  hipLaunchKernelGGL(stats_partial_kernel, dim3((C + 63) / 64, RS), dim3(256), 0, stream, M, C, y, ldy, part);
  hipLaunchKernelGGL(stats_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, stream, M, C, y,
                     (const double*)part, RS, mean, var, running_mean, running_var, momentum, num_batches);
  AVC_CHECK_LAUNCH("autovc_bn_stats_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_act_fwd_f32(int64_t M, int C, const float* y, int64_t ldy, const float* mean,
                                     const float* var, const float* gamma, const float* beta, float eps, int act,
                                     const float* residual, int64_t ldr, float* z, int64_t ldz, hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0 && y && mean && var && z, "autovc_bn_act_fwd_f32: bad args");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_bn_act_fwd_f32: unknown activation %d", act);
  hipLaunchKernelGGL(apply_kernel, grid2d(M, C), dim3(256), 0, stream, M, C, y, ldy, mean, var, gamma,
                     beta, eps, act, residual, ldr, z, ldz);
  AVC_CHECK_LAUNCH("autovc_bn_act_fwd_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_act_bwd_f32(int64_t M, int C, const float* dz, int64_t lddz, const float* z, int64_t ldz,
                                     const float* y, int64_t ldy, const float* mean, const float* var,
                                     const float* gamma, float eps, int act, float* dy, int64_t lddy,
                                     float* dgamma, float* dbeta, int accumulate, void* workspace,
                                     hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0 && dz && y && mean && var && dy && workspace, "autovc_bn_act_bwd_f32: bad args");
  AVC_CHECK_ARG(act == kNone || z, "autovc_bn_act_bwd_f32: activation backward needs the output z");
  double* part = reinterpret_cast<double*>(workspace);
  float* sums = reinterpret_cast<float*>(part + (int64_t)kRowSplits * C * 2);
  const int RS = (int)std::min<int64_t>(kRowSplits, M);
  hipLaunchKernelGGL(bwd_partial_kernel, dim3((C + 63) / 64, RS), dim3(256), 0, stream, M, C, dz, lddz, z, ldz, y,
                     ldy, mean, act, part);
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, stream, C, (const double*)part, RS,
                     var, eps, sums, dgamma, dbeta, accumulate);
  hipLaunchKernelGGL(bwd_apply_kernel, grid2d(M, C), dim3(256), 0, stream, M, C, dz, lddz, z, ldz, y, ldy,
                     mean, var, gamma, eps, act, (const float*)sums, dy, lddy);
  AVC_CHECK_LAUNCH("autovc_bn_act_bwd_f32");
  return avc::kOk;
}

// ------------------------------------------------------------------ fused Conv-BN chain
extern "C" int autovc_bn_finalize_f32(int RS, int64_t M, int C, const double* part, const float* gamma,
                                      const float* beta, float eps, float* mean, float* var, float* coef,
                                      float* running_mean, float* running_var, float momentum, int64_t* num_batches,
                                      hipStream_t stream) {
  AVC_CHECK_ARG(RS > 0 && M > 0 && C > 0 && part && mean && var && coef, "autovc_bn_finalize_f32: bad args");
  hipLaunchKernelGGL(stats_finalize_raw_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, stream, M, C, part, RS, gamma,
                     beta, eps, mean, var, coef, running_mean, running_var, momentum, num_batches);
  AVC_CHECK_LAUNCH("autovc_bn_finalize_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_coef_f32(int C, const float* mean, const float* var, const float* gamma, const float* beta,
                                  float eps, float* coef, hipStream_t stream) {
  AVC_CHECK_ARG(C > 0 && mean && var && coef, "autovc_bn_coef_f32: bad args");
  hipLaunchKernelGGL(coef_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, C, mean, var, gamma, beta, eps, coef);
  AVC_CHECK_LAUNCH("autovc_bn_coef_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_partial_rows(int64_t M) { return (int)std::min<int64_t>(kRowSplits, M); }

extern "C" int autovc_bn_bwd_partial_f32(int64_t M, int C, const float* dz, int64_t lddz, const float* z, int64_t ldz,
                                         const float* y, int64_t ldy, const float* mean, int act, double* part,
                                         hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0 && dz && y && mean && part, "autovc_bn_bwd_partial_f32: bad args");
  AVC_CHECK_ARG(act == kNone || z, "autovc_bn_bwd_partial_f32: activation backward needs the output z");
  hipLaunchKernelGGL(bwd_partial_kernel, dim3((C + 63) / 64, autovc_bn_partial_rows(M)), dim3(256), 0, stream, M, C,
                     dz, lddz, z, ldz, y, ldy, mean, act, part);
  AVC_CHECK_LAUNCH("autovc_bn_bwd_partial_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_bwd_finalize_f32(int RS, int C, const double* part, const float* var, float eps, float* sums,
                                          float* dgamma, float* dbeta, int accumulate, hipStream_t stream) {
  AVC_CHECK_ARG(RS > 0 && C > 0 && part && var && sums, "autovc_bn_bwd_finalize_f32: bad args");
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, stream, C, part, RS, var, eps, sums,
                     dgamma, dbeta, accumulate);
  AVC_CHECK_LAUNCH("autovc_bn_bwd_finalize_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_bwd_finalize_bias_f32(int RS, int C, const double* part, const float* var, float eps,
                                               float* sums, float* dgamma, float* dbeta, int accumulate, int RSb,
                                               int Cb, const double* bias_part, float* db, int acc_b,
                                               hipStream_t stream) {
  AVC_CHECK_ARG(RS > 0 && C > 0 && part && var && sums && RSb > 0 && Cb > 0 && bias_part && db,
                "autovc_bn_bwd_finalize_bias_f32: bad args");
  const int nb = (C + kFinCh - 1) / kFinCh, nbb = (Cb + kFinCh - 1) / kFinCh;
  hipLaunchKernelGGL(bwd_finalize_bias_kernel, dim3(nb + nbb), dim3(256), 0, stream, C, part, RS, var, eps, sums,
                     dgamma, dbeta, accumulate, nb, Cb, RSb, bias_part, db, acc_b);
  AVC_CHECK_LAUNCH("autovc_bn_bwd_finalize_bias_f32");
  return avc::kOk;
}

extern "C" int autovc_colsum_f64_finalize_f32(int RS, int C, const double* part, float* out, int accumulate,
                                              hipStream_t stream) {
  AVC_CHECK_ARG(RS > 0 && C > 0 && part && out, "autovc_colsum_f64_finalize_f32: bad args");
  hipLaunchKernelGGL(colsum_f64_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, stream, C, RS, part, out,
                     accumulate);
  AVC_CHECK_LAUNCH("autovc_colsum_f64_finalize_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_dy_f32(int64_t M, int C, const float* dz, const float* y, const float* coef, int act,
                                const float* sums, float* dy, void* dy_bf16, double* bias_part, hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0 && dz && y && coef && sums && (dy || dy_bf16) && bias_part, "autovc_bn_dy_f32: bad args");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_bn_dy_f32: unknown activation %d", act);
  const dim3 grid((C + 63) / 64, autovc_bn_partial_rows(M));
  __bf16* dyh = static_cast<__bf16*>(dy_bf16);
  if (act == kRelu) hipLaunchKernelGGL(bn_dy_kernel<kRelu>, grid, dim3(256), 0, stream, M, C, dz, y, coef, sums, dy, dyh, bias_part);
  else if (act == kTanh) hipLaunchKernelGGL(bn_dy_kernel<kTanh>, grid, dim3(256), 0, stream, M, C, dz, y, coef, sums, dy, dyh, bias_part);
  else hipLaunchKernelGGL(bn_dy_kernel<kNone>, grid, dim3(256), 0, stream, M, C, dz, y, coef, sums, dy, dyh, bias_part);
  AVC_CHECK_LAUNCH("autovc_bn_dy_f32");
  return avc::kOk;
}

extern "C" int autovc_bn_apply_bf16(int64_t M, int C, const float* y, const float* coef, int act, void* z,
                                    hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && y && coef && z && AVC_ALIGNED16(y) && AVC_ALIGNED16(coef),
                "autovc_bn_apply_bf16: bad args");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_bn_apply_bf16: unknown activation %d", act);
  const int64_t n4 = M * (C / 4);
  const dim3 grid((unsigned)std::min<int64_t>((n4 + 255) / 256, 2048));
  __bf16* zh = static_cast<__bf16*>(z);
  if (act == kRelu) hipLaunchKernelGGL(apply_bf16_kernel<kRelu>, grid, dim3(256), 0, stream, n4, C / 4, y, coef, zh);
  else if (act == kTanh) hipLaunchKernelGGL(apply_bf16_kernel<kTanh>, grid, dim3(256), 0, stream, n4, C / 4, y, coef, zh);
  else hipLaunchKernelGGL(apply_bf16_kernel<kNone>, grid, dim3(256), 0, stream, n4, C / 4, y, coef, zh);
  AVC_CHECK_LAUNCH("autovc_bn_apply_bf16");
  return avc::kOk;
}
