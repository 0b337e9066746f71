// BatchNorm statistics finalize of one channel, shared by bn.hip's stats_finalize_raw_kernel
// and the fused finalize at the end of winograd.hip's output transform: raw fp64 sums (sum y,
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

// 16 bytes (two doubles) written through to memory / read from it (sc1): hand-offs between
// workgroups of one launch that may sit on different XCDs
__device__ __forceinline__ void st_f64x2_sc1(double* base, int64_t idx, double x, double y) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 w = {(unsigned)__double_as_longlong(x), (unsigned)((unsigned long long)__double_as_longlong(x) >> 32),
                   (unsigned)__double_as_longlong(y), (unsigned)((unsigned long long)__double_as_longlong(y) >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (uint32_t)(idx * 8), 0, 16);
}
__device__ __forceinline__ double2 ld_f64x2_sc1(const double* base, int64_t idx) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, 0x7fffffff,
                                                                     0x00020000);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(idx * 8), 0, 16));
  return make_double2(__longlong_as_double((long long)(((unsigned long long)w[1] << 32) | w[0])),
                      __longlong_as_double((long long)(((unsigned long long)w[3] << 32) | w[2])));
}

// what the fused statistics finalize writes (autovc_bn_finalize_f32's outputs)
struct BnFin {
  const float* gamma;
  const float* beta;
  float eps;
  float* mean;
  float* var;
  float* coef;
  float* run_mean;
  float* run_var;
  float momentum;
  int64_t* nbt;
  int64_t M;
};

constexpr int kBnTickets = 1024;              // ints: 16 per column block, then 1 per column block

// Completion of the BatchNorm statistics inside the launch that produced them.  Called by every
// block of a (column block cb: channels c0 .. c0 + CB - 1) x (row block rs of RS) grid AFTER its
// partial row part[rs][c][2] is written through (sc1) and its stores are complete.  The block
// that completes row group g = rs mod 16 sums that group's rows in row order into gpart[g]; the
// block that completes the column block's groups adds them in group order (bn.hip
// sum_partials' order: bit-identical to stats_finalize_raw_kernel) and finishes the channels.
// Threads < CB each own one channel.  At most 16 arrivals per counter.
__device__ __forceinline__ void bn_stats_complete(int* __restrict__ tk, const double* __restrict__ part,
                                                  double* __restrict__ gpart, int C, int c0, int CB, int rs, int RS,
                                                  int cb, const BnFin& f) {
  __shared__ int s_last;
  const int g = rs & 15, ng = RS < 16 ? RS : 16;
  if (threadIdx.x == 0) {
    const int n_in = (RS - g + 15) / 16;
    int* t1 = tk + cb * 16 + g;
    const int old = __hip_atomic_fetch_add(t1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == n_in - 1;
    if (s_last) __hip_atomic_store(t1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  const int ch = c0 + (int)threadIdx.x;
  const bool own = (int)threadIdx.x < CB && ch < C;
  if (own) {
    double a = 0.0, b = 0.0;
    for (int q = g; q < RS; q += 16) {
      const double2 v = ld_f64x2_sc1(part, ((int64_t)q * C + ch) * 2);
      a += v.x;
      b += v.y;
    }
    st_f64x2_sc1(gpart, ((int64_t)g * C + ch) * 2, a, b);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* t2 = tk + kBnTickets / 2 + cb;
    const int old = __hip_atomic_fetch_add(t2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == ng - 1;
    if (s_last) __hip_atomic_store(t2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  if (cb == 0 && threadIdx.x == 0 && f.nbt) *f.nbt += 1;
  if (own) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < 16; ++q) {             // groups without rows add 0.0, as sum_partials does
      double2 v = make_double2(0.0, 0.0);
      if (q < ng) v = ld_f64x2_sc1(gpart, ((int64_t)q * C + ch) * 2);
      a += v.x;
      b += v.y;
    }
    bn_finalize_channel(f.M, C, ch, a, b, f.gamma, f.beta, f.eps, f.mean, f.var, f.coef, f.run_mean, f.run_var,
                        f.momentum);
  }
}

}  // namespace avc
