// Winograd F(4,5) for AutoVC's ConvNorm (Conv1d k=5, pad=2; model_vc_mel.py:20-38) on gfx950.
//
// Per sequence of T frames (T % 4 == 0) the output is cut into tiles of 4 frames; tile q
// reads the 8 input frames 4q-2 .. 4q+5 (zero outside the sequence: the reference's
// padding).  With interpolation points {0, ±1, ±2, ±1/2, ∞} (Toom-Cook, exact matrices
// below; fp32 error ~1e-6 relative vs ~2e-7 for the direct sum, tests at 1e-4):
//   X~[i][tile][c] = sum_j BT[i][j] x[4q-2+j][c]                 (input transform)
//   W~[i][co][ci]  = sum_k G[i][k]  W[co][ci][k]                 (weight transform)
//   Y~[i]          = X~[i] W~[i]^T          8 GEMMs, one batched launch (autovc_gemm_batched_f32)
//   y[4q+o][co]    = sum_i AT[o][i] Y~[i][tile][co] + b[co]      (output transform)
// 8/(4·5) = 0.4 of the im2col GEMM's multiply-adds; the input gradient of the same conv is
// the same correlation of dy with the flipped, transposed kernel (W~ built with flip).
#include <algorithm>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr float kBT[8][8] = {
    {-1.f, 0.f, 5.25f, 0.f, -5.25f, 0.f, 1.f, 0.f},
    {0.f, 1.f, 1.f, -4.25f, -4.25f, 1.f, 1.f, 0.f},
    {0.f, -1.f, 1.f, 4.25f, -4.25f, -1.f, 1.f, 0.f},
    {0.f, 0.5f, 0.25f, -2.5f, -1.25f, 2.f, 1.f, 0.f},
    {0.f, -0.5f, 0.25f, 2.5f, -1.25f, -2.f, 1.f, 0.f},
    {0.f, 2.f, 4.f, -2.5f, -5.f, 0.5f, 1.f, 0.f},
    {0.f, -2.f, 4.f, 2.5f, -5.f, -0.5f, 1.f, 0.f},
    {0.f, -1.f, 0.f, 5.25f, 0.f, -5.25f, 0.f, 1.f}};

constexpr float kAT[4][8] = {
    {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
    {0.f, 1.f, -1.f, 2.f, -2.f, 0.5f, -0.5f, 0.f},
    {0.f, 1.f, 1.f, 4.f, 4.f, 0.25f, 0.25f, 0.f},
    {0.f, 1.f, -1.f, 8.f, -8.f, 0.125f, -0.125f, 1.f}};

// G in double (2/9, 1/90, ... are not binary fractions): the weight transform runs once per
// call over 8·Co·Ci outputs and rounds once.
__constant__ double kG[8][5] = {
    {-1.0, 0.0, 0.0, 0.0, 0.0},
    {-2.0 / 9, -2.0 / 9, -2.0 / 9, -2.0 / 9, -2.0 / 9},
    {-2.0 / 9, 2.0 / 9, -2.0 / 9, 2.0 / 9, -2.0 / 9},
    {1.0 / 90, 2.0 / 90, 4.0 / 90, 8.0 / 90, 16.0 / 90},
    {1.0 / 90, -2.0 / 90, 4.0 / 90, -8.0 / 90, 16.0 / 90},
    {32.0 / 45, 16.0 / 45, 8.0 / 45, 4.0 / 45, 2.0 / 45},
    {32.0 / 45, -16.0 / 45, 8.0 / 45, -4.0 / 45, 2.0 / 45},
    {0.0, 0.0, 0.0, 0.0, 1.0}};

// out[i][r][c] (8, R, Cc): flip = 0: R = Co, Cc = Ci, tap k of W[r][c];  flip = 1: R = Ci,
// Cc = Co, tap 4-k of W[c][r] (the input-gradient kernel).  W (Co, Ci, 5) contiguous.
__global__ void wino_weight_kernel(int Co, int Ci, const float* __restrict__ W, int flip, float* __restrict__ out) {
  const int R = flip ? Ci : Co, Cc = flip ? Co : Ci;
  const int64_t n = (int64_t)R * Cc;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / Cc), c = (int)(e % Cc);
    const float* w = flip ? W + ((int64_t)c * Ci + r) * 5 : W + ((int64_t)r * Ci + c) * 5;
    double g[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) g[k] = w[flip ? 4 - k : k];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < 5; ++k) v += kG[i][k] * g[k];
      out[(int64_t)i * n + e] = (float)v;
    }
  }
}

// thread = (tile, 4 channels); grid (ceil(C/4 / 64), B * T / 4), block 64
__global__ __launch_bounds__(64) void wino_input_kernel(int T, int C, const float* __restrict__ x, int64_t ldx,
                                                        float* __restrict__ out, int64_t ntiles) {
  const int c = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (c >= C) return;
  const int64_t tile = blockIdx.y;
  const int64_t b = tile / (T / 4);
  const int q = (int)(tile % (T / 4));
  f32x4 d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 4 * q - 2 + j;
    d[j] = (t >= 0 && t < T) ? *reinterpret_cast<const f32x4*>(x + (b * T + t) * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (kBT[i][j] != 0.f) v += kBT[i][j] * d[j];
    *reinterpret_cast<f32x4*>(out + ((int64_t)i * ntiles + tile) * C + c) = v;
  }
}

__global__ __launch_bounds__(64) void wino_output_kernel(int T, int C, const float* __restrict__ Yt,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         int64_t ldy, int64_t ntiles) {
  const int c = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (c >= C) return;
  const int64_t tile = blockIdx.y;
  const int64_t b = tile / (T / 4);
  const int q = (int)(tile % (T / 4));
  f32x4 m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = *reinterpret_cast<const f32x4*>(Yt + ((int64_t)i * ntiles + tile) * C + c);
  const f32x4 bv = bias ? *reinterpret_cast<const f32x4*>(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    f32x4 v = bv;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (kAT[o][i] != 0.f) v += kAT[o][i] * m[i];
    *reinterpret_cast<f32x4*>(y + (b * T + 4 * q + o) * ldy + c) = v;
  }
}

// Weight gradient (the transpose of the forward algorithm): with
//   dY~[i][tile][c] = sum_o AT[o][i] dy[4q+o][c]   and   X~ the forward's input transform,
//   dW[co][ci][k]  = sum_i G[i][k] sum_tile dY~[i][tile][co] X~[i][tile][ci]
// = 8 GEMMs over K = B*T/4 tiles (one batched launch) and a G^T combine.
__global__ __launch_bounds__(64) void wino_dy_kernel(int T, int C, const float* __restrict__ dy, int64_t lddy,
                                                     float* __restrict__ out, int64_t ntiles) {
  const int c = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (c >= C) return;
  const int64_t tile = blockIdx.y;
  const int64_t b = tile / (T / 4);
  const int q = (int)(tile % (T / 4));
  f32x4 d[4];
#pragma unroll
  for (int o = 0; o < 4; ++o) d[o] = *reinterpret_cast<const f32x4*>(dy + (b * T + 4 * q + o) * lddy + c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < 4; ++o)
      if (kAT[o][i] != 0.f) v += kAT[o][i] * d[o];
    *reinterpret_cast<f32x4*>(out + ((int64_t)i * ntiles + tile) * C + c) = v;
  }
}

// dW (Co, Ci, 5) (=|+=) G^T M,  M (8, Co, Ci); the combine runs in double, rounds once
__global__ void wino_wgrad_kernel(int64_t n, const float* __restrict__ Mt, float* __restrict__ dW, int acc) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    double m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = Mt[(int64_t)i * n + e];
    float* w = dW + e * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      double v = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i) v += kG[i][k] * m[i];
      w[k] = acc ? w[k] + (float)v : (float)v;
    }
  }
}

}  // namespace

extern "C" int autovc_wino5_weights_f32(int Co, int Ci, const float* W, int flip, float* out, hipStream_t stream) {
  AVC_CHECK_ARG(Co > 0 && Ci > 0 && W && out && (flip == 0 || flip == 1), "autovc_wino5_weights_f32: bad args");
  const int64_t n = (int64_t)Co * Ci;
  hipLaunchKernelGGL(wino_weight_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                     stream, Co, Ci, W, flip, out);
  AVC_CHECK_LAUNCH("autovc_wino5_weights_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_input_f32(int B, int T, int C, const float* x, int64_t ldx, float* out,
                                      hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0 && x && out,
                "autovc_wino5_input_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(AVC_ALIGNED16(x) && AVC_ALIGNED16(out), "autovc_wino5_input_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_input_kernel, dim3((C / 4 + 63) / 64, (unsigned)ntiles), dim3(64), 0, stream, T, C, x, ldx,
                     out, ntiles);
  AVC_CHECK_LAUNCH("autovc_wino5_input_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_output_f32(int B, int T, int C, const float* Yt, const float* bias, float* y, int64_t ldy,
                                       hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldy % 4 == 0 && Yt && y,
                "autovc_wino5_output_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(AVC_ALIGNED16(Yt) && AVC_ALIGNED16(y) && (!bias || AVC_ALIGNED16(bias)),
                "autovc_wino5_output_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_output_kernel, dim3((C / 4 + 63) / 64, (unsigned)ntiles), dim3(64), 0, stream, T, C, Yt,
                     bias, y, ldy, ntiles);
  AVC_CHECK_LAUNCH("autovc_wino5_output_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_dy_f32(int B, int T, int C, const float* dy, int64_t lddy, float* out,
                                   hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && lddy % 4 == 0 && dy && out,
                "autovc_wino5_dy_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(AVC_ALIGNED16(dy) && AVC_ALIGNED16(out), "autovc_wino5_dy_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_dy_kernel, dim3((C / 4 + 63) / 64, (unsigned)ntiles), dim3(64), 0, stream, T, C, dy, lddy,
                     out, ntiles);
  AVC_CHECK_LAUNCH("autovc_wino5_dy_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_wgrad_f32(int Co, int Ci, const float* Mt, float* dW, int accumulate,
                                      hipStream_t stream) {
  AVC_CHECK_ARG(Co > 0 && Ci > 0 && Mt && dW, "autovc_wino5_wgrad_f32: bad args");
  const int64_t n = (int64_t)Co * Ci;
  hipLaunchKernelGGL(wino_wgrad_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                     stream, n, Mt, dW, accumulate);
  AVC_CHECK_LAUNCH("autovc_wino5_wgrad_f32");
  return avc::kOk;
}
