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
__device__ __forceinline__ void wino_weight_elem(int Co, int Ci, const float* __restrict__ W, int flip,
                                                 float* __restrict__ out, int64_t n, int Cc, int64_t e) {
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

__global__ void wino_weight_kernel(int Co, int Ci, const float* __restrict__ W, int flip, float* __restrict__ out) {
  const int R = flip ? Ci : Co, Cc = flip ? Co : Ci;
  const int64_t n = (int64_t)R * Cc;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    wino_weight_elem(Co, Ci, W, flip, out, n, Cc, e);
}

// Every conv weight transform of a training step in one launch (blockIdx.y = job):
// kind 0 / 1 = the Winograd W~ (forward / flipped, as wino_weight_kernel), kind 2 / 3 =
// the im2col GEMM packs Wf[co][k*Ci + ci] / Wd[(4-k)*Co + co][ci] (elementwise.hip's
// conv_pack_kernel layouts), kind 4 / 5 = the same packs as bf16 (the bf16 GEMMs' bf16-source
// weight operands).  Same arithmetic per element as the single-layer kernels.
struct WJob { const float* W; float* out; int Co, Ci, kind; };
constexpr int kMaxWJobs = 48;
struct WJobs { WJob j[kMaxWJobs]; };

// kinds 6 / 7 / 8 take W as an (Co rows x Ci cols) matrix (the LSTM weights, model_vc_mel.py
// :90,104): 6 = its RNE bf16 copy, 7 = its fp32 transpose (Ci x Co), 8 = the bf16 transpose
// (32 x 32 LDS tiles, grid-stride over the tiles: the trip count is uniform per block).
__global__ __launch_bounds__(256) void conv_weights_batched_kernel(WJobs jobs) {
  __shared__ float tile[32][33];
  const WJob jb = jobs.j[blockIdx.y];
  const int Co = jb.Co, Ci = jb.Ci;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (jb.kind == 6) {
    const int64_t n = (int64_t)Co * Ci;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
      reinterpret_cast<__bf16*>(jb.out)[i] = (__bf16)jb.W[i];
    return;
  }
  if (jb.kind >= 7) {
    const int R = Co, C = Ci, tc = (C + 31) / 32;
    const int64_t ntiles = (int64_t)tc * ((R + 31) / 32);
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
      const int c0 = (int)(t % tc) * 32, r0 = (int)(t / tc) * 32;
      for (int k = ty; k < 32; k += 8) {
        const int r = r0 + k, c = c0 + tx;
        if (r < R && c < C) tile[k][tx] = jb.W[(int64_t)r * C + c];
      }
      __syncthreads();
      for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k, r = r0 + tx;
        if (r < R && c < C) {
          if (jb.kind == 7) jb.out[(int64_t)c * R + r] = tile[tx][k];
          else reinterpret_cast<__bf16*>(jb.out)[(int64_t)c * R + r] = (__bf16)tile[tx][k];
        }
      }
      __syncthreads();
    }
    return;
  }
  if (jb.kind <= 1) {
    const int flip = jb.kind;
    const int R = flip ? Ci : Co, Cc = flip ? Co : Ci;
    const int64_t n = (int64_t)R * Cc;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
      wino_weight_elem(Co, Ci, jb.W, flip, jb.out, n, Cc, e);
  } else {
    const int64_t total = (int64_t)Co * Ci * 5;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
      const int k = (int)(i % 5);
      const int64_t r = i / 5;
      const int ci = (int)(r % Ci), co = (int)(r / Ci);
      const float w = jb.W[i];
      const int64_t of = jb.kind == 2 || jb.kind == 4 ? (int64_t)co * 5 * Ci + (int64_t)k * Ci + ci
                                                       : ((int64_t)(4 - k) * Co + co) * Ci + ci;
      if (jb.kind <= 3) jb.out[of] = w;
      else reinterpret_cast<__bf16*>(jb.out)[of] = (__bf16)w;   // RNE, as the GEMM's staging rounds
    }
  }
}

enum Act { kNone = 0, kRelu = 1, kTanh = 2 };

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// BatchNorm + activation of the previous layer applied to its pre-BN output y on load:
// z = act(y * alpha + shift), coef = [alpha | shift | mean | invstd] (4 x C floats, from
// autovc_bn_finalize_f32 / autovc_bn_coef_f32) — the same fmaf as bn.hip's apply_kernel
__device__ __forceinline__ f32x4 bn_act(f32x4 y, f32x4 al, f32x4 sh, int act) {
  f32x4 z;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float v = fmaf(y[e], al[e], sh[e]);
    z[e] = act == kRelu ? fmaxf(v, 0.f) : (act == kTanh ? tanhf(v) : v);
  }
  return z;
}

// g = d act / d pre * dz at pre = y * alpha + shift (bn.hip's act_grad through the output:
// relu z > 0 <=> pre > 0, tanh 1 - z^2 with z = tanhf(pre) recomputed bit for bit)
__device__ __forceinline__ f32x4 act_back(f32x4 dz, f32x4 y, f32x4 al, f32x4 sh, int act) {
  if (act == kNone) return dz;
  f32x4 g;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float v = fmaf(y[e], al[e], sh[e]);
    if (act == kRelu) {
      g[e] = v > 0.f ? dz[e] : 0.f;
    } else {
      const float z = tanhf(v);
      g[e] = dz[e] * (1.f - z * z);
    }
  }
  return g;
}

// thread = (tile, 4 channels); grid (ceil(C/4 / 64), B * T / 4), block 64.  BN: the input
// is the previous layer's pre-BN output and its BatchNorm + activation are applied on load
// (the padding frames stay zero: the reference pads the activation, model_vc_mel.py:33)
template <bool BN>
__global__ __launch_bounds__(64) void wino_input_kernel(int T, int C, const float* __restrict__ x, int64_t ldx,
                                                        float* __restrict__ out, int64_t ntiles,
                                                        const float* __restrict__ coef, int act) {
  const int c = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (c >= C) return;
  const int64_t tile = blockIdx.y;
  const int64_t b = tile / (T / 4);
  const int q = (int)(tile % (T / 4));
  f32x4 al = {}, sh = {};
  if (BN) {
    al = ld4(coef + c);
    sh = ld4(coef + C + c);
  }
  f32x4 d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 4 * q - 2 + j;
    d[j] = (t >= 0 && t < T) ? *reinterpret_cast<const f32x4*>(x + (b * T + t) * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (BN && t >= 0 && t < T) d[j] = bn_act(d[j], al, sh, act);
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

// ---------------------------------------------------------------- fused Conv-BN chain
// (autovc_amd.functional.ConvBNChainFn: the encoder / decoder / postnet stacks,
// model_vc_mel.py:49-59,68-69,92-102,113-115,132-169).  These kernels share one geometry:
// block = 4 waves x 64 lanes, lane = 4 channels, wave = kTPW consecutive tiles of ONE
// sequence (T % (4 kTPW) == 0), so a block covers kTPB tiles and writes one partial row
// per channel (the finalize kernels sum the rows in fixed order: deterministic, no
// atomics), every load of a wave is issued before its first use, and the input-type
// transforms read each frame of the wave's window (4 kTPW + 4 frames) once instead of
// twice (neighbouring tiles share their 4 halo frames).
constexpr int kTPW = 1;                  // tiles per wave: 4 (1024 waves, halo frames shared)
                                         // measured 16.11-16.21 vs 16.00 ms/step for 1 (4096 waves),
                                         // profiles/r03/ab_conv_chain.txt
constexpr int kWaves = 8;                // waves per block
constexpr int kThreads = 64 * kWaves;
constexpr int kTPB = kWaves * kTPW;
constexpr int kWin = 4 * kTPW + 4;       // frames of a wave's window: 4q0 - 2 .. 4(q0 + kTPW) + 1

struct WaveTiles {
  int64_t tile0, b;
  int q0;
  bool live;
};

__device__ __forceinline__ WaveTiles wave_tiles(int T, int64_t ntiles) {
  WaveTiles w;
  w.tile0 = (int64_t)blockIdx.y * kTPB + (threadIdx.x >> 6) * kTPW;
  w.live = w.tile0 < ntiles;                 // ntiles % kTPW == 0: a live wave has all kTPW tiles
  w.b = w.tile0 / (T / 4);
  w.q0 = (int)(w.tile0 % (T / 4));
  return w;
}

// the 4 waves' per-channel double pairs (s1, s2) summed in fixed order into partial row
// blockIdx.y (w == 0 lanes write)
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], int C, int c, double* __restrict__ out, int stride) {
  __shared__ double red[kWaves][64][NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < NV; ++e) red[w][lane][e] = v[e];
  __syncthreads();
  if (w != 0 || c >= C) return;
#pragma unroll
  for (int e = 0; e < NV; ++e) {
    double a = red[0][lane][e];
#pragma unroll
    for (int q = 1; q < kWaves; ++q) a += red[q][lane][e];      // fixed order
    out[(int64_t)blockIdx.y * C * stride + (c + e / stride) * stride + e % stride] = a;
  }
}

__device__ __forceinline__ void block_pairs(double (&s1)[4], double (&s2)[4], int C, int c, double* __restrict__ part) {
  double v[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = s1[e];
    v[2 * e + 1] = s2[e];
  }
  block_sum<8>(v, C, c, part, 2);
}

// Input transform over a wave's window (T % 16 == 0): X~ of kTPW tiles from 4 kTPW + 4
// frames; BN: the previous layer's BatchNorm + activation applied on load (pads stay zero)
template <bool BN>
__global__ __launch_bounds__(kThreads) void wino_input_win_kernel(int T, int C, const float* __restrict__ x, int64_t ldx,
                                                             float* __restrict__ out, int64_t ntiles,
                                                             const float* __restrict__ coef, int act) {
  const int c = 4 * (blockIdx.x * 64 + (threadIdx.x & 63));
  const WaveTiles wt = wave_tiles(T, ntiles);
  if (c >= C || !wt.live) return;
  f32x4 al = {}, sh = {};
  if (BN) {
    al = ld4(coef + c);
    sh = ld4(coef + C + c);
  }
  f32x4 d[kWin];
#pragma unroll
  for (int s = 0; s < kWin; ++s) {
    const int t = 4 * wt.q0 - 2 + s;
    d[s] = (t >= 0 && t < T) ? ld4(x + (wt.b * T + t) * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (BN)
#pragma unroll
    for (int s = 0; s < kWin; ++s) {
      const int t = 4 * wt.q0 - 2 + s;
      if (t >= 0 && t < T) d[s] = bn_act(d[s], al, sh, act);
    }
#pragma unroll
  for (int i = 0; i < kTPW; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (kBT[k][j] != 0.f) v += kBT[k][j] * d[4 * i + j];
      st4(out + ((int64_t)k * ntiles + wt.tile0 + i) * C + c, v);
    }
}

// y = A^T Y~ + bias (the output transform) and the per-block BatchNorm statistics of y:
// part[rs][c] = (sum y, sum y^2) in double (raw sums: fp64 keeps the cancellation of
// E[y^2] - E[y]^2 far below fp32 resolution for activations of this scale)
__global__ __launch_bounds__(kThreads) void wino_output_stats_kernel(int T, int C, const float* __restrict__ Yt,
                                                                const float* __restrict__ bias, float* __restrict__ y,
                                                                int64_t ldy, int64_t ntiles,
                                                                double* __restrict__ part) {
  const int c = 4 * (blockIdx.x * 64 + (threadIdx.x & 63));
  const WaveTiles wt = wave_tiles(T, ntiles);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C && wt.live) {
    f32x4 m[kTPW][8];
#pragma unroll
    for (int i = 0; i < kTPW; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) m[i][k] = ld4(Yt + ((int64_t)k * ntiles + wt.tile0 + i) * C + c);
    const f32x4 bv = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < kTPW; ++i)
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        f32x4 v = bv;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (kAT[o][k] != 0.f) v += kAT[o][k] * m[i][k];
        st4(y + (wt.b * T + 4 * (wt.q0 + i) + o) * ldy + c, v);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[e] += (double)v[e];
          s2[e] += (double)v[e] * (double)v[e];
        }
      }
  }
  block_pairs(s1, s2, C, c, part);
}

// Input gradient of a conv whose input is the previous layer's BN + activation output:
// dz = A^T Yd~ (the output transform of the flipped correlation) and, for that layer's
// BatchNorm backward, part[rs][c] = (sum g, sum g (y - mean)) with g = act'(pre) dz
// (bn.hip's bwd_partial_kernel sums, here produced where dz is)
__global__ __launch_bounds__(kThreads) void wino_output_bnbwd_kernel(int T, int C, const float* __restrict__ Yt,
                                                                const float* __restrict__ yprev, int64_t ldy,
                                                                const float* __restrict__ coef, int act,
                                                                float* __restrict__ dz, int64_t lddz, int64_t ntiles,
                                                                double* __restrict__ part) {
  const int c = 4 * (blockIdx.x * 64 + (threadIdx.x & 63));
  const WaveTiles wt = wave_tiles(T, ntiles);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C && wt.live) {
    f32x4 m[kTPW][8], yv[kTPW][4];
#pragma unroll
    for (int i = 0; i < kTPW; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) m[i][k] = ld4(Yt + ((int64_t)k * ntiles + wt.tile0 + i) * C + c);
#pragma unroll
    for (int i = 0; i < kTPW; ++i)
#pragma unroll
      for (int o = 0; o < 4; ++o) yv[i][o] = ld4(yprev + (wt.b * T + 4 * (wt.q0 + i) + o) * ldy + c);
    const f32x4 al = ld4(coef + c), sh = ld4(coef + C + c), mu = ld4(coef + 2 * C + c);
#pragma unroll
    for (int i = 0; i < kTPW; ++i)
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (kAT[o][k] != 0.f) v += kAT[o][k] * m[i][k];
        st4(dz + (wt.b * T + 4 * (wt.q0 + i) + o) * lddz + c, v);
        const f32x4 g = act_back(v, yv[i][o], al, sh, act);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[e] += (double)g[e];
          s2[e] += (double)g[e] * (double)(yv[i][o][e] - mu[e]);
        }
      }
  }
  block_pairs(s1, s2, C, c, part);
}

// BatchNorm + activation backward of one layer fused with every consumer of its dy:
//   dy = (g - sum_g / M - xhat sum_gxhat / M) * alpha,  g = act'(pre) dz,  xhat = (y - mean) invstd
// (bn.hip's bwd_apply_kernel arithmetic) computed once per frame of the wave's window from
// dz and y, then per tile
//   Dt  = the weight gradient's dY~ transform of the tile's 4 frames (wino_dy_kernel),
//   Xt  = the input gradient's input transform of frames 4q-2 .. 4q+5 (wino_input_kernel),
//   bpart[rs][c] = sum over the block's frames of dy (the conv bias gradient, double).
// Dt / Xt / bpart may be null.  sums = [C][2] from autovc_bn_bwd_finalize_f32.  dy itself
// is never stored.
__global__ __launch_bounds__(kThreads) void wino_bnbwd_kernel(int T, int C, const float* __restrict__ dz, int64_t lddz,
                                                         const float* __restrict__ y, int64_t ldy,
                                                         const float* __restrict__ coef, int act,
                                                         const float* __restrict__ sums, float inv_m,
                                                         float* __restrict__ Dt, float* __restrict__ Xt,
                                                         double* __restrict__ bpart, int64_t ntiles) {
  const int c = 4 * (blockIdx.x * 64 + (threadIdx.x & 63));
  const WaveTiles wt = wave_tiles(T, ntiles);
  double sb[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C && wt.live) {
    // the window: own frames (slots 2 .. 4 kTPW + 1) always, halo slots only for the input transform
    f32x4 g[kWin], yv[kWin];
#pragma unroll
    for (int s = 0; s < kWin; ++s) {
      const int t = 4 * wt.q0 - 2 + s;
      const bool in = (s >= 2 && s < kWin - 2) || (Xt && t >= 0 && t < T);
      g[s] = in ? ld4(dz + (wt.b * T + t) * lddz + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      yv[s] = in ? ld4(y + (wt.b * T + t) * ldy + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const f32x4 al = ld4(coef + c), sh = ld4(coef + C + c), mu = ld4(coef + 2 * C + c), is = ld4(coef + 3 * C + c);
    f32x4 s0, s1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s0[e] = sums[2 * (c + e)] * inv_m;
      s1[e] = sums[2 * (c + e) + 1] * inv_m;
    }
#pragma unroll
    for (int s = 0; s < kWin; ++s) {
      const int t = 4 * wt.q0 - 2 + s;
      const bool in = (s >= 2 && s < kWin - 2) || (Xt && t >= 0 && t < T);
      const f32x4 gg = act_back(g[s], yv[s], al, sh, act);
      f32x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = (gg[e] - s0[e] - (yv[s][e] - mu[e]) * is[e] * s1[e]) * al[e];
      g[s] = in ? r : f32x4{0.f, 0.f, 0.f, 0.f};     // g now holds dy (zero outside the sequence)
    }
#pragma unroll
    for (int s = 2; s < kWin - 2; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) sb[e] += (double)g[s][e];
#pragma unroll
    for (int i = 0; i < kTPW; ++i) {
      if (Dt)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int o = 0; o < 4; ++o)
            if (kAT[o][k] != 0.f) v += kAT[o][k] * g[4 * i + 2 + o];
          st4(Dt + ((int64_t)k * ntiles + wt.tile0 + i) * C + c, v);
        }
      if (Xt)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (kBT[k][j] != 0.f) v += kBT[k][j] * g[4 * i + j];
          st4(Xt + ((int64_t)k * ntiles + wt.tile0 + i) * C + c, v);
        }
    }
  }
  if (bpart) block_sum<4>(sb, C, c, bpart, 1);
}

}  // namespace

extern "C" int64_t autovc_wino5_rows(int B, int T) {
  if (B <= 0 || T <= 0 || T % (4 * kTPW)) return -1;
  return ((int64_t)B * T / 4 + kTPB - 1) / kTPB;
}

extern "C" int autovc_wino5_weights_f32(int Co, int Ci, const float* W, int flip, float* out, hipStream_t stream) {
  AVC_CHECK_ARG(Co > 0 && Ci > 0 && W && out && (flip == 0 || flip == 1), "autovc_wino5_weights_f32: bad args");
  const int64_t n = (int64_t)Co * Ci;
  hipLaunchKernelGGL(wino_weight_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                     stream, Co, Ci, W, flip, out);
  AVC_CHECK_LAUNCH("autovc_wino5_weights_f32");
  return avc::kOk;
}

extern "C" int autovc_conv_weights_batched_f32(int n, const int* kinds, const int* Co, const int* Ci,
                                               const float* const* W, float* const* out, hipStream_t stream) {
  AVC_CHECK_ARG(n > 0 && kinds && Co && Ci && W && out, "autovc_conv_weights_batched_f32: bad args");
  for (int j0 = 0; j0 < n; j0 += kMaxWJobs) {
    WJobs jobs{};
    const int m = std::min(n - j0, kMaxWJobs);
    int64_t most = 1;
    for (int q = 0; q < m; ++q) {
      const int j = j0 + q;
      AVC_CHECK_ARG(kinds[j] >= 0 && kinds[j] <= 8 && Co[j] > 0 && Ci[j] > 0 && W[j] && out[j],
                    "autovc_conv_weights_batched_f32: bad job %d (kind %d, Co %d, Ci %d)", j, kinds[j], Co[j], Ci[j]);
      jobs.j[q] = WJob{W[j], out[j], Co[j], Ci[j], kinds[j]};
      const int64_t work = kinds[j] <= 1 ? (int64_t)Co[j] * Ci[j]
                         : kinds[j] <= 5 ? (int64_t)Co[j] * Ci[j] * 5
                         : kinds[j] == 6 ? (int64_t)Co[j] * Ci[j]
                                         : 256 * (int64_t)((Co[j] + 31) / 32) * ((Ci[j] + 31) / 32);   // a block per tile
      most = std::max<int64_t>(most, work);
    }
    hipLaunchKernelGGL(conv_weights_batched_kernel, dim3((unsigned)std::min<int64_t>((most + 255) / 256, 1024), m),
                       dim3(256), 0, stream, jobs);
  }
  AVC_CHECK_LAUNCH("autovc_conv_weights_batched_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_input_f32(int B, int T, int C, const float* x, int64_t ldx, float* out,
                                      hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0 && x && out,
                "autovc_wino5_input_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(AVC_ALIGNED16(x) && AVC_ALIGNED16(out), "autovc_wino5_input_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  if (T % (4 * kTPW) == 0)
    hipLaunchKernelGGL(wino_input_win_kernel<false>, dim3((C / 4 + 63) / 64, (unsigned)autovc_wino5_rows(B, T)),
                       dim3(kThreads), 0, stream, T, C, x, ldx, out, ntiles, (const float*)nullptr, 0);
  else
    hipLaunchKernelGGL(wino_input_kernel<false>, dim3((C / 4 + 63) / 64, (unsigned)ntiles), dim3(64), 0, stream, T, C,
                       x, ldx, out, ntiles, (const float*)nullptr, 0);
  AVC_CHECK_LAUNCH("autovc_wino5_input_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_input_bn_f32(int B, int T, int C, const float* y, int64_t ldy, const float* coef, int act,
                                         float* out, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldy % 4 == 0 && y && coef && out,
                "autovc_wino5_input_bn_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_wino5_input_bn_f32: unknown activation %d", act);
  AVC_CHECK_ARG(AVC_ALIGNED16(y) && AVC_ALIGNED16(out) && AVC_ALIGNED16(coef), "autovc_wino5_input_bn_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  if (T % (4 * kTPW) == 0)
    hipLaunchKernelGGL(wino_input_win_kernel<true>, dim3((C / 4 + 63) / 64, (unsigned)autovc_wino5_rows(B, T)),
                       dim3(kThreads), 0, stream, T, C, y, ldy, out, ntiles, coef, act);
  else
    hipLaunchKernelGGL(wino_input_kernel<true>, dim3((C / 4 + 63) / 64, (unsigned)ntiles), dim3(64), 0, stream, T, C,
                       y, ldy, out, ntiles, coef, act);
  AVC_CHECK_LAUNCH("autovc_wino5_input_bn_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_output_stats_f32(int B, int T, int C, const float* Yt, const float* bias, float* y,
                                             int64_t ldy, double* part, hipStream_t stream) {
  AVC_CHECK_ARG(T % (4 * kTPW) == 0, "%s: T must be a multiple of %d", "autovc_wino5_output_stats_f32", 4 * kTPW);
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldy % 4 == 0 && Yt && y && part,
                "autovc_wino5_output_stats_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(AVC_ALIGNED16(Yt) && AVC_ALIGNED16(y) && (!bias || AVC_ALIGNED16(bias)),
                "autovc_wino5_output_stats_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_output_stats_kernel, dim3((C / 4 + 63) / 64, (unsigned)autovc_wino5_rows(B, T)), dim3(kThreads),
                     0, stream, T, C, Yt, bias, y, ldy, ntiles, part);
  AVC_CHECK_LAUNCH("autovc_wino5_output_stats_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_output_bnbwd_f32(int B, int T, int C, const float* Yt, const float* yprev, int64_t ldy,
                                             const float* coef, int act, float* dz, int64_t lddz, double* part,
                                             hipStream_t stream) {
  AVC_CHECK_ARG(T % (4 * kTPW) == 0, "%s: T must be a multiple of %d", "autovc_wino5_output_bnbwd_f32", 4 * kTPW);
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && ldy % 4 == 0 && lddz % 4 == 0 && Yt && yprev &&
                coef && dz && part, "autovc_wino5_output_bnbwd_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_wino5_output_bnbwd_f32: unknown activation %d", act);
  AVC_CHECK_ARG(AVC_ALIGNED16(Yt) && AVC_ALIGNED16(yprev) && AVC_ALIGNED16(dz) && AVC_ALIGNED16(coef),
                "autovc_wino5_output_bnbwd_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_output_bnbwd_kernel, dim3((C / 4 + 63) / 64, (unsigned)autovc_wino5_rows(B, T)), dim3(kThreads),
                     0, stream, T, C, Yt, yprev, ldy, coef, act, dz, lddz, ntiles, part);
  AVC_CHECK_LAUNCH("autovc_wino5_output_bnbwd_f32");
  return avc::kOk;
}

extern "C" int autovc_wino5_bnbwd_f32(int B, int T, int C, const float* dz, int64_t lddz, const float* y, int64_t ldy,
                                      const float* coef, int act, const float* sums, float* Dt, float* Xt,
                                      double* bias_part, hipStream_t stream) {
  AVC_CHECK_ARG(T % (4 * kTPW) == 0, "%s: T must be a multiple of %d", "autovc_wino5_bnbwd_f32", 4 * kTPW);
  AVC_CHECK_ARG(B > 0 && T > 0 && T % 4 == 0 && C > 0 && C % 4 == 0 && lddz % 4 == 0 && ldy % 4 == 0 && dz && y &&
                coef && sums && (Dt || Xt || bias_part), "autovc_wino5_bnbwd_f32: bad args (T and C multiples of 4)");
  AVC_CHECK_ARG(act >= 0 && act <= 2, "autovc_wino5_bnbwd_f32: unknown activation %d", act);
  AVC_CHECK_ARG(AVC_ALIGNED16(dz) && AVC_ALIGNED16(y) && AVC_ALIGNED16(coef) && (!Dt || AVC_ALIGNED16(Dt)) &&
                (!Xt || AVC_ALIGNED16(Xt)), "autovc_wino5_bnbwd_f32: alignment");
  const int64_t ntiles = (int64_t)B * T / 4;
  hipLaunchKernelGGL(wino_bnbwd_kernel, dim3((C / 4 + 63) / 64, (unsigned)autovc_wino5_rows(B, T)), dim3(kThreads), 0,
                     stream, T, C, dz, lddz, y, ldy, coef, act, sums, 1.0f / (float)((int64_t)B * T), Dt, Xt,
                     bias_part, ntiles);
  AVC_CHECK_LAUNCH("autovc_wino5_bnbwd_f32");
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
