// LSTM recurrences (torch nn.LSTM semantics, used at model_vc_mel.py:61,90,104) on gfx950.
//
//   gates_t = gx_t + h_{t-1} W_hh^T            (gx_t = x_t W_ih^T + b_ih + b_hh: one GEMM
//                                               over all frames, done before the recurrence)
//   i,f,o = sigmoid, g = tanh;  c_t = f c_{t-1} + i g;  h_t = o tanh(c_t);  h_{-1} = c_{-1} = 0
//   torch gate order [i | f | g | o] along the 4H axis.
//
// Two regimes:
//  * large H (decoder lstm1 H=512, lstm2 H=1024): one launch per time step on the
//    caller's stream (a kernel boundary is cheaper than a grid barrier on MI355X,
//    MI355X_MICROARCH.md price list "boundary" vs "barrier-xcd").  Workgroup = 4 hidden
//    units x all 4 gates (16 W_hh rows) x every batch row; the 64x16xH product runs on
//    v_mfma_f32_16x16x4_f32 with h and W read as float4 straight from L2/MALL, and the
//    cell update is fused (no gates round trip through HBM).  Backward = per step a
//    pointwise kernel (dG_t from dh, dc) and a split-K recurrent product
//    dh_rec = dG_t W_hh through the pre-transposed W_hh^T.
//  * small H (encoder BLSTM, H=32): the whole sequence in one launch, one workgroup per
//    (direction, 8 batch rows), W_hh in LDS, one barrier per step (two in backward).
#include <hip/hip_ext.h>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int kThreads = 256;
constexpr int U = 4;          // hidden units per workgroup (large-H kernels)
constexpr int NCOL = 4 * U;   // 16 MFMA columns = 4 gates x U units

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// acc(16 rows of X x 16 W rows) += X[16 x K] * Wr[16 x K]^T with f32 MFMA 16x16x4.
// xrow: this lane's X row (already offset by 4*(lane>>4)), or null (row absent -> 0)
// wrow: this lane's W row (already offset by 4*(lane>>4))
__device__ __forceinline__ f32x4 mfma_rows(const float* xrow, const float* wrow, int K) {
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  int kc = 0;
  for (; kc + 32 <= K; kc += 32) {
    const f32x4 x0 = xrow ? ld4(xrow + kc) : z, w0 = ld4(wrow + kc);
    const f32x4 x1 = xrow ? ld4(xrow + kc + 16) : z, w1 = ld4(wrow + kc + 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[j], w0[j], a0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[j], w1[j], a1, 0, 0, 0);
  }
  for (; kc < K; kc += 16) {
    const f32x4 x0 = xrow ? ld4(xrow + kc) : z, w0 = ld4(wrow + kc);
#pragma unroll
    for (int j = 0; j < 4; ++j) a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[j], w0[j], a0, 0, 0, 0);
  }
  return a0 + a1;
}

struct StepArgs {
  int B, T, H;
  const float* gx; int64_t gx_ldb, gx_ldt;   // gx[b*gx_ldb + t*gx_ldt + r]
  const float* W;                            // W_hh (4H, H)
  float* h; int64_t h_ldb, h_ldt;            // h out/in: h[b*h_ldb + t*h_ldt + j]
  float* c;                                  // (B, T, H) cell states
  float* gates;                              // (B, T, 4H) post-activation gates or null
};

// One forward time step of a large-H layer.  grid.x = H / U.
__global__ __launch_bounds__(kThreads) void lstm_fwd_step_kernel(StepArgs a, int t, int tp) {
  __shared__ float tile[4][16][NCOL + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.x * U;
  const int H = a.H;
  const int n = lane & 15;                         // MFMA column: gate n>>2, unit n&3
  const int wr = (n >> 2) * H + j0 + (n & 3);      // W_hh row of that column
  const int nbt = (a.B + 15) >> 4;
  for (int bt0 = 0; bt0 < nbt; bt0 += 4) {
    const int bt = bt0 + w;
    const int b = bt * 16 + n;                     // A row (batch) of this lane
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (tp >= 0 && bt < nbt) {
      const float* xrow = b < a.B ? a.h + (int64_t)b * a.h_ldb + (int64_t)tp * a.h_ldt + 4 * (lane >> 4) : nullptr;
      acc = mfma_rows(xrow, a.W + (int64_t)wr * H + 4 * (lane >> 4), H);
    }
    // C/D map: col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[w][4 * (lane >> 4) + r][n] = acc[r];
    __syncthreads();
    {
      const int bl = lane >> 2, u = lane & 3;
      const int bb = bt * 16 + bl, j = j0 + u;
      if (bt < nbt && bb < a.B) {
        const float* g = a.gx + (int64_t)bb * a.gx_ldb + (int64_t)t * a.gx_ldt;
        const float gi = tile[w][bl][0 * U + u] + g[0 * H + j];
        const float gf = tile[w][bl][1 * U + u] + g[1 * H + j];
        const float gg = tile[w][bl][2 * U + u] + g[2 * H + j];
        const float go = tile[w][bl][3 * U + u] + g[3 * H + j];
        const float i_ = avc_sigmoid(gi), f_ = avc_sigmoid(gf), g_ = tanhf(gg), o_ = avc_sigmoid(go);
        const int64_t cb = (int64_t)bb * a.T * H;
        const float cp = tp >= 0 ? a.c[cb + (int64_t)tp * H + j] : 0.f;
        const float cn = f_ * cp + i_ * g_;
        a.c[cb + (int64_t)t * H + j] = cn;
        a.h[(int64_t)bb * a.h_ldb + (int64_t)t * a.h_ldt + j] = o_ * tanhf(cn);
        if (a.gates) {
          float* gs = a.gates + ((int64_t)bb * a.T + t) * 4 * H;
          gs[0 * H + j] = i_; gs[1 * H + j] = f_; gs[2 * H + j] = g_; gs[3 * H + j] = o_;
        }
      }
    }
    __syncthreads();
  }
}

// Backward pointwise for one step of a large-H layer: thread per (b, j).
//   dh = dh_out[t] + sum_s P[s]           (P: split-K partials of dG_{t'} W_hh, t' = later step)
//   dc = dc_state + dh o (1 - tanh(c)^2);  dG = [dc g i(1-i), dc c_prev f(1-f), dc i (1-g^2),
//   dh tanh(c) o(1-o)];  dc_state <- dc f
struct BwdArgs {
  int B, T, H;
  const float* dh_out; int64_t d_ldb, d_ldt;  // dL/dh from above (may be null)
  const float* gates;                          // (B,T,4H)
  const float* c;                              // (B,T,H)
  float* dG;                                   // (B,T,4H) out
  float* dc_state;                             // (B,H)
  const float* P; int S;                       // (S,B,H) partials or null
};

__global__ void lstm_bwd_pointwise_kernel(BwdArgs a, int t, int tp, int first) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t BH = (int64_t)a.B * a.H;
  if (idx >= BH) return;
  const int b = (int)(idx / a.H), j = (int)(idx % a.H);
  const int H = a.H;
  float dh = a.dh_out ? a.dh_out[(int64_t)b * a.d_ldb + (int64_t)t * a.d_ldt + j] : 0.f;
  if (!first && a.P)
    for (int s = 0; s < a.S; ++s) dh += a.P[(int64_t)s * BH + idx];
  const float* gs = a.gates + ((int64_t)b * a.T + t) * 4 * H;
  const float i_ = gs[j], f_ = gs[H + j], g_ = gs[2 * H + j], o_ = gs[3 * H + j];
  const float cc = a.c[((int64_t)b * a.T + t) * H + j];
  const float cp = tp >= 0 ? a.c[((int64_t)b * a.T + tp) * H + j] : 0.f;
  const float tc = tanhf(cc);
  const float dc = (first ? 0.f : a.dc_state[idx]) + dh * o_ * (1.f - tc * tc);
  float* d = a.dG + ((int64_t)b * a.T + t) * 4 * H;
  d[j] = dc * g_ * i_ * (1.f - i_);
  d[H + j] = dc * cp * f_ * (1.f - f_);
  d[2 * H + j] = dc * i_ * (1.f - g_ * g_);
  d[3 * H + j] = dh * tc * o_ * (1.f - o_);
  a.dc_state[idx] = dc * f_;
}

// Split-K recurrent product P[s][b][j] = sum_{r in split s} dG[b][t][r] W^T[j][r].
// grid = (H/16, S); 4 waves cover batch tiles of 16.
__global__ __launch_bounds__(kThreads) void lstm_bwd_rec_kernel(int B, int T, int H, const float* dG,
                                                               int t, const float* WT, float* P, int S) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.x * 16, s = blockIdx.y;
  const int K4 = 4 * H, ks = K4 / S, kb = s * ks;
  const int n = lane & 15;
  const int nbt = (B + 15) >> 4;
  for (int bt = w; bt < nbt; bt += 4) {
    const int b = bt * 16 + n;
    const float* xrow = b < B ? dG + ((int64_t)b * T + t) * K4 + kb + 4 * (lane >> 4) : nullptr;
    const f32x4 acc = mfma_rows(xrow, WT + (int64_t)(j0 + n) * K4 + kb + 4 * (lane >> 4), ks);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int bb = bt * 16 + 4 * (lane >> 4) + r;
      if (bb < B) P[((int64_t)s * B + bb) * H + j0 + n] = acc[r];
    }
  }
}

// ------------------------------------------------------------------ small H (BLSTM)
// Whole sequence, both directions in one launch.  grid = (ceil(B/8), ndir); block 256 =
// 8 batch rows x 32 units.  gx: (B,T,ndir*4H) [dir-major blocks]; h out: (B,T,ndir*H).
constexpr int SH = 32, SB = 8;

__global__ __launch_bounds__(kThreads) void blstm_fwd_kernel(int B, int T, const float* gx, const float* Whh_f,
                                                            const float* Whh_b, float* hout, float* call,
                                                            float* gates, int ndir) {
  __shared__ float Ws[4 * SH][SH + 1];
  __shared__ float hs[2][SB][SH];
  const int dir = blockIdx.y;
  const int bl = threadIdx.x / SH, j = threadIdx.x % SH;
  const int b = blockIdx.x * SB + bl;
  const float* W = dir ? Whh_b : Whh_f;
  for (int e = threadIdx.x; e < 4 * SH * SH; e += kThreads) Ws[e / SH][e % SH] = W[e];
  hs[0][bl][j] = 0.f;
  __syncthreads();
  const int G = ndir * 4 * SH, HO = ndir * SH;
  float c = 0.f;
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = dir ? T - 1 - s : s;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (b < B) {
      const float* g = gx + ((int64_t)b * T + t) * G + dir * 4 * SH;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = g[q * SH + j];
    }
#pragma unroll 8
    for (int k = 0; k < SH; ++k) {
      const float hv = hs[cur][bl][k];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = fmaf(hv, Ws[q * SH + j][k], acc[q]);
    }
    const float i_ = avc_sigmoid(acc[0]), f_ = avc_sigmoid(acc[1]), g_ = tanhf(acc[2]), o_ = avc_sigmoid(acc[3]);
    c = f_ * c + i_ * g_;
    const float h = o_ * tanhf(c);
    hs[cur ^ 1][bl][j] = h;
    if (b < B) {
      hout[((int64_t)b * T + t) * HO + dir * SH + j] = h;
      if (call) call[((int64_t)b * T + t) * HO + dir * SH + j] = c;
      if (gates) {
        float* gs = gates + ((int64_t)b * T + t) * G + dir * 4 * SH;
        gs[j] = i_; gs[SH + j] = f_; gs[2 * SH + j] = g_; gs[3 * SH + j] = o_;
      }
    }
    cur ^= 1;
    __syncthreads();
  }
}

// Backward of blstm_fwd_kernel: per direction, walk the sequence in reverse processing
// order.  dG: (B,T,ndir*4H).  dh_out: (B,T,ndir*H) or null.
__global__ __launch_bounds__(kThreads) void blstm_bwd_kernel(int B, int T, const float* dh_out, const float* gates,
                                                            const float* call, const float* Whh_f,
                                                            const float* Whh_b, float* dG, int ndir) {
  __shared__ float Ws[4 * SH][SH + 1];
  __shared__ float dgs[SB][4 * SH + 1];
  __shared__ float dhr[SB][SH];
  const int dir = blockIdx.y;
  const int bl = threadIdx.x / SH, j = threadIdx.x % SH;
  const int b = blockIdx.x * SB + bl;
  const float* W = dir ? Whh_b : Whh_f;
  for (int e = threadIdx.x; e < 4 * SH * SH; e += kThreads) Ws[e / SH][e % SH] = W[e];
  dhr[bl][j] = 0.f;
  __syncthreads();
  const int G = ndir * 4 * SH, HO = ndir * SH;
  float dcs = 0.f;
  for (int s = T - 1; s >= 0; --s) {
    const int t = dir ? T - 1 - s : s;
    const int tp = dir ? t + 1 : t - 1;   // previous step in processing order
    const bool has_prev = s > 0;
    float di = 0.f, df = 0.f, dg = 0.f, dO = 0.f;
    if (b < B) {
      const int64_t bt = (int64_t)b * T + t;
      float dh = dhr[bl][j] + (dh_out ? dh_out[bt * HO + dir * SH + j] : 0.f);
      const float* gs = gates + bt * G + dir * 4 * SH;
      const float i_ = gs[j], f_ = gs[SH + j], g_ = gs[2 * SH + j], o_ = gs[3 * SH + j];
      const float cc = call[bt * HO + dir * SH + j];
      const float cp = has_prev ? call[((int64_t)b * T + tp) * HO + dir * SH + j] : 0.f;
      const float tc = tanhf(cc);
      const float dc = dcs + dh * o_ * (1.f - tc * tc);
      di = dc * g_ * i_ * (1.f - i_);
      df = dc * cp * f_ * (1.f - f_);
      dg = dc * i_ * (1.f - g_ * g_);
      dO = dh * tc * o_ * (1.f - o_);
      dcs = dc * f_;
      float* d = dG + bt * G + dir * 4 * SH;
      d[j] = di; d[SH + j] = df; d[2 * SH + j] = dg; d[3 * SH + j] = dO;
    }
    dgs[bl][j] = di; dgs[bl][SH + j] = df; dgs[bl][2 * SH + j] = dg; dgs[bl][3 * SH + j] = dO;
    __syncthreads();
    // dh_rec[b][j] = sum_r dG[b][r] W[r][j]
    float acc = 0.f;
#pragma unroll 8
    for (int r = 0; r < 4 * SH; ++r) acc = fmaf(dgs[bl][r], Ws[r][j], acc);
    dhr[bl][j] = acc;
    __syncthreads();
  }
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" int autovc_lstm_fwd_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                   const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                   float* gates, int reverse, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && H > 0, "autovc_lstm_fwd_f32: bad dims B=%d T=%d H=%d", B, T, H);
  AVC_CHECK_ARG(H % 16 == 0, "autovc_lstm_fwd_f32: H must be a multiple of 16 (got %d)", H);
  AVC_CHECK_ARG(gx && W_hh && h && c_all, "autovc_lstm_fwd_f32: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh) && AVC_ALIGNED16(h) && (h_ldb % 4 == 0) && (h_ldt % 4 == 0),
                "autovc_lstm_fwd_f32: W_hh / h must be 16-byte aligned with strides %% 4 == 0");
  StepArgs a{B, T, H, gx, gx_ldb, gx_ldt, W_hh, h, h_ldb, h_ldt, c_all, gates};
  for (int s = 0; s < T; ++s) {
    const int t = reverse ? T - 1 - s : s;
    const int tp = s == 0 ? -1 : (reverse ? t + 1 : t - 1);
    hipLaunchKernelGGL(lstm_fwd_step_kernel, dim3(H / U), dim3(kThreads), 0, stream, a, t, tp);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_fwd_f32");
  return avc::kOk;
}

extern "C" int64_t autovc_lstm_bwd_workspace_floats(int B, int H, int splits) {
  return (int64_t)splits * B * H + (int64_t)B * H;
}

extern "C" int autovc_lstm_bwd_f32(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                                   const float* gates, const float* c_all, const float* W_hh_T, float* dG,
                                   int reverse, int splits, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && H > 0 && H % 16 == 0, "autovc_lstm_bwd_f32: bad dims");
  AVC_CHECK_ARG(splits >= 1 && (4 * H) % (16 * splits) == 0, "autovc_lstm_bwd_f32: 4H must split into multiples of 16");
  AVC_CHECK_ARG(gates && c_all && W_hh_T && dG && workspace, "autovc_lstm_bwd_f32: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_T) && AVC_ALIGNED16(dG), "autovc_lstm_bwd_f32: W_hh_T/dG alignment");
  float* P = workspace;
  float* dcs = workspace + (int64_t)splits * B * H;
  BwdArgs a{B, T, H, dh_out, d_ldb, d_ldt, gates, c_all, dG, dcs, P, splits};
  const int64_t BH = (int64_t)B * H;
  const int pw_blocks = (int)((BH + 255) / 256);
  for (int s = T - 1; s >= 0; --s) {
    const int t = reverse ? T - 1 - s : s;
    const int tp = s == 0 ? -1 : (reverse ? t + 1 : t - 1);
    const int first = s == T - 1;
    hipLaunchKernelGGL(lstm_bwd_pointwise_kernel, dim3(pw_blocks), dim3(256), 0, stream, a, t, tp, first);
    if (s > 0)
      hipLaunchKernelGGL(lstm_bwd_rec_kernel, dim3(H / 16, splits), dim3(kThreads), 0, stream, B, T, H,
                         (const float*)dG, t, W_hh_T, P, splits);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_bwd_f32");
  return avc::kOk;
}

extern "C" int autovc_blstm_fwd_f32(int B, int T, int H, int ndir, const float* gx, const float* W_hh_f,
                                    const float* W_hh_b, float* h, float* c_all, float* gates, hipStream_t stream) {
  AVC_CHECK_ARG(H == SH, "autovc_blstm_fwd_f32: small-H kernel is built for H=%d (got %d)", SH, H);
  AVC_CHECK_ARG(B > 0 && T > 0 && (ndir == 1 || ndir == 2), "autovc_blstm_fwd_f32: bad dims");
  AVC_CHECK_ARG(gx && W_hh_f && h && c_all && (ndir == 1 || W_hh_b), "autovc_blstm_fwd_f32: null pointer");
  hipLaunchKernelGGL(blstm_fwd_kernel, dim3((B + SB - 1) / SB, ndir), dim3(kThreads), 0, stream, B, T, gx,
                     W_hh_f, W_hh_b, h, c_all, gates, ndir);
  AVC_CHECK_LAUNCH("autovc_blstm_fwd_f32");
  return avc::kOk;
}

extern "C" int autovc_blstm_bwd_f32(int B, int T, int H, int ndir, const float* dh_out, const float* gates,
                                    const float* c_all, const float* W_hh_f, const float* W_hh_b, float* dG,
                                    hipStream_t stream) {
  AVC_CHECK_ARG(H == SH, "autovc_blstm_bwd_f32: small-H kernel is built for H=%d (got %d)", SH, H);
  AVC_CHECK_ARG(B > 0 && T > 0 && (ndir == 1 || ndir == 2), "autovc_blstm_bwd_f32: bad dims");
  AVC_CHECK_ARG(gates && c_all && W_hh_f && dG && (ndir == 1 || W_hh_b), "autovc_blstm_bwd_f32: null pointer");
  hipLaunchKernelGGL(blstm_bwd_kernel, dim3((B + SB - 1) / SB, ndir), dim3(kThreads), 0, stream, B, T, dh_out,
                     gates, c_all, W_hh_f, W_hh_b, dG, ndir);
  AVC_CHECK_LAUNCH("autovc_blstm_bwd_f32");
  return avc::kOk;
}

// ------------------------------------------------------------------ measurement
// Same launches as autovc_lstm_fwd_f32, each bracketed by hipExtLaunchKernelGGL's own
// start/stop events (timestamps taken by the dispatch itself, so the inter-kernel gap is
// excluded); synchronises and writes the mean per-launch kernel time in microseconds to
// *avg_us (host).  Used by bench.py for the roofline of the recurrent kernel.
extern "C" int autovc_lstm_fwd_timed_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                         const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                         float* gates, hipStream_t stream, float* avg_us) {
  AVC_CHECK_ARG(B > 0 && T > 1 && H > 0 && H % 16 == 0 && avg_us, "autovc_lstm_fwd_timed_f32: bad args");
  AVC_CHECK_ARG(gx && W_hh && h && c_all, "autovc_lstm_fwd_timed_f32: null pointer");
  StepArgs a{B, T, H, gx, gx_ldb, gx_ldt, W_hh, h, h_ldb, h_ldt, c_all, gates};
  hipEvent_t* ev = new hipEvent_t[2 * T];
  for (int i = 0; i < 2 * T; ++i) AVC_HIP(hipEventCreate(&ev[i]), "autovc_lstm_fwd_timed_f32/event");
  for (int s = 0; s < T; ++s) {
    const int tp = s == 0 ? -1 : s - 1;
    hipExtLaunchKernelGGL(lstm_fwd_step_kernel, dim3(H / U), dim3(kThreads), 0, stream, ev[2 * s], ev[2 * s + 1], 0,
                          a, s, tp);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_fwd_timed_f32");
  AVC_HIP(hipStreamSynchronize(stream), "autovc_lstm_fwd_timed_f32/sync");
  double tot = 0.0;
  int n = 0;
  for (int s = 1; s < T; ++s) {  // step 0 has no recurrent product: excluded from the mean
    float ms = 0.f;
    AVC_HIP(hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]), "autovc_lstm_fwd_timed_f32/elapsed");
    tot += ms;
    ++n;
  }
  for (int i = 0; i < 2 * T; ++i) (void)hipEventDestroy(ev[i]);
  delete[] ev;
  *avg_us = (float)(tot / n * 1000.0);
  return avc::kOk;
}
