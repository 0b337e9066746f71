// Byte/index and elementwise kernels of the Generator step (gfx950).
//
//   frame_concat      model_vc_mel.py:64-66 (mel ++ emb over time) and :186-192 (code
//                     up-sample x freq ++ c_trg): out[b,t] = [X[b, t/rep], E[b]]
//   code_gather       model_vc_mel.py:74-79: codes[b,k] = [h_fwd[b, k*freq+freq-1],
//                     h_bwd[b, k*freq]]   (bit-exact copies, backward = exact scatter)
//   mse / l1          solver_encoder.py:230,233,236 (F.mse_loss, F.l1_loss, mean)
//   adam              torch.optim.Adam (solver_encoder.py:130,300; torch 1.8.1 update
//                     order: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//                     p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)) over ONE flat buffer
//   conv weight pack  Conv1d weight (Co,Ci,K) -> the GEMM operand images (gemm.hip)
//   transpose, column sums (bias gradients)
#include <algorithm>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

int grid_for(int64_t total, int per = 256) { return (int)std::min<int64_t>((total + per - 1) / per, 8192); }

#define GRID_STRIDE(i, total) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (total); i += (int64_t)gridDim.x * blockDim.x)

__global__ __launch_bounds__(256) void zero_words_kernel(uint32_t* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0u;
}

__global__ void frame_concat_kernel(int B, int T, int C1, int C2, int rep, const float* __restrict__ X,
                                    int64_t ldx, const float* __restrict__ E, float* __restrict__ out) {
  const int C = C1 + C2;
  const int64_t total = (int64_t)B * T * C;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    const int64_t bt = i / C;
    const int t = (int)(bt % T), b = (int)(bt / T);
    float v;
    if (c < C1) {
      const int64_t row = (int64_t)b * (T / rep) + t / rep;
      v = X[row * ldx + c];
    } else {
      v = E[(int64_t)b * C2 + (c - C1)];
    }
    out[i] = v;
  }
}

// dX[b, tx, c] (+)= sum_{t in [tx*rep, (tx+1)*rep)} dout[b, t, c]  for c < C1
__global__ void frame_concat_bwd_x_kernel(int B, int T, int C1, int C2, int rep, const float* __restrict__ dout,
                                          float* __restrict__ dX, int64_t ldx, int accumulate) {
  const int C = C1 + C2, Tx = T / rep;
  const int64_t total = (int64_t)B * Tx * C1;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C1);
    const int64_t bt = i / C1;
    const int tx = (int)(bt % Tx), b = (int)(bt / Tx);
    float s = 0.f;
    for (int r = 0; r < rep; ++r) s += dout[((int64_t)b * T + tx * rep + r) * C + c];
    float* d = dX + ((int64_t)b * Tx + tx) * ldx + c;
    *d = accumulate ? *d + s : s;
  }
}

// dE[b, c] (+)= sum_t dout[b, t, C1 + c]
__global__ void frame_concat_bwd_e_kernel(int B, int T, int C1, int C2, const float* __restrict__ dout,
                                          float* __restrict__ dE, int accumulate) {
  const int C = C1 + C2;
  const int64_t total = (int64_t)B * C2;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C2), b = (int)(i / C2);
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += dout[((int64_t)b * T + t) * C + C1 + c];
    dE[i] = accumulate ? dE[i] + s : s;
  }
}

// h: (B, T, 2D) [fwd D | bwd D] -> codes (B, (T/freq)*2D)
__global__ void code_gather_kernel(int B, int T, int D, int freq, const float* __restrict__ h,
                                   float* __restrict__ codes) {
  const int nc = T / freq, W = nc * 2 * D;
  const int64_t total = (int64_t)B * W;
  GRID_STRIDE(i, total) {
    const int q = (int)(i % W), b = (int)(i / W);
    const int k = q / (2 * D), d = q % (2 * D);
    const int t = d < D ? k * freq + freq - 1 : k * freq;
    codes[i] = h[((int64_t)b * T + t) * 2 * D + d];
  }
}

// exact inverse scatter: every element of dh written (zeros where no code reads)
__global__ void code_gather_bwd_kernel(int B, int T, int D, int freq, const float* __restrict__ dcodes,
                                       float* __restrict__ dh) {
  const int nc = T / freq, W = nc * 2 * D;
  const int64_t total = (int64_t)B * T * 2 * D;
  GRID_STRIDE(i, total) {
    const int d = (int)(i % (2 * D));
    const int64_t bt = i / (2 * D);
    const int t = (int)(bt % T), b = (int)(bt / T);
    const int k = t / freq, r = t % freq;
    const bool hit = d < D ? (r == freq - 1) : (r == 0);
    dh[i] = (hit && k < nc) ? dcodes[(int64_t)b * W + k * 2 * D + d] : 0.f;
  }
}

// ---- losses: two-stage deterministic mean reductions ------------------------------
constexpr int kLossBlocks = 256;

__global__ __launch_bounds__(256) void loss_partial_kernel(int kind, int64_t n, const float* __restrict__ a,
                                                          const float* __restrict__ b, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  GRID_STRIDE(i, n) {
    const float d = a[i] - b[i];
    s += kind == 0 ? (double)(d * d) : (double)fabsf(d);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void loss_finalize_kernel(int64_t n, const double* __restrict__ part, int nb, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
#pragma unroll 16
  for (int i = 0; i < nb; ++i) s += part[i];
  *out = (float)(s / (double)n);
}

// ga (+)= gout * scale * f'(a - b);  gb (+)= -(same)    (mse: 2(a-b)/n, l1: sign(a-b)/n)
__global__ void loss_bwd_kernel(int kind, int64_t n, const float* __restrict__ a, const float* __restrict__ b,
                                const float* __restrict__ gout, float* __restrict__ ga, float* __restrict__ gb,
                                int acc_a, int acc_b) {
  const float g = *gout / (float)n;
  GRID_STRIDE(i, n) {
    const float d = a[i] - b[i];
    const float v = kind == 0 ? 2.f * d * g : (d > 0.f ? g : (d < 0.f ? -g : 0.f));
    if (ga) ga[i] = acc_a ? ga[i] + v : v;
    if (gb) gb[i] = acc_b ? gb[i] - v : -v;
  }
}

// ---- Adam over a flat parameter buffer (torch 1.8.1 formula order) -----------------
__global__ void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, float lr, float beta1, float beta2, float eps, float wd,
                            float bc1, float bc2_sqrt) {
  const int64_t n4 = n / 4;
  const float step_size = lr / bc1;
  GRID_STRIDE(i, n4) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gg[k];
      if (wd != 0.f) gk = gk + wd * pp[k];
      mm[k] = mm[k] * beta1 + (1.f - beta1) * gk;
      vv[k] = vv[k] * beta2 + (1.f - beta2) * gk * gk;
      const float denom = sqrtf(vv[k]) / bc2_sqrt + eps;
      pp[k] = pp[k] - step_size * (mm[k] / denom);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t k = n4 * 4 + threadIdx.x;
    float gk = g[k];
    if (wd != 0.f) gk = gk + wd * p[k];
    m[k] = m[k] * beta1 + (1.f - beta1) * gk;
    v[k] = v[k] * beta2 + (1.f - beta2) * gk * gk;
    p[k] = p[k] - step_size * (m[k] / (sqrtf(v[k]) / bc2_sqrt + eps));
  }
}

// ---- conv weight images -----------------------------------------------------------
// W (Co, Ci, K) -> Wf[co][k*Ci + ci] = W[co][ci][k]           (forward B operand, NK)
//               -> Wd[(k*Co + co)*Ci + ci] = W[co][ci][K-1-k]  (input-grad B operand, KN)
__global__ void conv_pack_kernel(int Co, int Ci, int K, const float* __restrict__ W, float* __restrict__ Wf,
                                 float* __restrict__ Wd) {
  const int64_t total = (int64_t)Co * Ci * K;
  GRID_STRIDE(i, total) {
    const int k = (int)(i % K);
    const int64_t r = i / K;
    const int ci = (int)(r % Ci), co = (int)(r / Ci);
    const float w = W[i];
    if (Wf) Wf[(int64_t)co * K * Ci + (int64_t)k * Ci + ci] = w;
    if (Wd) Wd[((int64_t)(K - 1 - k) * Co + co) * Ci + ci] = w;
  }
}

// dWf[co][k*Ci + ci] -> dW[co][ci][k] (+)=
__global__ void conv_unpack_grad_kernel(int Co, int Ci, int K, const float* __restrict__ dWf,
                                        float* __restrict__ dW, int accumulate) {
  const int64_t total = (int64_t)Co * Ci * K;
  GRID_STRIDE(i, total) {
    const int k = (int)(i % K);
    const int64_t r = i / K;
    const int ci = (int)(r % Ci), co = (int)(r / Ci);
    const float v = dWf[(int64_t)co * K * Ci + (int64_t)k * Ci + ci];
    dW[i] = accumulate ? dW[i] + v : v;
  }
}

// out[c][r] = in[r][c], 32x32 LDS tiles
// out[m] = x[m] / ||x[m]||_2 (model_bl.py:17-19): one 256-thread workgroup per row, the
// squares summed in fixed order (per-thread strided partials, then an LDS tree).
__global__ __launch_bounds__(256) void l2norm_rows_kernel(int N, const float* __restrict__ x, int64_t ldx,
                                                          float* __restrict__ out, int64_t ldo) {
  __shared__ float part[256];
  const float* row = x + (int64_t)blockIdx.x * ldx;
  float s = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) s += row[n] * row[n];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  const float norm = sqrtf(part[0]);
  float* o = out + (int64_t)blockIdx.x * ldo;
  for (int n = threadIdx.x; n < N; n += 256) o[n] = row[n] / norm;
}

__global__ void transpose_kernel(int R, int C, const float* __restrict__ in, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    if (r < R && c < C) tile[k][tx] = in[(int64_t)r * C + c];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < R && c < C) out[(int64_t)c * R + r] = tile[tx][k];
  }
}

// column sums: out[c] (+)= sum_r X[r*ld + c]  (two-stage, deterministic)
constexpr int kColSplits = 128;

__global__ __launch_bounds__(256) void colsum_partial_kernel(int64_t M, int N, const float* __restrict__ X,
                                                            int64_t ld, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rs = blockIdx.y, RS = gridDim.y;
  const int64_t r0 = M * rs / RS, r1 = M * (rs + 1) / RS;
  float s = 0.f;
  if (c < N)
#pragma unroll 4
    for (int64_t r = r0 + w; r < r1; r += 4) s += X[r * ld + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < N) part[(int64_t)rs * N + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// 16 row groups x 16 columns per block (as bn.hip's finalize kernels): RS/16 loads in
// flight per thread, the 16 group sums added in group order (deterministic)
__global__ __launch_bounds__(256) void colsum_finalize_kernel(int N, int RS, const float* __restrict__ part,
                                                              float* __restrict__ out, float* __restrict__ out2,
                                                              int accumulate) {
  __shared__ float red[16][16];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < N)
#pragma unroll 8
    for (int rs = g; rs < RS; rs += 16) s += part[(int64_t)rs * N + c];
  red[g][cl] = s;
  __syncthreads();
  if (threadIdx.x >= 16 || c >= N) return;
  s = 0.f;
  for (int q = 0; q < 16; ++q) s += red[q][cl];
  out[c] = accumulate ? out[c] + s : s;
  if (out2) out2[c] = accumulate ? out2[c] + s : s;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" int autovc_frame_concat_f32(int B, int T, int C1, int C2, int rep, const float* X, int64_t ldx,
                                       const float* E, float* out, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && C1 >= 0 && C2 >= 0 && rep > 0 && T % rep == 0,
                "autovc_frame_concat_f32: bad dims (T=%d must be a multiple of rep=%d)", T, rep);
  AVC_CHECK_ARG(out && (C1 == 0 || X) && (C2 == 0 || E), "autovc_frame_concat_f32: null pointer");
  const int64_t total = (int64_t)B * T * (C1 + C2);
  hipLaunchKernelGGL(frame_concat_kernel, dim3(grid_for(total)), dim3(256), 0, stream, B, T, C1, C2, rep, X, ldx, E,
                     out);
  AVC_CHECK_LAUNCH("autovc_frame_concat_f32");
  return avc::kOk;
}

extern "C" int autovc_frame_concat_bwd_f32(int B, int T, int C1, int C2, int rep, const float* dout, float* dX,
                                           int64_t ldx, float* dE, int accumulate, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && rep > 0 && T % rep == 0 && dout, "autovc_frame_concat_bwd_f32: bad args");
  if (dX && C1 > 0)
    hipLaunchKernelGGL(frame_concat_bwd_x_kernel, dim3(grid_for((int64_t)B * (T / rep) * C1)), dim3(256), 0, stream,
                       B, T, C1, C2, rep, dout, dX, ldx, accumulate);
  if (dE && C2 > 0)
    hipLaunchKernelGGL(frame_concat_bwd_e_kernel, dim3(grid_for((int64_t)B * C2)), dim3(256), 0, stream, B, T, C1,
                       C2, dout, dE, accumulate);
  AVC_CHECK_LAUNCH("autovc_frame_concat_bwd_f32");
  return avc::kOk;
}

extern "C" int autovc_code_gather_f32(int B, int T, int D, int freq, const float* h, float* codes,
                                      hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && D > 0 && freq > 0 && T >= freq && T % freq == 0,
                "autovc_code_gather_f32: T=%d must be a positive multiple of freq=%d", T, freq);
  AVC_CHECK_ARG(h && codes, "autovc_code_gather_f32: null pointer");
  hipLaunchKernelGGL(code_gather_kernel, dim3(grid_for((int64_t)B * (T / freq) * 2 * D)), dim3(256), 0, stream, B,
                     T, D, freq, h, codes);
  AVC_CHECK_LAUNCH("autovc_code_gather_f32");
  return avc::kOk;
}

extern "C" int autovc_code_gather_bwd_f32(int B, int T, int D, int freq, const float* dcodes, float* dh,
                                          hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && D > 0 && freq > 0 && T >= freq && T % freq == 0, "autovc_code_gather_bwd_f32: bad dims");
  AVC_CHECK_ARG(dcodes && dh, "autovc_code_gather_bwd_f32: null pointer");
  hipLaunchKernelGGL(code_gather_bwd_kernel, dim3(grid_for((int64_t)B * T * 2 * D)), dim3(256), 0, stream, B, T, D,
                     freq, dcodes, dh);
  AVC_CHECK_LAUNCH("autovc_code_gather_bwd_f32");
  return avc::kOk;
}

extern "C" int64_t autovc_loss_workspace_bytes(void) { return kLossBlocks * sizeof(double); }

extern "C" int autovc_loss_f32(int kind, int64_t n, const float* a, const float* b, float* out, void* workspace,
                               hipStream_t stream) {
  AVC_CHECK_ARG(kind == 0 || kind == 1, "autovc_loss_f32: kind must be 0 (mse) or 1 (l1)");
  AVC_CHECK_ARG(n > 0 && a && b && out && workspace, "autovc_loss_f32: bad args");
  hipLaunchKernelGGL(loss_partial_kernel, dim3(kLossBlocks), dim3(256), 0, stream, kind, n, a, b,
                     reinterpret_cast<double*>(workspace));
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, stream, n,
                     reinterpret_cast<const double*>(workspace), kLossBlocks, out);
  AVC_CHECK_LAUNCH("autovc_loss_f32");
  return avc::kOk;
}

extern "C" int autovc_loss_bwd_f32(int kind, int64_t n, const float* a, const float* b, const float* gout,
                                   float* ga, float* gb, int acc_a, int acc_b, hipStream_t stream) {
  AVC_CHECK_ARG(kind == 0 || kind == 1, "autovc_loss_bwd_f32: kind must be 0 (mse) or 1 (l1)");
  AVC_CHECK_ARG(n > 0 && a && b && gout, "autovc_loss_bwd_f32: bad args");
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, stream, kind, n, a, b, gout, ga, gb, acc_a,
                     acc_b);
  AVC_CHECK_LAUNCH("autovc_loss_bwd_f32");
  return avc::kOk;
}

extern "C" int autovc_adam_f32(int64_t n, float* p, const float* g, float* m, float* v, float lr, float beta1,
                               float beta2, float eps, float weight_decay, float bias_correction1,
                               float bias_correction2_sqrt, hipStream_t stream) {
  AVC_CHECK_ARG(n >= 0 && p && g && m && v, "autovc_adam_f32: bad args");
  AVC_CHECK_ARG(AVC_ALIGNED16(p) && AVC_ALIGNED16(g) && AVC_ALIGNED16(m) && AVC_ALIGNED16(v),
                "autovc_adam_f32: buffers must be 16-byte aligned");
  if (n == 0) return avc::kOk;
  hipLaunchKernelGGL(adam_kernel, dim3(std::max(1, grid_for(n / 4))), dim3(256), 0, stream, n, p, g, m, v, lr, beta1,
                     beta2, eps, weight_decay, bias_correction1, bias_correction2_sqrt);
  AVC_CHECK_LAUNCH("autovc_adam_f32");
  return avc::kOk;
}

extern "C" int autovc_conv_pack_f32(int Co, int Ci, int K, const float* W, float* Wf, float* Wd,
                                    hipStream_t stream) {
  AVC_CHECK_ARG(Co > 0 && Ci > 0 && K > 0 && W && (Wf || Wd), "autovc_conv_pack_f32: bad args");
  hipLaunchKernelGGL(conv_pack_kernel, dim3(grid_for((int64_t)Co * Ci * K)), dim3(256), 0, stream, Co, Ci, K, W, Wf,
                     Wd);
  AVC_CHECK_LAUNCH("autovc_conv_pack_f32");
  return avc::kOk;
}

extern "C" int autovc_conv_unpack_grad_f32(int Co, int Ci, int K, const float* dWf, float* dW, int accumulate,
                                           hipStream_t stream) {
  AVC_CHECK_ARG(Co > 0 && Ci > 0 && K > 0 && dWf && dW, "autovc_conv_unpack_grad_f32: bad args");
  hipLaunchKernelGGL(conv_unpack_grad_kernel, dim3(grid_for((int64_t)Co * Ci * K)), dim3(256), 0, stream, Co, Ci, K,
                     dWf, dW, accumulate);
  AVC_CHECK_LAUNCH("autovc_conv_unpack_grad_f32");
  return avc::kOk;
}

extern "C" int autovc_transpose_f32(int R, int C, const float* in, float* out, hipStream_t stream) {
  AVC_CHECK_ARG(R > 0 && C > 0 && in && out && in != out, "autovc_transpose_f32: bad args");
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, stream, R, C, in, out);
  AVC_CHECK_LAUNCH("autovc_transpose_f32");
  return avc::kOk;
}

extern "C" int autovc_l2norm_rows_f32(int M, int N, const float* x, int64_t ldx, float* out, int64_t ldo,
                                     hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && N > 0 && x && out && ldx >= N && ldo >= N, "autovc_l2norm_rows_f32: bad args");
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3(M), dim3(256), 0, stream, N, x, ldx, out, ldo);
  AVC_CHECK_LAUNCH("autovc_l2norm_rows_f32");
  return avc::kOk;
}

extern "C" int64_t autovc_colsum_workspace_floats(int N) { return (int64_t)kColSplits * N; }

extern "C" int autovc_colsum_f32(int64_t M, int N, const float* X, int64_t ld, float* out, float* out2,
                                 int accumulate, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(M > 0 && N > 0 && X && out && workspace, "autovc_colsum_f32: bad args");
  const int RS = (int)std::min<int64_t>(kColSplits, M);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 63) / 64, RS), dim3(256), 0, stream, M, N, X, ld, workspace);
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3((N + 15) / 16), dim3(256), 0, stream, N, RS,
                     (const float*)workspace, out, out2, accumulate);
  AVC_CHECK_LAUNCH("autovc_colsum_f32");
  return avc::kOk;
}

hipError_t avc::zero_async(void* p, size_t bytes, hipStream_t stream) {
  const int64_t n = (int64_t)(bytes / 4);
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, static_cast<uint32_t*>(p), n);
  return hipGetLastError();
}
