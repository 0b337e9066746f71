// Prototype (not part of the product): LSTM step GEMMs fed straight from global memory into
// v_mfma_f32_32x32x2_f32 fragments, no LDS staging.  Operands are kept k-major (h^T, a
// gate-interleaved W^T, dG^T) so that the 32 lanes of a half-wave read 128 contiguous bytes
// per k.  Each of the NW waves of a workgroup owns a k-slice; partial tiles meet once in LDS.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lstm_direct_bench.hip -o tools/lstm_direct_bench
#include "../autovc_amd/csrc/lstm.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cmath>
#include <cstdio>
#include <vector>

namespace {

struct Direct {
  int B, Bp, T, H;
  const float* gx; int64_t gx_ldb, gx_ldt;
  const float* WpT;     // (H, 4H): WpT[k][x*32 + q*8 + u] = W_hh[q*H + 8x + u][k]
  const float* hT_prev; // (H, Bp)
  float* hT_next;       // (H, Bp)
  float* h; int64_t h_ldb, h_ldt;
  float* c;
  float* gates;
};

template <int NW, int U>
__global__ __launch_bounds__(64 * NW) void fwd_direct(Direct a, int t, int tp) {
  __shared__ float red[NW][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int H = a.H, G4 = 4 * H;
  const int x = blockIdx.x, b0 = blockIdx.y * 32, j0 = x * 8;
  const int bl = (threadIdx.x & 255) >> 3, u = threadIdx.x & 7;
  const int b = b0 + bl, j = j0 + u;
  const bool own = threadIdx.x < 256 && b < a.B;
  float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f;
  if (own) {
    const float* g = a.gx + (int64_t)b * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
    for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + j];
    if (tp >= 0) cp = a.c[(int64_t)b * a.T * H + (int64_t)tp * H + j];
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (tp >= 0) {
    const int Kw = H / NW;
    const int k0 = w * Kw + (lane >> 5);
    const float* pa = a.hT_prev + (int64_t)k0 * a.Bp + b0 + (lane & 31);
    const float* pb = a.WpT + (int64_t)k0 * G4 + x * 32 + (lane & 31);
    const int64_t sa = 2 * (int64_t)a.Bp, sb = 2 * (int64_t)G4;
    const int n = Kw / 2;
    for (int i0 = 0; i0 < n; i0 += U) {
      float va[U], vb[U];
#pragma unroll
      for (int i = 0; i < U; ++i) { va[i] = pa[(i0 + i) * sa]; vb[i] = pb[(i0 + i) * sb]; }
#pragma unroll
      for (int i = 0; i < U; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(va[i], vb[i], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][lane & 31] = acc[r];
  __syncthreads();
  if (!own) return;
  float s[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][bl][q * 8 + u];
    s[q] = v;
  }
  const float i_ = avc_sigmoid(s[0] + gxv[0]), f_ = avc_sigmoid(s[1] + gxv[1]);
  const float g_ = tanhf(s[2] + gxv[2]), o_ = avc_sigmoid(s[3] + gxv[3]);
  const float cn = f_ * cp + i_ * g_;
  const float hn = o_ * tanhf(cn);
  a.c[(int64_t)b * a.T * H + (int64_t)t * H + j] = cn;
  a.h[(int64_t)b * a.h_ldb + (int64_t)t * a.h_ldt + j] = hn;
  a.hT_next[(int64_t)j * a.Bp + b] = hn;
  if (a.gates) {
    float* gs = a.gates + ((int64_t)b * a.T + t) * 4 * H;
    gs[0 * H + j] = i_; gs[1 * H + j] = f_; gs[2 * H + j] = g_; gs[3 * H + j] = o_;
  }
}

__global__ void make_wpt(const float* W, float* WpT, int H) {
  const int64_t n = (int64_t)4 * H * H;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e / (4 * H)), col = (int)(e % (4 * H));
    const int x = col / 32, q = (col % 32) / 8, u = col % 8;
    WpT[e] = W[((int64_t)q * H + 8 * x + u) * H + k];
  }
}

// backward recurrent partials: P[s][b][j] = sum_{n in split s} dG[b][n] W[n][j]
// A = dGT (4H, Bp), B = W (4H, H) natural.  grid (H/32, Bp/32, S)
template <int NW, int U>
__global__ __launch_bounds__(64 * NW) void rec_direct(int B, int Bp, int H, const float* dGT, const float* W,
                                                      float* P) {
  __shared__ float red[NW][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.x * 32, b0 = blockIdx.y * 32, s = blockIdx.z, S = gridDim.z;
  const int ks = 4 * H / S, Kw = ks / NW;
  const int k0 = s * ks + w * Kw + (lane >> 5);
  const float* pa = dGT + (int64_t)k0 * Bp + b0 + (lane & 31);
  const float* pb = W + (int64_t)k0 * H + j0 + (lane & 31);
  const int64_t sa = 2 * (int64_t)Bp, sb = 2 * (int64_t)H;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int n = Kw / 2;
  for (int i0 = 0; i0 < n; i0 += U) {
    float va[U], vb[U];
#pragma unroll
    for (int i = 0; i < U; ++i) { va[i] = pa[(i0 + i) * sa]; vb[i] = pb[(i0 + i) * sb]; }
#pragma unroll
    for (int i = 0; i < U; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(va[i], vb[i], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][lane & 31] = acc[r];
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += 64 * NW) {
    const int m = e / 32, jj = e % 32;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][m][jj];
    if (b0 + m < B) P[((int64_t)s * B + b0 + m) * H + j0 + jj] = v;
  }
}

__global__ void transpose_w(const float* W, float* WT, int R, int C) {  // WT[c][r] = W[r][c]
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)R * C; e += (int64_t)gridDim.x * blockDim.x)
    WT[(e % C) * R + e / C] = W[e];
}

__global__ void transpose_bt(const float* dG, float* dGT, int B, int Bp, int T, int t, int G4) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < B * G4; e += gridDim.x * blockDim.x) {
    const int b = e / G4, n = e % G4;
    dGT[(int64_t)n * Bp + b] = dG[((int64_t)b * T + t) * G4 + n];
  }
}

}  // namespace

template <class F>
static float time_launches(int n, F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) f(i);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < n; ++i) f(i);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(err)); exit(1); }
  return ms * 1000.f / n;
}

int main() {
  const int B = 64, Bp = 64, T = 128;
  for (int H : {1024, 512}) {
    const int64_t G4 = 4 * H;
    std::vector<float> hW(G4 * H), hgx((size_t)B * T * G4);
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) * (1.0f / 16777216.f)) * 2.f - 1.f; };
    for (auto& v : hW) v = rnd() / sqrtf((float)H);
    for (auto& v : hgx) v = rnd() * 0.5f;
    float *W, *WT, *WpT, *gx, *h1, *h2, *c1, *c2, *g1, *g2, *hT, *P, *dGT;
    (void)hipMalloc(&W, G4 * H * 4);
    (void)hipMalloc(&WT, G4 * H * 4);
    (void)hipMalloc(&WpT, G4 * H * 4);
    (void)hipMalloc(&gx, hgx.size() * 4);
    for (float** p : {&h1, &h2, &c1, &c2}) (void)hipMalloc(p, (size_t)B * T * H * 4);
    for (float** p : {&g1, &g2}) (void)hipMalloc(p, (size_t)B * T * G4 * 4);
    (void)hipMalloc(&hT, (size_t)2 * H * Bp * 4);
    (void)hipMalloc(&P, (size_t)8 * B * H * 4);
    (void)hipMalloc(&dGT, (size_t)G4 * Bp * 4);
    (void)hipMemcpy(W, hW.data(), G4 * H * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(gx, hgx.data(), hgx.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemset(hT, 0, (size_t)2 * H * Bp * 4);
    hipLaunchKernelGGL(make_wpt, dim3(1024), dim3(256), 0, 0, W, WpT, H);
    hipLaunchKernelGGL(transpose_w, dim3(1024), dim3(256), 0, 0, W, WT, (int)G4, H);
    // reference: product kernel sequence
    (void)autovc_lstm_fwd_f32(B, T, H, gx, T * G4, G4, W, h1, (int64_t)T * H, H, c1, g1, 0, 0);
    Direct d{B, Bp, T, H, gx, T * G4, G4, WpT, hT, hT + (int64_t)H * Bp, h2, (int64_t)T * H, H, c2, g2};
    auto run_direct = [&](auto kern, int s) {
      Direct dd = d;
      dd.hT_prev = hT + (int64_t)((s + 1) & 1) * H * Bp;
      dd.hT_next = hT + (int64_t)(s & 1) * H * Bp;
      hipLaunchKernelGGL(kern, dim3(H / 8, Bp / 32), dim3(512), 0, 0, dd, s, s - 1);
    };
    for (int s = 0; s < T; ++s) run_direct(fwd_direct<8, 8>, s);
    (void)hipDeviceSynchronize();
    std::vector<float> a((size_t)B * T * H), bb((size_t)B * T * H);
    (void)hipMemcpy(a.data(), h1, a.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(bb.data(), h2, bb.size() * 4, hipMemcpyDeviceToHost);
    double md = 0, mx = 0;
    for (size_t i = 0; i < a.size(); ++i) { md = fmax(md, fabs(a[i] - bb[i])); mx = fmax(mx, fabs(a[i])); }
    printf("H=%d direct fwd vs product: max|diff| %.3g (max|h| %.3g)\n", H, md, mx);
    const dim3 grid_old(H / 8, (B + 31) / 32);
    printf("H=%d fwd product %.2f us | direct U8 %.2f | U16 %.2f | U4 %.2f | NW4 U8 %.2f\n", H,
           time_launches(T, [&](int s) {
             hipLaunchKernelGGL((lstm_fwd_step_kernel<0, KCH, NWV, DPF>), grid_old, dim3(64 * NWV), 0, 0,
                                StepArgs{B, T, H, gx, T * G4, G4, W, h1, (int64_t)T * H, H, c1, g1}, s % T,
                                (s % T) - 1);
           }),
           time_launches(T, [&](int s) { run_direct(fwd_direct<8, 8>, s % T); }),
           time_launches(T, [&](int s) { run_direct(fwd_direct<8, 16>, s % T); }),
           time_launches(T, [&](int s) { run_direct(fwd_direct<8, 4>, s % T); }),
           time_launches(T, [&](int s) {
             Direct dd = d;
             dd.hT_prev = hT + (int64_t)(((s % T) + 1) & 1) * H * Bp;
             dd.hT_next = hT + (int64_t)((s % T) & 1) * H * Bp;
             hipLaunchKernelGGL((fwd_direct<4, 8>), dim3(H / 8, Bp / 32), dim3(256), 0, 0, dd, s % T, (s % T) - 1);
           }));
    // backward recurrent product
    const int S = 4;
    hipLaunchKernelGGL(transpose_bt, dim3(256), dim3(256), 0, 0, g1, dGT, B, Bp, T, 5, (int)G4);
    hipLaunchKernelGGL((lstm_bwd_rec_kernel<KCH, NWV, DPF>), dim3(H / 32, (B + 31) / 32, S), dim3(64 * NWV), 0, 0,
                       B, T, H, (const float*)g1, 5, (const float*)WT, P);
    (void)hipDeviceSynchronize();
    std::vector<float> p1((size_t)S * B * H), p2((size_t)S * B * H);
    (void)hipMemcpy(p1.data(), P, p1.size() * 4, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL((rec_direct<8, 8>), dim3(H / 32, Bp / 32, S), dim3(512), 0, 0, B, Bp, H, dGT, W, P);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(p2.data(), P, p2.size() * 4, hipMemcpyDeviceToHost);
    md = 0; mx = 0;
    for (size_t i = 0; i < p1.size(); ++i) { md = fmax(md, fabs(p1[i] - p2[i])); mx = fmax(mx, fabs(p1[i])); }
    printf("H=%d direct rec vs product: max|diff| %.3g (max %.3g)\n", H, md, mx);
    printf("H=%d rec S=4 product %.2f us | direct U8 %.2f | U16 %.2f | NW4 U8 %.2f\n", H,
           time_launches(T, [&](int s) {
             hipLaunchKernelGGL((lstm_bwd_rec_kernel<KCH, NWV, DPF>), dim3(H / 32, (B + 31) / 32, S),
                                dim3(64 * NWV), 0, 0, B, T, H, (const float*)g1, s % T, (const float*)WT, P);
           }),
           time_launches(T, [&](int) {
             hipLaunchKernelGGL((rec_direct<8, 8>), dim3(H / 32, Bp / 32, S), dim3(512), 0, 0, B, Bp, H, dGT, W, P);
           }),
           time_launches(T, [&](int) {
             hipLaunchKernelGGL((rec_direct<8, 16>), dim3(H / 32, Bp / 32, S), dim3(512), 0, 0, B, Bp, H, dGT, W, P);
           }),
           time_launches(T, [&](int) {
             hipLaunchKernelGGL((rec_direct<4, 8>), dim3(H / 32, Bp / 32, S), dim3(256), 0, 0, B, Bp, H, dGT, W, P);
           }));
    for (float* p : {W, WT, WpT, gx, h1, h2, c1, c2, g1, g2, hT, P, dGT}) (void)hipFree(p);
  }
  return 0;
}
