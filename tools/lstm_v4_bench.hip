// Microbenchmark (not part of the product): where the time of one large-H LSTM step goes
// (H=1024 / 512, B=64).  Decomposes the product step kernel (LDS-staged tile core) into
// launch floor, prologue/epilogue, MFMA stream and operand fill, and times a probe of the
// alternative "direct-fragment" core: operands loaded global -> VGPR straight in the
// v_mfma_f32_16x16x4_f32 layout from a k-blocked copy X[k/4][row][4] (16 lanes read 256
// contiguous bytes), no LDS staging, every wave owning a K slice of the whole 32x32 tile.
// Results (round 1): see the log this prints.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lstm_v4_bench.hip -o tools/lstm_v4_bench
#include "../autovc_amd/csrc/lstm.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

constexpr int DNW = 8;
__global__ __launch_bounds__(512) void empty_kernel(float* p, int t) {
  if (t == -5) p[0] = 1.f;
}

// the direct core's MFMA stream (nb 16-k blocks per wave, 16 MFMAs each) on VGPR operands
__global__ __launch_bounds__(512) void mfma_only(float* p, int nb, int t) {
  const int lane = threadIdx.x & 63;
  f32x4 x[4];
  for (int i = 0; i < 4; ++i) x[i] = f32x4{lane * 1e-3f + i, 1.f, 2.f, (float)t};
  f32x4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int bk = 0; bk < nb; ++bk)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][jj], x[2][jj], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][jj], x[3][jj], acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][jj], x[2][jj], acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][jj], x[3][jj], acc[3], 0, 0, 0);
    }
  const float v = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (v == -12345.f) p[threadIdx.x] = v;
}

// k-blocked operand layout X[(k/4)][row][4]: lane (s, i) of a 16-k block reads 16 B at
// ((4 kb + s) R + row0 + i) * 4 -> 16 lanes cover 256 contiguous bytes (timing probe).
__device__ __forceinline__ unsigned long long rt_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int NR, int ABL = 0, int NWK = 8>
__global__ __launch_bounds__(64 * NWK) void fwd_kb(StepArgs a, const float* hk, int RA, const float* Wk, int RB, int t,
                                              int tp, unsigned long long* stamps = nullptr) {
  unsigned long long ts[6] = {0, 0, 0, 0, 0, 0};
  if (ABL & 8) ts[0] = rt_stamp();
  __shared__ float red[NWK * 32 * 33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int H = a.H;
  const int j0 = blockIdx.x * UT, b0 = blockIdx.y * TB;
  const int bl = (threadIdx.x & 255) >> 3, u = threadIdx.x & 7;
  const int b = b0 + bl, j = j0 + u;
  const bool own = threadIdx.x < 256 && b < a.B;
  float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f;
  if (own) {
    const float* g = a.gx + (int64_t)b * a.gx_ldb + (int64_t)t * a.gx_ldt;
    for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + j];
    if (tp >= 0) cp = a.c[(int64_t)b * a.T * H + (int64_t)tp * H + j];
  }
  constexpr int RK = 64, NB = RK / 16;
  const int i16 = lane & 15, sg = lane >> 4;
  const float* pa = hk + ((int64_t)sg * RA + ((ABL & 2) ? 0 : b0) + i16) * 4;
  const float* pb = Wk + ((int64_t)sg * RB + ((ABL & 1) ? 0 : blockIdx.x * 32) + i16) * 4;
  const int64_t sa = (int64_t)16 * RA, sb = (int64_t)16 * RB;   // floats per 4 k-blocks
  const int kb0 = w * NR * NB;
  f32x4 v[2][4][NB];
  auto load = [&](f32x4 (&x)[4][NB], int kb) {
#pragma unroll
    for (int bk = 0; bk < NB; ++bk) {
      x[0][bk] = *reinterpret_cast<const f32x4*>(pa + (kb + bk) * sa);
      x[1][bk] = *reinterpret_cast<const f32x4*>(pa + (kb + bk) * sa + 64);
      x[2][bk] = *reinterpret_cast<const f32x4*>(pb + (kb + bk) * sb);
      x[3][bk] = *reinterpret_cast<const f32x4*>(pb + (kb + bk) * sb + 64);
    }
  };
  f32x4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (tp >= 0) {
    load(v[0], kb0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int rd = 0; rd < NR; ++rd) {
      if (rd + 1 < NR) load(v[(rd + 1) & 1], kb0 + (rd + 1) * NB);
      __builtin_amdgcn_sched_barrier(0);
      if ((ABL & 8) && rd == 0) ts[1] = rt_stamp();
      const auto& x = v[rd & 1];
#pragma unroll
      for (int bk = 0; bk < NB; ++bk)
        if (ABL & 4) {
          acc[0] += x[0][bk]; acc[1] += x[1][bk]; acc[2] += x[2][bk]; acc[3] += x[3][bk];
        } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][bk][jj], x[2][bk][jj], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][bk][jj], x[3][bk][jj], acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][bk][jj], x[2][bk][jj], acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][bk][jj], x[3][bk][jj], acc[3], 0, 0, 0);
        }
        }
      if ((ABL & 8) && rd < 2) ts[2 + rd] = rt_stamp();
    }
  }
  float* rw = red + w * 32 * 33;
  for (int i = 0; i < 4; ++i)
    for (int rr = 0; rr < 4; ++rr) rw[((i >> 1) * 16 + 4 * sg + rr) * 33 + (i & 1) * 16 + i16] = acc[i][rr];
  __syncthreads();
  if (ABL & 8) ts[4] = rt_stamp();
  if ((ABL & 8) && lane == 0) {
    unsigned long long* st = stamps + ((int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * NWK + w) * 6;
    for (int i = 0; i < 5; ++i) st[i] = ts[i];
  }
  if (!own) return;
  float pre[4];
  for (int q = 0; q < 4; ++q) {
    float vv = 0.f;
    for (int ww = 0; ww < NWK; ++ww) vv += red[ww * 32 * 33 + bl * 33 + q * UT + u];
    pre[q] = vv;
  }
  const float i_ = avc_sigmoid(pre[0] + gxv[0]), f_ = avc_sigmoid(pre[1] + gxv[1]);
  const float g_ = tanhf(pre[2] + gxv[2]), o_ = avc_sigmoid(pre[3] + gxv[3]);
  const float cn = f_ * cp + i_ * g_;
  a.c[(int64_t)b * a.T * H + (int64_t)t * H + j] = cn;
  a.h[(int64_t)b * a.h_ldb + (int64_t)t * a.h_ldt + j] = o_ * tanhf(cn);
  if (a.gates) {
    float* gs = a.gates + ((int64_t)b * a.T + t) * 4 * H;
    gs[0 * H + j] = i_; gs[1 * H + j] = f_; gs[2 * H + j] = g_; gs[3 * H + j] = o_;
  }
}

// stacked two-layer probe on the k-blocked direct core (timing only): blockIdx.z = 0 runs
// a K = H step (h0, W_hh0), z = 1 a K = 2H step ([h0 ; h1] x [W_ih1 ; W_hh1]); rounds of
// RK k per wave, double-buffered; 2 workgroups per CU -> <= 128 VGPRs.
template <int RK, int NR>
__device__ __forceinline__ void kb_core(float* red, const float* const* pa, const float* const* pb, int K1, int RA,
                                        int RB) {
  constexpr int NB = RK / 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i16 = lane & 15, sg = lane >> 4;
  const int64_t sa = (int64_t)16 * RA, sb = (int64_t)16 * RB;
  const int kb0 = w * NR * NB;
  const int nb1 = K1 / 16;
  f32x4 v[2][4][NB];
  auto load = [&](f32x4 (&x)[4][NB], int kb) {
    const bool s2 = kb >= nb1;
    const int kk = s2 ? kb - nb1 : kb;
    const float* A = pa[s2] + (int64_t)kk * sa + (int64_t)sg * RA * 4 + i16 * 4;
    const float* Bq = pb[s2] + (int64_t)kk * sb + (int64_t)sg * RB * 4 + i16 * 4;
#pragma unroll
    for (int bk = 0; bk < NB; ++bk) {
      x[0][bk] = *reinterpret_cast<const f32x4*>(A + bk * sa);
      x[1][bk] = *reinterpret_cast<const f32x4*>(A + bk * sa + 64);
      x[2][bk] = *reinterpret_cast<const f32x4*>(Bq + bk * sb);
      x[3][bk] = *reinterpret_cast<const f32x4*>(Bq + bk * sb + 64);
    }
  };
  f32x4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(v[0], kb0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int rd = 0; rd < NR; ++rd) {
    if (rd + 1 < NR) load(v[(rd + 1) & 1], kb0 + (rd + 1) * NB);
    __builtin_amdgcn_sched_barrier(0);
    const auto& x = v[rd & 1];
#pragma unroll
    for (int bk = 0; bk < NB; ++bk)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][bk][jj], x[2][bk][jj], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0][bk][jj], x[3][bk][jj], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][bk][jj], x[2][bk][jj], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1][bk][jj], x[3][bk][jj], acc[3], 0, 0, 0);
      }
  }
  float* rw = red + w * 32 * 33;
  for (int i = 0; i < 4; ++i)
    for (int rr = 0; rr < 4; ++rr) rw[((i >> 1) * 16 + 4 * sg + rr) * 33 + (i & 1) * 16 + i16] = acc[i][rr];
}

template <int RK>
__global__ __launch_bounds__(512, 2) void stk_kb(StepArgs a0, StepArgs a1, const float* hk0, const float* hk1,
                                                 const float* Wk0, const float* Wih1k, const float* Whh1k, int t) {
  __shared__ float red[8 * 32 * 33];
  const StepArgs& a = blockIdx.z ? a1 : a0;
  const int H = a.H, B = a.B;
  const int j0 = blockIdx.x * UT, b0 = blockIdx.y * TB;
  const int bl = (threadIdx.x & 255) >> 3, u = threadIdx.x & 7;
  const int b = b0 + bl, j = j0 + u;
  const bool own = threadIdx.x < 256 && b < B;
  const int tt = blockIdx.z ? t - 1 : t;
  float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f;
  if (own) {
    const float* g = a.gx + (int64_t)b * a.gx_ldb + (int64_t)tt * a.gx_ldt;
    for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + j];
    cp = a.c[(int64_t)b * a.T * H + (int64_t)max(tt - 1, 0) * H + j];
  }
  const int rowB = blockIdx.x * 32;
  if (blockIdx.z == 0) {
    const float* pa[2] = {hk0 + b0 * 4, hk0 + b0 * 4};
    const float* pb[2] = {Wk0 + rowB * 4, Wk0 + rowB * 4};
    kb_core<RK, 1024 / 8 / RK>(red, pa, pb, H, 64, 4 * H);
  } else {
    const float* pa[2] = {hk0 + b0 * 4, hk1 + b0 * 4};
    const float* pb[2] = {Wih1k + rowB * 4, Whh1k + rowB * 4};
    kb_core<RK, 2048 / 8 / RK>(red, pa, pb, H, 64, 4 * H);
  }
  __syncthreads();
  if (!own) return;
  float pre[4];
  for (int q = 0; q < 4; ++q) {
    float vv = 0.f;
    for (int ww = 0; ww < 8; ++ww) vv += red[ww * 32 * 33 + bl * 33 + q * UT + u];
    pre[q] = vv;
  }
  const float i_ = avc_sigmoid(pre[0] + gxv[0]), f_ = avc_sigmoid(pre[1] + gxv[1]);
  const float g_ = tanhf(pre[2] + gxv[2]), o_ = avc_sigmoid(pre[3] + gxv[3]);
  const float cn = f_ * cp + i_ * g_;
  a.c[(int64_t)b * a.T * H + (int64_t)tt * H + j] = cn;
  a.h[(int64_t)b * a.h_ldb + (int64_t)tt * a.h_ldt + j] = o_ * tanhf(cn);
  if (a.gates) {
    float* gs = a.gates + ((int64_t)b * a.T + tt) * 4 * H;
    gs[0 * H + j] = i_; gs[1 * H + j] = f_; gs[2 * H + j] = g_; gs[3 * H + j] = o_;
  }
}

template <class F>
static float per_launch_us(int n, F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < n; ++i) f(i);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < n; ++i) f(i);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, ms * 1000.f / n);
  }
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(err)); exit(1); }
  return best;
}

static double maxdiff(const float* a, const float* b, size_t n, double* mx) {
  std::vector<float> x(n), y(n);
  (void)hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost);
  double md = 0, m = 0;
  for (size_t i = 0; i < n; ++i) { md = fmax(md, fabs((double)x[i] - y[i])); m = fmax(m, fabs((double)x[i])); }
  *mx = m;
  return md;
}

int main() {
  const int B = 64, T = 128;
  uint32_t st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) * (1.0f / 16777216.f)) * 2.f - 1.f; };
  for (int H : {1024, 512}) {
    const int64_t G4 = 4 * H;
    std::vector<float> hW(G4 * H), hgx((size_t)B * T * G4), hb(G4);
    for (auto& v : hW) v = rnd() / sqrtf((float)H);
    for (auto& v : hgx) v = rnd() * 0.5f;
    for (auto& v : hb) v = rnd() * 0.1f;
    float *W, *W2, *gx, *bias, *h[4], *c[4], *g[4], *P1, *P2;
    (void)hipMalloc(&W, G4 * H * 4);
    (void)hipMalloc(&W2, G4 * H * 4);
    (void)hipMalloc(&gx, hgx.size() * 4);
    (void)hipMalloc(&bias, G4 * 4);
    for (int i = 0; i < 4; ++i) {
      (void)hipMalloc(&h[i], (size_t)B * T * H * 4);
      (void)hipMalloc(&c[i], (size_t)B * T * H * 4);
      (void)hipMalloc(&g[i], (size_t)B * T * G4 * 4);
    }
    (void)hipMalloc(&P1, (size_t)8 * B * H * 4);
    (void)hipMalloc(&P2, (size_t)8 * B * H * 4);
    (void)hipMemcpy(W, hW.data(), G4 * H * 4, hipMemcpyHostToDevice);
    for (auto& v : hW) v = rnd() / sqrtf((float)H);
    (void)hipMemcpy(W2, hW.data(), G4 * H * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(gx, hgx.data(), hgx.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(bias, hb.data(), G4 * 4, hipMemcpyHostToDevice);
    const dim3 grid(H / UT, (B + TB - 1) / TB);
    auto sa = [&](int i) { return StepArgs{B, T, H, gx, T * G4, G4, W, h[i], (int64_t)T * H, H, c[i], g[i], nullptr}; };
    auto step_lds = [&](int s) {
      hipLaunchKernelGGL((lstm_fwd_step_kernel<0, 64, 8, 2>), grid, dim3(512), 0, 0, sa(0), s % T, (s % T) - 1);
    };
    printf("H=%d fwd step per launch (back-to-back): product %.2f us\n", H, per_launch_us(T, step_lds));
    // no recurrent product at all (tp = -1): prologue loads + epilogue + launch
    printf("H=%d fwd step without GEMM: product kernel %.2f us | empty %.2f us\n", H,
           per_launch_us(T, [&](int s) {
             hipLaunchKernelGGL((lstm_fwd_step_kernel<0, 64, 8, 2>), grid, dim3(512), 0, 0, sa(0), s % T, -1);
           }),
           per_launch_us(T, [&](int s) { hipLaunchKernelGGL(empty_kernel, grid, dim3(512), 0, 0, c[3], s); }));
    {
      float *hk, *Wk;
      (void)hipMalloc(&hk, (size_t)H * B * 4);
      (void)hipMalloc(&Wk, (size_t)G4 * H * 4);
      (void)hipMemset(hk, 0, (size_t)H * B * 4);
      (void)hipMemcpy(Wk, W, G4 * H * 4, hipMemcpyDeviceToDevice);
      auto kb = [&](int s) {
        if (H == 1024)
          hipLaunchKernelGGL(fwd_kb<2>, grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1);
        else
          hipLaunchKernelGGL(fwd_kb<1>, grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1);
      };
      printf("H=%d k-blocked direct (timing probe): %.2f us\n", H, per_launch_us(T, kb));
      if (H == 1024) {
        printf("H=%d k-blocked ablations: W-shared %.2f | h-shared %.2f | both %.2f us\n", H,
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<2, 1>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }),
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<2, 2>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }),
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<2, 3>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }));
        {
          const int nwg = grid.x * grid.y;
          unsigned long long* st;
          (void)hipMalloc(&st, (size_t)nwg * 8 * 6 * 8);
          for (int s = 0; s < 40; ++s)
            hipLaunchKernelGGL((fwd_kb<2, 8>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, 5, 4, st);
          (void)hipDeviceSynchronize();
          std::vector<unsigned long long> hs((size_t)nwg * 8 * 6);
          (void)hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost);
          unsigned long long t0 = ~0ull, tend = 0;
          for (int i = 0; i < nwg * 8; ++i) { t0 = std::min(t0, hs[i * 6]); tend = std::max(tend, hs[i * 6 + 4]); }
          for (int k = 0; k < 5; ++k) {
            std::vector<double> v;
            for (int i = 0; i < nwg * 8; ++i) v.push_back((hs[i * 6 + k] - t0) * 0.01);   // 100 MHz -> us
            std::sort(v.begin(), v.end());
            printf("  stamp %d (entry, loads issued, round0 MFMAs issued, round1 MFMAs issued, reduced): "
                   "min %.2f med %.2f max %.2f us\n", k, v[0], v[v.size() / 2], v.back());
          }
          (void)hipFree(st);
        }
        {
          float *hk1, *Wk2, *Wk3;
          (void)hipMalloc(&hk1, (size_t)H * B * 4);
          (void)hipMalloc(&Wk2, (size_t)G4 * H * 4);
          (void)hipMalloc(&Wk3, (size_t)G4 * H * 4);
          (void)hipMemset(hk1, 0, (size_t)H * B * 4);
          (void)hipMemcpy(Wk2, W, G4 * H * 4, hipMemcpyDeviceToDevice);
          (void)hipMemcpy(Wk3, W, G4 * H * 4, hipMemcpyDeviceToDevice);
          const dim3 g3(H / UT, (B + TB - 1) / TB, 2);
          const StepArgs l1 = sa(3);
          printf("H=%d stacked k-blocked direct (2 WG/CU): RK32 %.2f | RK16 %.2f us (product stacked LDS: %.2f us)\n", H,
                 per_launch_us(T, [&](int s) { hipLaunchKernelGGL(stk_kb<32>, g3, dim3(512), 0, 0, sa(2), l1, hk, hk1, Wk, Wk2, Wk3, 1 + s % (T - 1)); }),
                 per_launch_us(T, [&](int s) { hipLaunchKernelGGL(stk_kb<16>, g3, dim3(512), 0, 0, sa(2), l1, hk, hk1, Wk, Wk2, Wk3, 1 + s % (T - 1)); }),
                 per_launch_us(T + 1, [&](int s) {
                   const Stack2Args st2{sa(0), StepArgs{B, T, H, gx, 0, 0, W, h[3], (int64_t)T * H, H, c[3], g[3], gx}, W2};
                   hipLaunchKernelGGL((lstm2_fwd_step_kernel<64, 8, 2>), g3, dim3(512), 0, 0, st2, s % (T + 1)); }));
          (void)hipFree(hk1); (void)hipFree(Wk2); (void)hipFree(Wk3);
        }
        printf("H=%d k-blocked loads only: %.2f | both-shared loads only %.2f us\n", H,
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<2, 4>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }),
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<2, 7>), grid, dim3(512), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }));
        printf("H=%d k-blocked 16 waves: %.2f | both-shared %.2f us\n", H,
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<1, 0, 16>), grid, dim3(1024), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }),
               per_launch_us(T, [&](int s) { hipLaunchKernelGGL((fwd_kb<1, 3, 16>), grid, dim3(1024), 0, 0, sa(2), hk, B, Wk, (int)G4, s % T, (s % T) - 1); }));
      }
      (void)hipFree(hk); (void)hipFree(Wk);
    }
    printf("H=%d MFMA-only (direct core, operands in VGPRs, same MFMA count): %.2f us\n", H,
           per_launch_us(T, [&](int s) { hipLaunchKernelGGL(mfma_only, grid, dim3(512), 0, 0, c[3], H / DNW / 16, s); }));


    (void)hipFree(W); (void)hipFree(W2); (void)hipFree(gx); (void)hipFree(bias);
    for (int i = 0; i < 4; ++i) { (void)hipFree(h[i]); (void)hipFree(c[i]); (void)hipFree(g[i]); }
    (void)hipFree(P1); (void)hipFree(P2);
  }
  return 0;
}
