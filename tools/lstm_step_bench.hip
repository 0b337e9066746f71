// Ablation / tuning microbenchmark of the large-H LSTM step kernels (not part of the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lstm_step_bench.hip -o tools/lstm_step_bench
// Times each step launch with hipExtLaunchKernelGGL dispatch events (these include a
// ~4 us dispatch floor on MI355X: compare variants, not absolute numbers; rocprofv3 gives
// the kernel-only durations).
//
// Record (round 1, H=1024, B=64): LDS-DMA ring (global_load_lds, 7 chunks in flight)
// 13.3 us and unchanged when all operands were L2-resident -> issue-bound at ~25 GB/s/CU;
// direct global->VGPR fragments 16-19 us; register-staged LDS tiles 8.8 us.
#include "../autovc_amd/csrc/lstm.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void empty_kernel(StepArgs a, int t, int tp) {
  if (t == -5) a.c[0] = 1.f;
}

template <class F>
static float timeit(F launch, int T, int reps) {
  std::vector<hipEvent_t> ev(2 * T);
  for (auto& e : ev) (void)hipEventCreate(&e);
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    for (int s = 0; s < T; ++s) launch(s, ev[2 * s], ev[2 * s + 1]);
    (void)hipDeviceSynchronize();
    double tot = 0;
    for (int s = 1; s < T; ++s) {
      float ms;
      (void)hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]);
      tot += ms;
    }
    best = std::min(best, (float)(tot / (T - 1) * 1000.0));
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    printf("HIP error: %s\n", hipGetErrorString(err));
    exit(1);
  }
  return best;
}

template <int ABL, int K, int NW, int D>
static float fwd(StepArgs a, int T) {
  const dim3 grid(a.H / UT, (a.B + TB - 1) / TB);
  return timeit([&](int s, hipEvent_t e0, hipEvent_t e1) {
    hipExtLaunchKernelGGL(lstm_fwd_step_kernel<ABL, K, NW, D>, grid, dim3(64 * NW), 0, 0, e0, e1, 0, a, s, s - 1);
  }, T, 3);
}

template <int K, int NW, int D>
static float rec(int B, int T, int H, const float* dG, const float* WT, float* P, int S) {
  const dim3 grid(H / TN, (B + TB - 1) / TB, S);
  return timeit([&](int s, hipEvent_t e0, hipEvent_t e1) {
    hipExtLaunchKernelGGL(lstm_bwd_rec_kernel<K, NW, D>, grid, dim3(64 * NW), 0, 0, e0, e1, 0, B, T, H, dG, s, WT, P);
  }, T, 3);
}

int main() {
  const int B = 64, T = 128;
  for (int H : {1024, 512}) {
    float *gx, *W, *h, *c, *g, *P;
    (void)hipMalloc(&gx, (size_t)B * T * 4 * H * 4);
    (void)hipMalloc(&W, (size_t)4 * H * H * 4);
    (void)hipMalloc(&h, (size_t)B * T * H * 4);
    (void)hipMalloc(&c, (size_t)B * T * H * 4);
    (void)hipMalloc(&g, (size_t)B * T * 4 * H * 4);
    (void)hipMalloc(&P, (size_t)8 * B * H * 4);
    (void)hipMemset(gx, 0, (size_t)B * T * 4 * H * 4);
    (void)hipMemset(W, 0, (size_t)4 * H * H * 4);
    (void)hipMemset(h, 0, (size_t)B * T * H * 4);
    (void)hipMemset(g, 0, (size_t)B * T * 4 * H * 4);
    StepArgs a{B, T, H, gx, (int64_t)T * 4 * H, 4 * H, W, h, (int64_t)T * H, H, c, g};
    const dim3 grid(H / UT, (B + TB - 1) / TB);
    printf("H=%d empty %.2f us\n", H, timeit([&](int s, hipEvent_t e0, hipEvent_t e1) {
      hipExtLaunchKernelGGL(empty_kernel, grid, dim3(256), 0, 0, e0, e1, 0, a, s, s - 1); }, T, 3));
    printf("H=%d fwd k64w8d1 %.2f | k64w8d2 %.2f | k64w8d3 %.2f | k64w8d4 %.2f | k128w8d1 %.2f | k128w8d2 %.2f | k128w8d3 %.2f | k128w4d2 %.2f\n", H,
           fwd<0, 64, 8, 1>(a, T), fwd<0, 64, 8, 2>(a, T), fwd<0, 64, 8, 3>(a, T), fwd<0, 64, 8, 4>(a, T),
           fwd<0, 128, 8, 1>(a, T), fwd<0, 128, 8, 2>(a, T), fwd<0, 128, 8, 3>(a, T), fwd<0, 128, 4, 2>(a, T));
    printf("H=%d fwd default ablations: full %.2f | W-shared %.2f | h-shared %.2f | both %.2f\n", H,
           fwd<0, KCH, NWV, DPF>(a, T), fwd<1, KCH, NWV, DPF>(a, T), fwd<2, KCH, NWV, DPF>(a, T), fwd<3, KCH, NWV, DPF>(a, T));
    for (int S : {4, 2}) {
      if ((4 * H / S) % 256) continue;
      printf("H=%d rec S=%d k64w8d1 %.2f | k64w8d2 %.2f | k64w8d3 %.2f | k128w8d1 %.2f | k128w8d2 %.2f | k128w8d3 %.2f\n", H, S,
             rec<64, 8, 1>(B, T, H, g, W, P, S), rec<64, 8, 2>(B, T, H, g, W, P, S), rec<64, 8, 3>(B, T, H, g, W, P, S),
             rec<128, 8, 1>(B, T, H, g, W, P, S), rec<128, 8, 2>(B, T, H, g, W, P, S), rec<128, 8, 3>(B, T, H, g, W, P, S));
    }
    (void)hipFree(gx); (void)hipFree(W); (void)hipFree(h); (void)hipFree(c); (void)hipFree(g); (void)hipFree(P);
  }
  return 0;
}
