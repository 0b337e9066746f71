// Tile-configuration sweep for autovc_gemm_f32 on the Generator-step shapes (not part of
// the product).  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm_bench.hip -o tools/gemm_bench
#include "../autovc_amd/csrc/gemm.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cstdio>
#include <cstdlib>
#include <string>

struct Case { const char* name; int M, N, K, at, bt, aconv, bconv, C, splits; };

int main(int argc, char** argv) {
  const int only_case = argc > 2 ? atoi(argv[1]) : -1, only_cfg = argc > 2 ? atoi(argv[2]) : -1;
  const int T = 128;
  Case cases[] = {
      {"conv fwd 512->512", 8192, 512, 2560, 0, 0, 1, 0, 512, 1},
      {"conv fwd 336->512", 8192, 512, 1680, 0, 0, 1, 0, 336, 1},
      {"conv dX 512<-512", 8192, 512, 2560, 0, 1, 1, 0, 512, 1},
      {"conv dW s1", 512, 2560, 8192, 1, 1, 0, 1, 512, 1},
      {"conv dW s2", 512, 2560, 8192, 1, 1, 0, 1, 512, 2},
      {"conv dW s3", 512, 2560, 8192, 1, 1, 0, 1, 512, 3},
      {"conv dW s4", 512, 2560, 8192, 1, 1, 0, 1, 512, 4},
      {"lstm2 proj K512", 8192, 4096, 512, 0, 0, 0, 0, 0, 1},
      {"lstm2 proj K1024", 8192, 4096, 1024, 0, 0, 0, 0, 0, 1},
      {"lstm1 proj K320", 8192, 2048, 320, 0, 0, 0, 0, 0, 1},
      {"lstm2 dW_ih/hh s1", 4096, 1024, 8192, 1, 1, 0, 0, 0, 1},
      {"lstm2 dW_ih l0 s1", 4096, 512, 8192, 1, 1, 0, 0, 0, 1},
      {"lstm2 dW_ih l0 s2", 4096, 512, 8192, 1, 1, 0, 0, 0, 2},
      {"lstm2 dx l1", 8192, 1024, 4096, 0, 1, 0, 0, 0, 1},
      {"lstm2 dx l0", 8192, 512, 4096, 0, 1, 0, 0, 0, 1},
  };
  float *A, *B, *Cm, *ws;
  const size_t big = (size_t)8192 * 4096;
  (void)hipMalloc(&A, big * 4);
  (void)hipMalloc(&B, big * 4);
  (void)hipMalloc(&Cm, big * 4);
  (void)hipMalloc(&ws, 4 * big * 4);
  {  // random operands (MFMA clocks differ on zeros)
    float* h = (float*)malloc(big * 4);
    for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    (void)hipMemcpy(A, h, big * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(B, h, big * 4, hipMemcpyHostToDevice);
    free(h);
  }
  if (argc > 1 && std::string(argv[1]) == "wino") {   // the Winograd F(4,5) batched GEMMs (8 per conv)
    struct W { const char* name; int M, N, K; };
    const W ws[] = {{"wino 512->512", 2048, 512, 512}, {"wino 336->512", 2048, 512, 336},
                    {"wino 512->80", 2048, 80, 512}, {"wino dX 512<-512", 2048, 512, 512}};
    hipEvent_t a0, a1;
    (void)hipEventCreate(&a0);
    (void)hipEventCreate(&a1);
    for (const W& w : ws) {
      printf("%-18s 8 x M=%5d N=%5d K=%5d :", w.name, w.M, w.N, w.K);
      for (int cfg = 0; cfg < 12; ++cfg) {
        g_force_cfg = cfg;
        auto run = [&]() {
          return autovc_gemm_batched_f32(8, w.M, w.N, w.K, A, w.K, (int64_t)w.M * w.K, 0, B, w.K, (int64_t)w.N * w.K, 0,
                                         Cm, w.N, (int64_t)w.M * w.N, 0, 0);
        };
        if (run() != 0) { printf(" cfg%d ERR", cfg); continue; }
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a0, 0);
        for (int i = 0; i < 20; ++i) run();
        (void)hipEventRecord(a1, 0);
        (void)hipEventSynchronize(a1);
        float ms;
        (void)hipEventElapsedTime(&ms, a0, a1);
        const double us = ms * 50.0;
        printf("  cfg%d %6.1fus %5.1fTF", cfg, us, 2.0 * 8 * w.M * w.N * w.K / (us * 1e-6) / 1e12);
      }
      printf("\n");
    }
    return 0;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int ci = -1;
  for (const Case& c : cases) {
    ++ci;
    if (only_case >= 0 && ci != only_case) continue;
    printf("%-20s M=%5d N=%5d K=%5d s=%d :", c.name, c.M, c.N, c.K, c.splits);
    for (int cfg = 2; cfg < 12; ++cfg) {
      if (cfg == 5 || cfg == 7) continue;
      if (only_cfg >= 0 && cfg != only_cfg) continue;
      g_force_cfg = cfg;
      const int lda = c.at ? c.M : (c.aconv ? c.C : c.K);
      const int ldb = c.bt ? (c.bconv ? c.C : c.N) : c.K;
      auto run = [&]() {
        return autovc_gemm_f32(c.M, c.N, c.K, A, lda, c.at, c.aconv ? T : 0, c.C, -2, B, ldb, c.bt,
                               c.bconv ? T : 0, c.C, -2, Cm, c.N, nullptr, nullptr, 0, c.splits, ws, 0);
      };
      if (run() != 0) { printf(" cfg%d ERR(%s)", cfg, autovc_last_error()); continue; }
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) run();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      printf("  cfg%d %7.1fus %6.1fTF", cfg, us, 2.0 * c.M * c.N * c.K / (us * 1e-6) / 1e12);
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) { printf("\nHIP error %s\n", hipGetErrorString(err)); return 1; }
    }
    printf("\n");
  }
  return 0;
}
