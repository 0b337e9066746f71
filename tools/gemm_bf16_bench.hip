// Tile-configuration sweep for autovc_gemm_bf16_f32 on the bf16 Generator-step shapes (not
// part of the product): every case at every (config, split) pair, each checked against the
// fp32 GEMM on bf16-exact operands (differences are summation order only).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm_bf16_bench.hip -o tools/build/gemm_bf16_bench
#include "../autovc_amd/csrc/gemm.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Case { const char* name; int M, N, K, at, bt, aconv, bconv, C; };

int main(int argc, char** argv) {
  const int only_case = argc > 1 ? atoi(argv[1]) : -1;
  const int T = 128;
  Case cases[] = {
      {"conv fwd 512->512", 8192, 512, 2560, 0, 0, 1, 0, 512},
      {"conv dX 512<-512", 8192, 512, 2560, 0, 1, 1, 0, 512},
      {"conv dW", 512, 2560, 8192, 1, 1, 0, 1, 512},
      {"lstm dW 4096x1024", 4096, 1024, 8192, 1, 1, 0, 0, 0},
      {"lstm proj K1024", 8192, 4096, 1024, 0, 0, 0, 0, 0},
      {"lstm dx 8192x1024", 8192, 1024, 4096, 0, 1, 0, 0, 0},
  };
  struct Run { int cfg, splits; };
  std::vector<Run> runs = {{-1, 0}, {0, 1}, {0, 2}, {0, 4}, {2, 1}, {2, 2}, {2, 4}, {4, 2}, {4, 4}};
  float *A, *B, *Cm, *Cr, *ws;
  const size_t big = (size_t)8192 * 4096;
  (void)hipMalloc(&A, big * 4);
  (void)hipMalloc(&B, big * 4);
  (void)hipMalloc(&Cm, big * 4);
  (void)hipMalloc(&Cr, big * 4);
  (void)hipMalloc(&ws, 4 * big * 4);
  {
    float* h = (float*)malloc(big * 4);
    // multiples of 1/256 in [-0.5, 0.5): exact in bf16, so the bf16 GEMM equals the fp32 one
    // up to summation order
    for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 256) / 256.f - 0.5f;
    (void)hipMemcpy(A, h, big * 4, hipMemcpyHostToDevice);
    for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 40503u + 17) % 253) / 256.f - 0.5f;
    (void)hipMemcpy(B, h, big * 4, hipMemcpyHostToDevice);
    free(h);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int ci = -1;
  for (const Case& c : cases) {
    ++ci;
    if (only_case >= 0 && ci != only_case) continue;
    const int lda = c.at ? c.M : (c.aconv ? c.C : c.K);
    const int ldb = c.bt ? (c.bconv ? c.C : c.N) : c.K;
    const size_t nC = (size_t)c.M * c.N;
    std::vector<float> ref(nC), got(nC);
    printf("%-20s M=%5d N=%5d K=%5d\n", c.name, c.M, c.N, c.K);
    for (size_t ri = 0; ri < runs.size(); ++ri) {
      g_force_cfg_bf16 = runs[ri].cfg;
      g_force_splits_bf16 = runs[ri].splits;
      float* out = ri == 0 ? Cr : Cm;
      auto run = [&]() {
        if (ri == 0)   // reference: the exact fp32 GEMM
          return autovc_gemm_f32(c.M, c.N, c.K, A, lda, c.at, c.aconv ? T : 0, c.C, -2, B, ldb, c.bt,
                                 c.bconv ? T : 0, c.C, -2, out, c.N, nullptr, nullptr, 0, 4, ws, 0);
        return autovc_gemm_bf16_f32(c.M, c.N, c.K, A, lda, c.at, c.aconv ? T : 0, c.C, -2, B, ldb, c.bt,
                                    c.bconv ? T : 0, c.C, -2, out, c.N, nullptr, nullptr, 0, 1, ws, 0);
      };
      if (run() != 0) { printf("   cfg%d s%d ERR(%s)\n", runs[ri].cfg, runs[ri].splits, autovc_last_error()); continue; }
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) run();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) { printf("\nHIP error %s\n", hipGetErrorString(err)); return 1; }
      double maxerr = 0, maxref = 0;
      if (ri == 0) {
        (void)hipMemcpy(ref.data(), Cr, nC * 4, hipMemcpyDeviceToHost);
      } else {
        (void)hipMemcpy(got.data(), Cm, nC * 4, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < nC; ++i) {
          maxerr = std::max(maxerr, (double)std::fabs(got[i] - ref[i]));
          maxref = std::max(maxref, (double)std::fabs(ref[i]));
        }
      }
      printf("   cfg%d s%d %8.1f us %7.1f TF  rel err vs fp32 %.2e\n", runs[ri].cfg, runs[ri].splits, us,
             2.0 * c.M * c.N * c.K / (us * 1e-6) / 1e12, maxref > 0 ? maxerr / maxref : 0.0);
      fflush(stdout);
    }
  }
  return 0;
}
