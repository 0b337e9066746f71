// Placement probe (tools only): which XCD each workgroup of a launch runs on, for a chain of
// back-to-back launches on one stream — the recurrence launches' shape (768 workgroups of 512
// threads) and a few others.  Prints, per launch, whether block b's XCD is (b + off) % 8 for
// one offset (exact round-robin), and that offset, so that cross-launch reuse of a per-XCD L2
// can be judged.   hipcc --offload-arch=gfx950 -O2 tools/xcd_probe.hip -o /tmp/xcd_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void probe(int* out, int spin) {
  __shared__ float pad[8192];   // 32 KB: a few workgroups per CU, like the recurrence kernels
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = x;
  float v = threadIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 0.999f + pad[(threadIdx.x + i) & 8191];
  if (v == 12345.f) out[blockIdx.x] = -1;
}

int main() {
  const int shapes[][2] = {{768, 512}, {256, 512}, {1024, 256}, {100, 256}};
  for (auto& s : shapes) {
    const int nb = s[0], nt = s[1], L = 12;
    int* d;
    hipMalloc(&d, sizeof(int) * nb * L);
    for (int l = 0; l < L; ++l) hipLaunchKernelGGL(probe, dim3(nb), dim3(nt), 0, 0, d + l * nb, 200);
    hipDeviceSynchronize();
    std::vector<int> h(nb * L);
    hipMemcpy(h.data(), d, sizeof(int) * nb * L, hipMemcpyDeviceToHost);
    printf("grid %d x %d threads:\n", nb, nt);
    for (int l = 0; l < L; ++l) {
      const int off = ((h[l * nb] - 0) % 8 + 8) % 8;
      int bad = 0;
      int cnt[8] = {};
      for (int b = 0; b < nb; ++b) {
        if (h[l * nb + b] != (b + off) % 8) ++bad;
        cnt[h[l * nb + b] & 7]++;
      }
      printf("  launch %2d: block 0 on XCD %d, %d blocks off the round-robin, per-XCD counts", l, off, bad);
      for (int x = 0; x < 8; ++x) printf(" %d", cnt[x]);
      printf("\n");
    }
    hipFree(d);
  }
  return 0;
}
