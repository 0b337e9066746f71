// Layout probe for v_mfma_f32_4x4x1_16b_f32 (tools only): A lane l = l + 1, B lane l =
// 1000 (l + 1); prints, for lanes 0..7, the 4 result registers, so D[i][j] of block b
// = A(lane 4b + i) * B(lane 4b + j) identifies which (i, j) each (lane, register) holds.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* o) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1000.f * (l + 1), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) o[l * 4 + r] = c[r];
}
int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  probe<<<1, 64>>>(d);
  float h[256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 8; ++l) {
    printf("lane %d:", l);
    for (int r = 0; r < 4; ++r) {
      int la = -1, lb = -1;
      for (int x = 0; x < 64; ++x)
        for (int y = 0; y < 64; ++y)
          if ((float)(x + 1) * 1000.f * (float)(y + 1) == h[l * 4 + r]) { la = x; lb = y; }
      printf("  r%d = A[lane %d] * B[lane %d]", r, la, lb);
    }
    printf("\n");
  }
  return 0;
}
