// Launch-chain microbenchmark (not part of the product): what a chain of dependent kernel
// launches costs per launch on MI355X, for kernels shaped like the WaveNet step kernels
// (256 workgroups; every workgroup reads data the previous launch wrote).
//   hipcc -O3 --offload-arch=gfx950 tools/chain_ubench.hip -o tools/build/chain_ubench
//   tools/build/chain_ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

struct Args { const float* in; float* out; const float* w; const int* ctr; int fresh_floats; int w_floats; int use_ctr; };

// every lane reads `fresh_floats` floats (f4 granules) of the previous launch's output
// (the same region for every workgroup), `w_floats` floats of a stable weight buffer (a
// different slice per workgroup), reduces, and one lane per workgroup writes 4 floats.
template <int NT>
__device__ __forceinline__ void chain_body(const Args& a) {
  const int lane = threadIdx.x;
  int off = 0;
  if (a.use_ctr) off = a.ctr[0] & 1;
  float s = 0.f;
  for (int k = lane * 4; k < a.fresh_floats; k += NT * 4) {
    const f4 v = *reinterpret_cast<const f4*>(a.in + k + off * 0);
    s += v[0] + v[1] + v[2] + v[3];
  }
  const float* wb = a.w + (size_t)blockIdx.x * a.w_floats;
  for (int k = lane * 4; k < a.w_floats; k += NT * 4) {
    const f4 v = *reinterpret_cast<const f4*>(wb + k);
    s += v[0] * v[1] + v[2] * v[3];
  }
  __shared__ float red[NT / 64];
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if ((lane & 63) == 0) red[lane >> 6] = s;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  t = t * 1e-3f + 1.0f;
  // this workgroup's slice of the region the next launch reads
  const int per = a.fresh_floats / 256 > 4 ? a.fresh_floats / 256 : 4;
  for (int k = lane * 4; k < per; k += NT * 4)
    *reinterpret_cast<f4*>(a.out + (size_t)blockIdx.x * per + k) = f4{t, t, t, t};
}

template <int NT>
__global__ __launch_bounds__(NT) void chain_kernel(Args a) { chain_body<NT>(a); }

__global__ void empty_kernel(Args) {}
// a second symbol with identical code: does switching kernels cost more than repeating one?
template <int NT>
__global__ __launch_bounds__(NT) void chain_kernel_b(Args a) { chain_body<NT>(a); }

template <int NT>
float run(int variant, int fresh, int wfl, int use_ctr, float* b0, float* b1, const float* w, const int* ctr,
          hipStream_t st) {
  const int L = 26, S = 64;
  hipGraph_t g;
  hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed);
  for (int s = 0; s < S; ++s)
    for (int l = 0; l < L; ++l) {
      Args a{(l & 1) ? b1 : b0, (l & 1) ? b0 : b1, w, ctr, fresh, wfl, use_ctr};
      if (variant == 0) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(NT), 0, st, a);
      else if (variant == 2 && (l & 1)) hipLaunchKernelGGL(chain_kernel_b<NT>, dim3(256), dim3(NT), 0, st, a);
      else if (variant == 3 && (l & 1)) hipLaunchKernelGGL(chain_kernel<128>, dim3(128), dim3(128), 0, st, a);
      else hipLaunchKernelGGL(chain_kernel<NT>, dim3(256), dim3(NT), 0, st, a);
    }
  hipStreamEndCapture(st, &g);
  hipGraphExec_t ex;
  hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  hipGraphLaunch(ex, st);
  hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, st);
    hipGraphLaunch(ex, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipGraphExecDestroy(ex); hipGraphDestroy(g);
  return best * 1e3f / (L * S);
}

int main() {
  float *b0, *b1, *w; int* ctr;
  CK(hipMalloc(&b0, 1 << 22)); CK(hipMalloc(&b1, 1 << 22)); CK(hipMalloc(&w, 256ull << 20)); CK(hipMalloc(&ctr, 256));
  CK(hipMemset(b0, 0, 1 << 22)); CK(hipMemset(b1, 0, 1 << 22)); CK(hipMemset(w, 0, 256ull << 20)); CK(hipMemset(ctr, 0, 256));
  hipStream_t st; CK(hipStreamCreate(&st));
  printf("us per launch, 256 workgroups, chains of 26 x 64 launches in one graph\n");
  printf("empty 256 thr      : %6.2f\n", run<256>(0, 0, 0, 0, b0, b1, w, ctr, st));
  printf("empty 576 thr      : %6.2f\n", run<576>(0, 0, 0, 0, b0, b1, w, ctr, st));
  printf("alternating symbols (576 thr, fresh 4096 B, weights 16384 B): same %6.2f  two symbols %6.2f  "
         "every other launch 128x128 threads %6.2f\n",
         run<576>(1, 1024, 4096, 0, b0, b1, w, ctr, st), run<576>(2, 1024, 4096, 0, b0, b1, w, ctr, st),
         run<576>(3, 1024, 4096, 0, b0, b1, w, ctr, st));
  if (getenv("CHAIN_ALT_ONLY")) return 0;
  const int fr[] = {0, 16, 1024, 4096, 8192, 16384};
  const int wf[] = {0, 4096, 8192};
  for (int nt = 0; nt < 2; ++nt)
    for (int c = 0; c < 2; ++c)
      for (int f : fr)
        for (int ww : wf) {
          float us = nt == 0 ? run<256>(1, f, ww, c, b0, b1, w, ctr, st) : run<576>(1, f, ww, c, b0, b1, w, ctr, st);
          printf("thr %3d ctr %d fresh %6d B  weights %6d B : %6.2f\n", nt ? 576 : 256, c, f * 4, ww * 4, us);
        }
  return 0;
}
