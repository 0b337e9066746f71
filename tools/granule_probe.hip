// Probe of the tagged-granule all-gather (tools only, not part of the library): 256
// workgroups (one per CU), generation g = 1..NG; in generation g every workgroup's wave 0
// polls the 256 granules of generation g-1 (lane o: granules o, o+64, o+128, o+192 of each of
// NB utterance copies: 4 NB loads in flight per poll), then publishes its own granules of
// generation g with ONE 16-byte write-through (sc1) store each {me, me, me, g}.  Variants: the
// load that polls the tag word.  Reports us per generation, or the first wait that timed out.
//   hipcc -O3 --offload-arch=gfx950 tools/granule_probe.hip -o tools/pbin/granule_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st16(float* base, int off, i32x4 w) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (uint32_t)off * 4u, 0, 16);
}

// the tag (4th word) of granule gi: MODE 0 16-B buffer sc1 load; 1 8-B atomic (relaxed, agent)
// load of words 2-3; 2 4-B atomic load of word 3; 3 8-B buffer sc1 load of words 2-3; 4 4-B
// buffer sc1 load of word 3
template <int MODE>
__device__ __forceinline__ int tag_load(const float* base, int gi) {
  if constexpr (MODE == 0) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff,
                                                                       0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)gi * 16u, 0, 16)[3];
  } else if constexpr (MODE == 1) {
    return (int)(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(base + gi * 4 + 2), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) >> 32);
  } else if constexpr (MODE == 2) {
    return __hip_atomic_load(reinterpret_cast<const int*>(base + gi * 4 + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == 3) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff,
                                                                       0x00020000);
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(i32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)gi * 16u + 8u, 0, 16))[1];
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff,
                                                                       0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)gi * 16u + 12u, 0, 16);
  }
}

template <int MODE, int NB>
__global__ __launch_bounds__(1024, 1) void probe(float* g, int NG, int* err, int* diag, long long ticks) {
  extern __shared__ int s_pad[];              // 100 KB dynamic: one workgroup per CU
  if (threadIdx.x == 1023) s_pad[0] = 0;
  if (threadIdx.x >= 64) return;              // wave 0 only
  const int o = threadIdx.x;
  const int me = blockIdx.x;
  for (int gen = 1; gen <= NG; ++gen) {
    if (gen > 1) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const float* base = g + (size_t)((gen - 1) & 1) * 8 * 256 * 4;
      while (true) {
        int tg[4 * NB];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int b = 0; b < NB; ++b) tg[q * NB + b] = tag_load<MODE>(base + b * 256 * 4, q * 64 + o);
        int bad = 0;
#pragma unroll
        for (int k = 0; k < 4 * NB; ++k) bad |= tg[k] != gen - 1;
        if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) break;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)ticks) {
          if (atomicCAS(err, 0, 1) == 0) { diag[0] = gen; diag[1] = me; }
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (o < NB) {
      const i32x4 w = {me, me, me, gen};
      st16(g + ((size_t)(gen & 1) * 8 + o) * 256 * 4, me * 4, w);
    }
  }
}

template <int MODE, int NB>
void run(float* g, int* err, int* diag, int NG) {
  const int lds = 100 * 1024;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(probe<MODE, NB>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds);
  (void)hipMemset(g, 0, 2 * 8 * 256 * 16);
  (void)hipMemset(err, 0, 64);
  (void)hipMemset(diag, 0, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((probe<MODE, NB>), dim3(256), dim3(1024), lds, 0, g, NG, err, diag, 20000000LL);
  const hipError_t le = hipGetLastError();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  int h_err = 0, h_diag[2] = {0, 0};
  (void)hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(h_diag, diag, 8, hipMemcpyDeviceToHost);
  static const char* names[] = {"16-B buffer sc1", "8-B atomic", "4-B atomic", "8-B buffer sc1", "4-B buffer sc1"};
  printf("tag load %-16s NB=%d: %s", names[MODE], NB, le != hipSuccess ? "LAUNCH FAILED" : h_err ? "TIMEOUT" : "ok");
  if (h_err) printf(" (gen %d, wg %d)", h_diag[0], h_diag[1]);
  else printf(" %.3f us per generation", ms * 1e3 / NG);
  printf("\n");
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int NG = argc > 1 ? atoi(argv[1]) : 20000;
  float* g;
  int *err, *diag;
  (void)hipMalloc(&g, 2 * 8 * 256 * 16);
  (void)hipMalloc(&err, 64);
  (void)hipMalloc(&diag, 64);
  run<1, 1>(g, err, diag, NG); run<1, 8>(g, err, diag, NG);
  run<2, 1>(g, err, diag, NG); run<2, 8>(g, err, diag, NG);
  run<3, 1>(g, err, diag, NG); run<3, 8>(g, err, diag, NG);
  run<4, 1>(g, err, diag, NG); run<4, 8>(g, err, diag, NG);
  run<0, 1>(g, err, diag, NG);
  return 0;
}
