// Shared helpers for the autovc_amd HIP library (gfx950 / MI355X only).
//
// Error model (DESIGN.md "Boundary"): every extern "C" entry point returns an
// int status (0 = ok, <0 = error) and records a message retrievable through
// autovc_last_error() (thread-local).  No C++ exception crosses the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

namespace avc {

void set_error(const char* fmt, ...);

// Zero `bytes` (a multiple of 4) at `p` on `stream` with a kernel (elementwise.hip).  Used
// instead of hipMemsetAsync on every path a step graph captures: a captured memset becomes
// a memset node, and replays of a single-stream (linear) step graph holding memset nodes
// faulted the GPU on this runtime; kernel nodes are the only
// node kind the graphs then contain.
hipError_t zero_async(void* p, size_t bytes, hipStream_t stream);

constexpr int kOk = 0;
constexpr int kErrArg = -1;     // bad shape / pointer / alignment
constexpr int kErrLaunch = -2;  // hip launch or runtime failure

}  // namespace avc

#define AVC_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      avc::set_error(__VA_ARGS__);               \
      return avc::kErrArg;                       \
    }                                            \
  } while (0)

#define AVC_CHECK_LAUNCH(name)                                              \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      avc::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return avc::kErrLaunch;                                               \
    }                                                                       \
  } while (0)

#define AVC_HIP(call, name)                                                 \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) {                                                 \
      avc::set_error("%s: %s", name, hipGetErrorString(e_));                \
      return avc::kErrLaunch;                                               \
    }                                                                       \
  } while (0)

#define AVC_ALIGNED16(p) ((reinterpret_cast<uintptr_t>(p) & 15u) == 0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Accurate (ocml) expf/tanhf: the LSTM parity bar is 1e-4 rel vs torch CPU.
__device__ __forceinline__ float avc_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }

// Short-latency forms for the latency-bound small-H recurrence (encoder BLSTM: 128 dependent
// steps per launch, where ocml's branchy tanhf and IEEE division dominated a step):
// v_exp_f32 + v_rcp_f32, a few ulp; tanh via 1 - 2 / (e^{2x} + 1) (absolute error ~1e-7 near
// 0, exact limits +-1).
__device__ __forceinline__ float avc_sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float avc_tanh_fast(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f);
}

// x + x[lane ^ M] inside each quad of lanes (M = 1 or 2): DPP quad_perm, VALU only
template <int M>
__device__ __forceinline__ float avc_quad_xor_add(float x) {
  static_assert(M == 1 || M == 2, "quad lanes");
  constexpr int ctrl = M == 1 ? 0xB1 : 0x4E;   // quad_perm [1,0,3,2] / [2,3,0,1]
  return x + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), ctrl, 0xF, 0xF, false));
}
