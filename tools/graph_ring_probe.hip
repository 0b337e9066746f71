// Graph replay probe (diagnostic, not product): does the HIP runtime execute every node of a
// captured graph exactly once per replay when many replays are queued without a host sync?
//
// A graph of `n` tiny kernel nodes is captured on one stream; node i adds 1 to cnt[i] (one
// vector atomic per launch).  After `r` back-to-back hipGraphLaunch calls and one
// hipStreamSynchronize, every cnt[i] must equal r.  Shapes:
//   forked = 0: a linear chain (one stream, one dependency list);
//   forked = 1: the same chain plus one node on a second stream, forked at the start and joined
//               at the end (the step graph's weight-gradient side branch has this shape).
// probe_run returns the number of counters that differ from r (0 = correct) or a negative
// HIP status; the first mismatch is reported through *first_bad / *first_val.
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ void tick_kernel(int* cnt, int i) {
  if (threadIdx.x == 0) atomicAdd(cnt + i, 1);
}

#define PCHK(x)                           \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return -(int)e_; \
  } while (0)

extern "C" int probe_run(int n, int r, int forked, int* first_bad, int* first_val, double* ms_per_replay) {
  int* cnt = nullptr;
  hipStream_t s, s2;
  hipEvent_t fork_ev, join_ev, t0, t1;
  PCHK(hipMalloc(&cnt, sizeof(int) * (n + 1)));
  PCHK(hipMemset(cnt, 0, sizeof(int) * (n + 1)));
  PCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  PCHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  PCHK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
  PCHK(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
  PCHK(hipEventCreate(&t0));
  PCHK(hipEventCreate(&t1));
  PCHK(hipDeviceSynchronize());

  hipGraph_t g;
  hipGraphExec_t ge;
  PCHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  if (forked) {
    PCHK(hipEventRecord(fork_ev, s));
    PCHK(hipStreamWaitEvent(s2, fork_ev, 0));
    hipLaunchKernelGGL(tick_kernel, dim3(1), dim3(64), 0, s2, cnt, n);   // the side node
    PCHK(hipGetLastError());
  }
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(tick_kernel, dim3(1), dim3(64), 0, s, cnt, i);
  PCHK(hipGetLastError());
  if (forked) {
    PCHK(hipEventRecord(join_ev, s2));
    PCHK(hipStreamWaitEvent(s, join_ev, 0));
  }
  PCHK(hipStreamEndCapture(s, &g));
  PCHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  PCHK(hipEventRecord(t0, s));
  for (int k = 0; k < r; ++k) PCHK(hipGraphLaunch(ge, s));
  PCHK(hipEventRecord(t1, s));
  PCHK(hipStreamSynchronize(s));
  float ms = 0.f;
  PCHK(hipEventElapsedTime(&ms, t0, t1));
  *ms_per_replay = r > 0 ? ms / r : 0.0;

  int* host = new int[n + 1];
  PCHK(hipMemcpy(host, cnt, sizeof(int) * (n + 1), hipMemcpyDeviceToHost));
  int bad = 0;
  *first_bad = -1;
  *first_val = 0;
  for (int i = 0; i < n + (forked ? 1 : 0); ++i)
    if (host[i] != r) {
      if (bad == 0) {
        *first_bad = i;
        *first_val = host[i];
      }
      ++bad;
    }
  delete[] host;
  PCHK(hipGraphExecDestroy(ge));
  PCHK(hipGraphDestroy(g));
  PCHK(hipEventDestroy(fork_ev));
  PCHK(hipEventDestroy(join_ev));
  PCHK(hipEventDestroy(t0));
  PCHK(hipEventDestroy(t1));
  PCHK(hipStreamDestroy(s));
  PCHK(hipStreamDestroy(s2));
  PCHK(hipFree(cnt));
  return bad;
}
