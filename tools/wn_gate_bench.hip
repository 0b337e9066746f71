// WaveNet step-kernel microbenchmark (not part of the product): times the production gate /
// resid / head kernels and ablated copies of the gate kernel to find what bounds a launch.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/wn_gate_bench.hip -o tools/wn_gate_bench
#include "../autovc_amd/csrc/wavenet.hip"
#include "../autovc_amd/csrc/capi.cpp"

#include <cstdio>
#include <vector>

namespace {

// MODE bits: 1 = skip pre loads, 2 = skip ring loads, 4 = skip weight loads, 8 = t from argument,
// 16 = no final store, 32 = no cross-wave LDS reduction, 64 = no tanh/sigmoid
template <int NW, int MODE>
__global__ __launch_bounds__(64 * NW) void gate_variant(WnArgs a, int layer, int slot, int targ) {
  __shared__ float s_red[NW][2 * kBT];
  const int t = (MODE & 8) ? targ : read_step(a, slot, 0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b0 = blockIdx.y * kBT;
  const int nb = min(kBT, a.B - b0);
  const int H = a.G / 2;
  const int o = blockIdx.x;
  const int KR = a.K * a.R;
  const float* WA = layer_base(a, layer);
  const float* wa = WA + (int64_t)o * KR;
  const float* wb = WA + (int64_t)(o + H) * KR;
  const int d = 1 << (layer % a.lps);
  float acc[2 * kBT];
#pragma unroll
  for (int j = 0; j < 2 * kBT; ++j) acc[j] = 0.f;
  for (int c = wave; c * 256 < KR; c += NW) {
    const int kc = c * 256;
    const int tap = kc / a.R;
    const int tau = t - (a.K - 1 - tap) * d;
    if (tau < 0) continue;
    const int k = kc + lane * 4;
    const int i = k - tap * a.R;
    f32x4 va = {1.f, 1.f, 1.f, 1.f}, vb = va;
    if (!(MODE & 4)) { va = ld4(wa + k); vb = ld4(wb + k); }
    f32x4 x[kBT];
    const float* xr = a.ring + (((int64_t)layer * a.RING + (tau & (a.RING - 1))) * a.B + b0) * a.R + i;
#pragma unroll
    for (int b = 0; b < kBT; ++b) {
      if (MODE & 2) x[b] = f32x4{(float)b, 1.f, 2.f, (float)lane};
      else x[b] = ld4(xr + (int64_t)(b < nb ? b : 0) * a.R);
    }
#pragma unroll
    for (int b = 0; b < kBT; ++b) {
      acc[b] = dot4(va, x[b], acc[b]);
      acc[kBT + b] = dot4(vb, x[b], acc[kBT + b]);
    }
  }
  const float s = wave_reduce_multi<2 * kBT>(acc, lane);
  if (MODE & 32) {
    if (wave == 0 && lane < nb) a.gbuf[(int64_t)(b0 + lane) * H + o] = s;
    return;
  }
  if ((lane & 3) == 0) s_red[wave][lane >> 2] = s;
  __syncthreads();
  if ((int)threadIdx.x < nb) {
    const int b = threadIdx.x;
    float za = 0.f, zb = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) { za += s_red[w][b]; zb += s_red[w][kBT + b]; }
    const int gb = b0 + b;
    if (!(MODE & 1)) {
      const float* pre = a.pre + ((int64_t)(t % a.Tch) * a.B + gb) * ((int64_t)a.n_layers * a.G) + (int64_t)layer * a.G;
      za += pre[o];
      zb += pre[o + H];
    }
    const float v = (MODE & 64) ? za + zb : tanhf(za) * avc_sigmoid(zb);
    if (!(MODE & 16) || v == 12345.f) a.gbuf[(int64_t)gb * H + o] = v;
  }
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1000000) p[0] = 1;
}

__global__ __launch_bounds__(384) void lds_barrier_kernel(float* p) {
  __shared__ float s_red[6][16];
  if ((threadIdx.x & 3) == 0) s_red[threadIdx.x >> 6][(threadIdx.x >> 2) & 15] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x < 8 && s_red[0][threadIdx.x] == 12345.f) p[0] = 1;
}

__global__ __launch_bounds__(384) void reduce16_kernel(float* p) {
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = threadIdx.x * (j + 1);
  const float s = wave_reduce_multi<16>(acc, threadIdx.x & 63);
  if (s == 12345.f) p[0] = 1;
}

__global__ __launch_bounds__(384) void reduce8_kernel(float* p) {
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = threadIdx.x * (j + 1);
  const float s = wave_reduce_multi<8>(acc, threadIdx.x & 63);
  if (s == 12345.f) p[0] = 1;
}

__global__ __launch_bounds__(384) void args_kernel(WnArgs a, int layer, int slot) {
  const int t = a.ctr[slot];
  const int d = 1 << (layer % a.lps);
  const int x = (t % a.Tch) + d + a.K * a.R;
  if (x == 1234567) a.gbuf[0] = 1.f;
}

}  // namespace

int main() {
  const int B = 8, T = 4096, L = 24, LPS = 6, K = 3, R = 512, G = 512, S = 256, NO = 30, Tch = 2048;
  const int64_t npk = autovc_wavenet_packed_floats(L, K, R, G, S, NO);
  const int64_t wsb = autovc_wavenet_workspace_bytes(B, T, L, LPS, K, R, G, S);
  float *packed, *pre, *y;
  void* ws;
  (void)hipMalloc(&packed, npk * 4);
  (void)hipMalloc(&pre, (size_t)Tch * B * L * G * 4);
  (void)hipMalloc(&y, (size_t)B * T * 4);
  (void)hipMalloc(&ws, wsb);
  (void)hipMemset(packed, 0, npk * 4);
  (void)hipMemset(pre, 0, (size_t)Tch * B * L * G * 4);
  (void)hipMemset(ws, 0, wsb);
  // Build WnArgs exactly as the entry point does by running one generate step.
  if (autovc_wavenet_generate_f32(B, T, 0, 1, L, LPS, K, R, G, S, NO, 1, packed, pre, Tch, 1, 0, -7.f, nullptr, 0, y,
                                  nullptr, ws, 0, 0) != 0) {
    printf("generate failed: %s\n", autovc_last_error());
    return 1;
  }
  (void)hipDeviceSynchronize();
  auto round64 = [](int64_t n) { return (n + 63) / 64 * 64; };
  WnArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.T = T; a.R = R; a.G = G; a.S = S; a.NO = NO; a.K = K; a.RING = (int)ring_frames(L, LPS, K);
  a.n_layers = L; a.lps = LPS; a.Tch = Tch; a.legacy = 1; a.packed = packed; a.pre = pre;
  float* w = static_cast<float*>(ws);
  a.ring = w; w += round64((int64_t)(L + 1) * a.RING * B * R);
  a.yin = w; w += round64((int64_t)B * T);
  a.skip = w; w += round64((int64_t)B * S);
  a.h1 = w; w += round64((int64_t)B * S);
  a.gbuf = w; w += round64((int64_t)B * (G / 2));
  a.ctr = reinterpret_cast<int*>(w);
  a.y_out = y; a.log_scale_min = -7.f;
  // step counter at 300 for every slot: all taps valid
  std::vector<int> h(kCtrSlots, 300);
  (void)hipMemcpy(a.ctr, h.data(), h.size() * 4, hipMemcpyHostToDevice);

  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int N = 400;
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 20; ++i) launch(i);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < N; ++i) launch(i);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const hipError_t err = hipGetLastError();
    printf("%-34s %8.2f us/launch %s\n", name, ms * 1000.f / N, err == hipSuccess ? "" : hipGetErrorString(err));
  };
  const dim3 gg(G / 2, 1);
  timeit("empty 256x384", [&](int) { hipLaunchKernelGGL(empty_kernel, gg, dim3(384), 0, 0, nullptr); });
  timeit("lds+barrier 256x384", [&](int) { hipLaunchKernelGGL(lds_barrier_kernel, gg, dim3(384), 0, 0, a.gbuf); });
  timeit("reduce16 256x384", [&](int) { hipLaunchKernelGGL(reduce16_kernel, gg, dim3(384), 0, 0, a.gbuf); });
  timeit("reduce8 256x384", [&](int) { hipLaunchKernelGGL(reduce8_kernel, gg, dim3(384), 0, 0, a.gbuf); });
  timeit("args 256x384", [&](int) { hipLaunchKernelGGL(args_kernel, gg, dim3(384), 0, 0, a, 5, 10); });
  timeit("gate production (layer 5)", [&](int) {
    hipLaunchKernelGGL((wn_gate_kernel<6, false>), gg, dim3(384), 0, 0, a, 5, 10); });
  timeit("gate copy MODE=0", [&](int) { hipLaunchKernelGGL((gate_variant<6, 0>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate no pre", [&](int) { hipLaunchKernelGGL((gate_variant<6, 1>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate no ring", [&](int) { hipLaunchKernelGGL((gate_variant<6, 2>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate no weights", [&](int) { hipLaunchKernelGGL((gate_variant<6, 4>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate t arg", [&](int) { hipLaunchKernelGGL((gate_variant<6, 8>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate no pre/ring/weights, t arg", [&](int) {
    hipLaunchKernelGGL((gate_variant<6, 15>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate 15 + no store", [&](int) { hipLaunchKernelGGL((gate_variant<6, 31>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate 15 + no LDS red", [&](int) { hipLaunchKernelGGL((gate_variant<6, 47>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate 15 + no tanh", [&](int) { hipLaunchKernelGGL((gate_variant<6, 79>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate 15 + no tanh, no store", [&](int) { hipLaunchKernelGGL((gate_variant<6, 95>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate 15 all off", [&](int) { hipLaunchKernelGGL((gate_variant<6, 127>), gg, dim3(384), 0, 0, a, 5, 10, 300); });
  timeit("gate NW=3", [&](int) { hipLaunchKernelGGL((gate_variant<3, 0>), gg, dim3(192), 0, 0, a, 5, 10, 300); });
  timeit("gate NW=2", [&](int) { hipLaunchKernelGGL((gate_variant<2, 0>), gg, dim3(128), 0, 0, a, 5, 10, 300); });
  timeit("gate layers rotating", [&](int i) {
    hipLaunchKernelGGL((wn_gate_kernel<6, false>), gg, dim3(384), 0, 0, a, 1 + i % 23, 2 * (1 + i % 23)); });
  timeit("resid production (layer 5)", [&](int) {
    hipLaunchKernelGGL((wn_resid_kernel<4>), dim3((R + S) / 4, 1), dim3(256), 0, 0, a, 5, 11); });
  timeit("head production", [&](int) {
    hipLaunchKernelGGL((wn_head_kernel<4>), dim3(S / 4, 1), dim3(256), 0, 0, a, 2 * L); });
  timeit("full step (direct)", [&](int) { (void)enqueue_step(a, 0); });
  return 0;
}
