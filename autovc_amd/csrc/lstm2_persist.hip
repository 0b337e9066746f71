// Decoder lstm2 forward (nn.LSTM(512, 1024, num_layers=2), model_vc_mel.py:104,118) as ONE
// persistent, weight-stationary launch for gfx950.
//
// The per-step launch (lstm.hip, lstm2_fwd_step_kernel) re-streams every weight row of both
// layers into every CU at every step, which bounds the step at ~24 us (the CU's operand fill,
// not the MFMA: 10.2 us of fp32 MFMA per CU at peak).  Here each of the 256 workgroups (one
// per CU) owns all 64 batch rows x 16 gate columns (4 hidden units x 4 gates) of BOTH layers
// for the whole sequence and keeps their weights on the CU:
//   W_hh0, W_ih1 tile rows -> LDS (64 KB each, k-blocked [k/4][col][4]: conflict-free b128 reads)
//   W_hh1 tile rows        -> VGPRs (64 floats per lane: the MFMA B fragments)
// so a step streams only the h rows (h0_{t-1}, shared by both layers, and h1_{t-2}): 512 KB
// per CU, L2-served.  Steps are separated by an XCD-hierarchical grid barrier instead of a
// launch boundary (MI355X_MICROARCH.md price list: barrier-xcd).
//
// Iteration t (t = 0..T) is the same wavefront as the per-step launch: layer 0 at step t
// (input h0_{t-1}), layer 1 at step t-1 (inputs h0_{t-1}, h1_{t-2}).  v_mfma_f32_16x16x4_f32
// (exact fp32), one wave per SIMD: wave w takes k in [256w, 256w + 256) of h0_{t-1} (layer 0,
// B = W_hh0 from LDS; layer 1's input product, B = W_ih1 from LDS) and h1_{t-2} (layer 1's
// recurrent product, B = W_hh1 from VGPRs).  MFMA k slot s = lane / 16 takes the 64
// consecutive k from k0 + 64 s, so a lane's weights and its h fragments are contiguous; the h
// rows come from a k-blocked copy [t][H/4][B][4] the epilogues write beside h (256 B
// contiguous per 16 lanes).  The 4 waves' partial tiles are summed through LDS in fixed order,
// then the cell update (v_exp / v_rcp sigmoid and tanh).
//
// Measured (profiles/r02/lstm2_persist_ab.txt, B=64 T=128): 23.9 us per iteration against
// 23.7 for the per-step launches, so it stays opt-in.  Ablations: no grid barrier 21.0, no
// products 8.0 (barrier + epilogue), products without the h loads 14.8.  The h stream is the
// limiter: 512 KB per CU per iteration at the L2-shared per-CU fill rate (66-73 GB/s,
// MI355X_MICROARCH.md "Indexed rows") is 7.3 us that the one-wave-per-SIMD MFMA stream does
// not hide; prefetch depth 2/3/4 groups measured 24.5/23.9/25.1.
//
// Inter-workgroup visibility (cdna_hip_programming.md Guideline 16, the write-through form of
// MI355X_MICROARCH.md "Valid forms", first row of its table): the only bytes handed between
// workgroups are the k-blocked h copies; they are stored sc1 (write-through), every wave
// waits vmcnt(0), the workgroup barrier, then ONE lane adds to its XCC's arrival counter
// (agent-scope atomic); the XCC's last arriver adds to the top counter, whose last arriver
// stores the generation word every workgroup polls (sc1 loads); every load of the handed-off
// bytes is an sc1 buffer load, so no release / acquire fence is needed.  Every k-blocked row
// is written once per call (fresh addresses).  Every spin is bounded by s_memrealtime; a
// timeout sets an error word and every workgroup exits.
#include "common.h"
#include "../../include/autovc_hip.h"

#include <hip/hip_runtime.h>

#include <type_traits>

namespace {

constexpr int PB = 64;             // batch rows per tile (all of them)
constexpr int PU = 4;              // hidden units per tile (x 4 gates = 16 columns)
constexpr int PC = 4 * PU;         // tile columns
constexpr int PNW = 8;             // waves per workgroup: two per SIMD (one wave's MFMAs run
                                   // while the other waits for its h loads)
constexpr int PNT = 64 * PNW;
constexpr int PRH = PNW == 16 ? 2 : 1;   // row halves: 16 waves = 8 k ranges x 2 row halves
constexpr int PKWN = PNW / PRH;    // k ranges
constexpr int PRB = PB / 16;       // 16-row blocks of the tile (4)
constexpr int PRBW = PRB / PRH;    // 16-row blocks per wave
constexpr int PWIN = 1;            // h groups in flight per stream
constexpr int RED_LD = PC + 1;     // padded row of a 64 x 16 partial tile in LDS
constexpr int RED_SLOT = PB * RED_LD;
constexpr int NSLOT = 4;                            // partial-tile slots (one layer at a time)
static_assert(PNW == 4 || PNW == 8 || PNW == 16, "waves per workgroup");
constexpr int LDS_RED = NSLOT * RED_SLOT;

// per hidden size HH: k per wave and segment, k per MFMA lane group, 4-k groups per lane,
// floats of one k-blocked [k/4][16][4] weight tile in LDS
template <int HH>
struct PK {
  static constexpr int KW = HH / PKWN, KL = KW / 4, GR = KL / 4, W = (HH / 4) * PC * 4;
};
// LDS floats of a launch: W_hh0 (+ W_ih1 for the stacked pair) and the partial-tile slots
template <int HH, bool TWO, bool BF = false>
constexpr int lds_bytes() {
  return (BF ? 2 : 4) * PK<HH>::W * (TWO ? 2 : 1) + 4 * LDS_RED;
}
static_assert(lds_bytes<1024, true>() <= 160 * 1024, "LDS budget");

// barrier block: one 128-B line per word (ints)
constexpr int L = 32;
constexpr int BAR_CENSUS = 0;      // 16 lines: workgroups per XCC
constexpr int BAR_START = 16;      // 1 line: workgroups arrived at the start
constexpr int BAR_ARRIVE = 17;     // 16 lines: per-XCC arrivals (cumulative)
constexpr int BAR_TOP = 33;        // 1 line: XCC leaders arrived (cumulative)
constexpr int BAR_GEN = 34;        // 16 lines: per-XCC generation released
constexpr int BAR_ERR = 50;        // 1 line: timeout / error code
constexpr int BAR_LINES = 52;
constexpr int64_t BAR_BYTES = BAR_LINES * L * 4;

struct PArgs {
  int B, T, H;
  const float* gx0;
  int64_t gx_ldb, gx_ldt;
  const float* W_hh0;
  const float* b_ih1;
  const float* b_hh1;
  const float* W_ih1;
  const float* W_hh1;
  float *h0, *c0, *g0, *h1, *c1, *g1;
  int64_t h0_ldb, h0_ldt;          // h0 strides (single layer: the caller's; stacked: T*H, H)
  float* hk0;                      // k-blocked h0: [t][H/4][B][4]
  float* hk1;                      // k-blocked h1
  // bf16 variant (precision("bf16"), numerics of autovc_lstm2_fwd_bf16): RNE weight copies,
  // and bf16 hand-off copies of h blocked by 8: [t][H/8][B][8]
  const __bf16 *W0b, *Wi1b, *W1b;
  __bf16 *hk0b, *hk1b;
  int* bar;
  int timeout_ticks;               // s_memrealtime ticks (100 MHz) before a spin gives up
};

__device__ __forceinline__ int ld_rlx(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int add_rlx(int* p, int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// spin until *p >= target or the deadline passes (returns false on timeout, after
// recording it); one lane polls, s_sleep between polls
__device__ __noinline__ bool wait_ge(int* p, int target, int* err, int timeout_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_rlx(p) < target) {
    if (ld_rlx(err) != 0) return false;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)timeout_ticks) {
      st_rlx(err, 1);
      return false;
    }
  }
  return true;
}

// Grid barrier number `gen` (0, 1, ...).  Called by every thread; returns false if any
// workgroup timed out (then every workgroup leaves the kernel).
// xcc / mine / nx: this workgroup's XCC, the workgroups on it and the XCCs in use (held by
// thread 0); *status: an LDS word broadcasting the outcome to the workgroup
__device__ __forceinline__ bool grid_sync(const PArgs& a, int xcc, int mine, int nx, const int (&census)[16],
                                          int* status, int gen) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this wave's stores are in L2
  __syncthreads();
  if (threadIdx.x == 0) {
    bool ok = true;
    const int old = add_rlx(a.bar + (BAR_ARRIVE + xcc) * L, 1);
    if (old == mine * (gen + 1) - 1) {                    // last of this XCC
      const int top = add_rlx(a.bar + BAR_TOP * L, 1);
      if (top == nx * (gen + 1) - 1)                      // last XCC: open every XCC's gate
        for (int x = 0; x < 16; ++x) st_rlx(a.bar + (BAR_GEN + x) * L, gen + 1);
    }
    ok = wait_ge(a.bar + (BAR_GEN + xcc) * L, gen + 1, a.bar + BAR_ERR * L, a.timeout_ticks);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler order only (sc1 loads follow)
    *status = ok ? 0 : 1;
  }
  __syncthreads();
  return *status == 0;
}

// grid_sync in two halves, so a workgroup can work between its arrival and
// the release: grid_arrive publishes this workgroup's hand-off (the last arriver of the last
// XCC opens every gate), grid_wait polls this XCC's gate
__device__ __forceinline__ void grid_arrive(const PArgs& a, int xcc, int mine, int nx, int gen) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = add_rlx(a.bar + (BAR_ARRIVE + xcc) * L, 1);
    if (old == mine * (gen + 1) - 1) {
      const int top = add_rlx(a.bar + BAR_TOP * L, 1);
      if (top == nx * (gen + 1) - 1)
        for (int x = 0; x < 16; ++x) st_rlx(a.bar + (BAR_GEN + x) * L, gen + 1);
    }
  }
}

__device__ __forceinline__ bool grid_wait(const PArgs& a, int xcc, int* status, int gen) {
  if (threadIdx.x == 0) {
    const bool ok = wait_ge(a.bar + (BAR_GEN + xcc) * L, gen + 1, a.bar + BAR_ERR * L, a.timeout_ticks);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler order only (sc1 loads follow)
    *status = ok ? 0 : 1;
  }
  __syncthreads();
  return *status == 0;
}

// Sticky per-device fault word: a launch whose grid barrier timed out (its workgroups were
// not all resident at once — e.g. another process's kernels held part of the chip) ORs its
// kernel family's bit into it, after writing NaN over every output it owns, so the failure
// reaches the loss.  The host reads and clears it at its sync points (autovc_fault_status:
// Solver log steps, bench.py) and raises, naming the kernel (autovc_amd.functional).
__device__ int g_avc_fault = 0;
constexpr int kFaultLstm2Persist = 1;    // lstm_persist_kernel, two layers (decoder lstm2 forward)
constexpr int kFaultLstmXcdFwd = 2;      // lstm_xcd_fwd_kernel (decoder lstm1 forward)
constexpr int kFaultLstmXcdBwd = 4;      // lstm_xcd_bwd_kernel (decoder lstm1 backward)
constexpr int kFaultLstm1Persist = 8;    // lstm_persist_kernel, one layer (opt-in)
int g_timeout_ticks = 0;             // 0 = the default 1 s; tests force a timeout with a tiny value

// per-step cell update of one (batch row b, unit j) from its 4 gate pre-activations
// Only the k-blocked h copy is handed to other workgroups, so only it is stored before the
// grid barrier (sc1, write-through); h, c and the gates are kept in registers and stored
// after the barrier, under the next iteration's products (the barrier's vmcnt(0) then waits
// for the hand-off stores alone).  The cell state is carried in registers, never re-read.
struct CellOut { float c, h, i, f, g, o; };

// Every multiply-add is spelled out (contraction off): the kernels that share this update
// (lstm_persist_kernel, lstm2_rs_kernel) then round it identically whatever the compiler
// would fuse in each context.
__device__ __forceinline__ float tanh_fast_nc(float x) {
#pragma clang fp contract(off)
  return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x * 2.88539008f) + 1.0f), 1.0f);
}
__device__ __forceinline__ float sigmoid_fast_nc(float x) {
#pragma clang fp contract(off)
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504f));
}

__device__ __forceinline__ CellOut cell(const float (&pre)[4], float cp) {
#pragma clang fp contract(off)
  CellOut r;
  r.i = sigmoid_fast_nc(pre[0]);
  r.f = sigmoid_fast_nc(pre[1]);
  r.g = tanh_fast_nc(pre[2]);
  r.o = sigmoid_fast_nc(pre[3]);
  r.c = __builtin_fmaf(r.f, cp, r.i * r.g);
  r.h = r.o * tanh_fast_nc(r.c);
  return r;
}

// the hand-off copy of h (sc1 write-through stores).  fp32: one dword per (row, unit) at
// [H/4][B][4]; bf16: the 4 units of a row held by 4 consecutive lanes are gathered into the
// first of them and stored as one 8-byte word at [H/8][B][8] (every lane of the wave calls)
template <bool BF>
__device__ __forceinline__ void handoff(float h, float* hk, __bf16* hkb, int B, int eb, int ej, int lane) {
  if constexpr (!BF) {
    __hip_atomic_store(hk + ((int64_t)(ej >> 2) * B + eb) * 4 + (ej & 3), h, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    const __bf16 hb = (__bf16)h;
    const int v = (int)__builtin_bit_cast(unsigned short, hb);
    const int q0 = lane & ~3;
    const unsigned long long w = (unsigned long long)(unsigned)(__shfl(v, q0, 64) | (__shfl(v, q0 + 1, 64) << 16)) |
                                 ((unsigned long long)(unsigned)(__shfl(v, q0 + 2, 64) |
                                                                 (__shfl(v, q0 + 3, 64) << 16)) << 32);
    if ((lane & 3) == 0)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(hkb + ((int64_t)(ej >> 3) * B + eb) * 8 + (ej & 7)), w,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void cell_store(const CellOut& r, float* c_out, float* h_out, float* g_out, int64_t H) {
  *c_out = r.c;
  *h_out = r.h;
  if (g_out) { g_out[0] = r.i; g_out[H] = r.f; g_out[2 * H] = r.g; g_out[3 * H] = r.o; }
}

// acc[rb] (16 x 16 MFMA tiles of the 64 x 16 tile) -> LDS partial slot: C/D map of
// v_mfma_f32_16x16x4f32: col = lane & 15, row = 4 (lane >> 4) + r
__device__ __forceinline__ void put_tile(float* slot, const f32x4 (&acc)[PRBW], int rb0, int lane) {
#pragma unroll
  for (int rb = 0; rb < PRBW; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) slot[(16 * (rb0 + rb) + 4 * (lane >> 4) + r) * RED_LD + (lane & 15)] = acc[rb][r];
}

__device__ __forceinline__ void add_tile(float* slot, const f32x4 (&acc)[PRBW], int rb0, int lane) {
#pragma unroll
  for (int rb = 0; rb < PRBW; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) slot[(16 * (rb0 + rb) + 4 * (lane >> 4) + r) * RED_LD + (lane & 15)] += acc[rb][r];
}

// One iteration's products of a wave over its k range of stream h0_{t-1}: S0 = layer 1's input
// product (B = W_ih1 from LDS), L0 = layer 0's recurrent product (B = W_hh0 from LDS); S1 =
// stream h1_{t-2}, layer 1's recurrent product (B = W_hh1 fragments in VGPRs).  Lane l: MFMA k slot
// l >> 4 covers k = kbase + 64 (l >> 4) + i, row block rb's A row 16 rb + (l & 15).
template <int KL, bool S0, bool L0, bool S1>
__device__ __forceinline__ void gemm_wave(const float* __restrict__ hk0_t, const float* __restrict__ hk1_t,
                                          const float (&wh)[KL], const float* W0, const float* W1, int kb0,
                                          int B, int rb0, int lane, f32x4 (&acc1)[PRBW], f32x4 (&acc0)[PRBW]) {
  // group g, row block rb: f32x4 at hk[kb0 + g][16 rb + (lane & 15)][0..3]; sc1 buffer loads
  // (every load of the handed-off rows bypasses L1: no acquire fence needed)
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hk0_t), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hk1_t), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t off0 = (uint32_t)((kb0 * B + 16 * rb0 + (lane & 15)) * 16);
  const uint32_t gstride = (uint32_t)B * 16;
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int g, int rb) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off0 + g * gstride + rb * 256, 0, 16));
  };
  f32x4 a0[PWIN][PRBW], a1[PWIN][PRBW];
#pragma unroll
  for (int g = 0; g < PWIN; ++g)
#pragma unroll
    for (int rb = 0; rb < PRBW; ++rb) {
      if (S0 || L0) a0[g][rb] = ld(r0, g, rb);
      if (S1) a1[g][rb] = ld(r1, g, rb);
    }
  const float* w0p = W0 + (kb0 * PC + (lane & 15)) * 4;
  const float* w1p = W1 + (kb0 * PC + (lane & 15)) * 4;
#pragma unroll
  for (int g = 0; g < KL / 4; ++g) {
    f32x4 x0[PRBW], x1[PRBW];
#pragma unroll
    for (int rb = 0; rb < PRBW; ++rb) {
      x0[rb] = a0[g % PWIN][rb];
      x1[rb] = a1[g % PWIN][rb];
    }
    if (g + PWIN < KL / 4) {
#pragma unroll
      for (int rb = 0; rb < PRBW; ++rb) {
        if (S0 || L0) a0[g % PWIN][rb] = ld(r0, g + PWIN, rb);
        if (S1) a1[g % PWIN][rb] = ld(r1, g + PWIN, rb);
      }
    }
    f32x4 bv0 = {}, bv1 = {};
    if (L0) bv0 = *reinterpret_cast<const f32x4*>(w0p + g * PC * 4);
    if (S0) bv1 = *reinterpret_cast<const f32x4*>(w1p + g * PC * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int rb = 0; rb < PRBW; ++rb) {
        if (S0) acc1[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[rb][q], bv1[q], acc1[rb], 0, 0, 0);
        if (S1) acc1[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[rb][q], wh[4 * g + q], acc1[rb], 0, 0, 0);
        if (L0) acc0[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[rb][q], bv0[q], acc0[rb], 0, 0, 0);
      }
  }
}

// bf16 products (v_mfma_f32_16x16x32_bf16): lane l supplies rows 16 rb + (l & 15) and the 8
// k of block k8 = k8_0 + 4 s (8 (l >> 4) within the 32-k step s) of the bf16 hand-off copy,
// B fragments from the bf16 LDS tiles [H/8][16][8] (W_hh0, W_ih1) or VGPRs (W_hh1).
template <int NS, bool S0, bool L0, bool S1>
__device__ __forceinline__ void gemm_wave_bf(const __bf16* __restrict__ hk0_t, const __bf16* __restrict__ hk1_t,
                                             const bf16x8 (&wh)[NS], const __bf16* W0, const __bf16* W1, int k8_0,
                                             int B, int rb0, int lane, f32x4 (&acc1)[PRBW], f32x4 (&acc0)[PRBW]) {
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(hk0_t), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(hk1_t), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t off0 = (uint32_t)((k8_0 * B + 16 * rb0 + (lane & 15)) * 16);
  const uint32_t sstride = (uint32_t)B * 64;          // 4 k8 blocks per 32-k step
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int st, int rb) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off0 + st * sstride + rb * 256, 0, 16));
  };
  bf16x8 a0[PRBW], a1[PRBW];
#pragma unroll
  for (int rb = 0; rb < PRBW; ++rb) {
    if (S0 || L0) a0[rb] = ld(r0, 0, rb);
    if (S1) a1[rb] = ld(r1, 0, rb);
  }
  const __bf16* w0p = W0 + (k8_0 * PC + (lane & 15)) * 8;
  const __bf16* w1p = W1 + (k8_0 * PC + (lane & 15)) * 8;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    bf16x8 x0[PRBW], x1[PRBW];
#pragma unroll
    for (int rb = 0; rb < PRBW; ++rb) {
      x0[rb] = a0[rb];
      x1[rb] = a1[rb];
    }
    if (st + 1 < NS) {
#pragma unroll
      for (int rb = 0; rb < PRBW; ++rb) {
        if (S0 || L0) a0[rb] = ld(r0, st + 1, rb);
        if (S1) a1[rb] = ld(r1, st + 1, rb);
      }
    }
    bf16x8 bv0 = {}, bv1 = {};
    if (L0) bv0 = *reinterpret_cast<const bf16x8*>(w0p + st * 4 * PC * 8);
    if (S0) bv1 = *reinterpret_cast<const bf16x8*>(w1p + st * 4 * PC * 8);
#pragma unroll
    for (int rb = 0; rb < PRBW; ++rb) {
      if (S0) acc1[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0[rb], bv1, acc1[rb], 0, 0, 0);
      if (S1) acc1[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[rb], wh[st], acc1[rb], 0, 0, 0);
      if (L0) acc0[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0[rb], bv0, acc0[rb], 0, 0, 0);
    }
  }
}

// TWO: the stacked pair (decoder lstm2); else one layer (decoder lstm1), whose "layer 0" is
// that layer and whose iteration t is its step t (no lag, T iterations).
// BF: bf16 weights and hand-off copies (the products' numerics of autovc_lstm2_fwd_bf16);
// cell math, c, h, gates fp32 either way.
template <int HH, bool TWO, bool BF = false, bool LAG2 = false>
__global__ __launch_bounds__(PNT, 1) void lstm_persist_kernel(PArgs a) {
  constexpr int KW = PK<HH>::KW, KL = PK<HH>::KL, GR = PK<HH>::GR, NS = KW / 32;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* W0 = lds;                          // fp32 [H/4][16][4]
  float* W1 = lds + PK<HH>::W;              // fp32 [H/4][16][4] (TWO)
  __bf16* W0b = reinterpret_cast<__bf16*>(lds);             // bf16 [H/8][16][8]
  __bf16* W1b = W0b + PK<HH>::W;                            // bf16 [H/8][16][8] (TWO)
  float* red = lds + (BF ? PK<HH>::W / 2 : PK<HH>::W) * (TWO ? 2 : 1);   // partial-tile slots
  // broadcast word: the pad column of slot 0's row 0, never written by put_tile / add_tile
  int* status = reinterpret_cast<int*>(red + PC);
  int xcc_id = 0, xcc_wgs = 0, xcc_n = 0;
  int census[16] = {};                     // workgroups per XCC (thread 0)
  constexpr int H = HH;
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware unit blocks: workgroups are dispatched round-robin over the 8 XCDs, so block
  // b (on XCD b % 8) owns unit block (b % 8) * (grid / 8) + b / 8 — each XCD's workgroups own
  // one contiguous run of H / 8 units, and the 16-B row pieces of h / c / gates that
  // neighbouring units write meet in that XCD's (write-back) L2 as whole lines instead of
  // leaving it as partial-line writes (PMC WRITE_SIZE 853 MB per launch with b -> block b)
  const int nxb = (int)gridDim.x / 8;
  const int j0 = ((int)blockIdx.x % 8 * nxb + (int)blockIdx.x / 8) * PU;
  auto grow = [&](int col) { return (col >> 2) * H + j0 + (col & 3); };   // tile column -> gate row
  // epilogue ownership: thread e owns (batch row e / 4, unit j0 + e % 4) of both layers
  const int eb = tid >> 2, ej = j0 + (tid & 3), eu = tid & 3;
  const bool eown = eb < B;
  // a timed-out barrier: NaN over everything this workgroup owns (its h / c of every step
  // and layer), the device fault word set once per workgroup, then the workgroup exits
  auto fail = [&]() {
    const float nan = __builtin_nanf("");
    if (eown)
      for (int t = 0; t < T; ++t) {
        a.h0[(int64_t)eb * a.h0_ldb + (int64_t)t * a.h0_ldt + ej] = nan;
        a.c0[((int64_t)eb * T + t) * H + ej] = nan;
        if (TWO) {
          a.h1[((int64_t)eb * T + t) * H + ej] = nan;
          a.c1[((int64_t)eb * T + t) * H + ej] = nan;
        }
      }
    if (tid == 0)
      __hip_atomic_fetch_or(&g_avc_fault, TWO ? kFaultLstm2Persist : kFaultLstm1Persist, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---- start: census of workgroups per XCC (the barrier's groups)
  if (tid == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 15;
    add_rlx(a.bar + (BAR_CENSUS + xcc) * L, 1);
    add_rlx(a.bar + BAR_START * L, 1);
    const bool ok = wait_ge(a.bar + BAR_START * L, gridDim.x, a.bar + BAR_ERR * L, a.timeout_ticks);
    int nx = 0;
    for (int x = 0; x < 16; ++x) {
      census[x] = ld_rlx(a.bar + (BAR_CENSUS + x) * L);
      nx += census[x] > 0;
    }
    xcc_id = (int)xcc;
    xcc_wgs = ld_rlx(a.bar + (BAR_CENSUS + xcc) * L);
    xcc_n = nx;
    *status = ok ? 0 : 1;
  }
  // ---- weights: W_hh0 (and W_ih1) tiles -> LDS (k-blocked), W_hh1 fragments -> VGPRs
  if (BF) {
    for (int e = tid; e < (H / 8) * PC; e += PNT) {
      const int kb = e / PC, col = e % PC;
      *reinterpret_cast<bf16x8*>(W0b + e * 8) = *reinterpret_cast<const bf16x8*>(a.W0b + (int64_t)grow(col) * H + kb * 8);
      if (TWO)
        *reinterpret_cast<bf16x8*>(W1b + e * 8) =
            *reinterpret_cast<const bf16x8*>(a.Wi1b + (int64_t)grow(col) * H + kb * 8);
    }
  } else for (int e = tid; e < (H / 4) * PC; e += PNT) {
    const int kb = e / PC, col = e % PC;
    *reinterpret_cast<f32x4*>(W0 + e * 4) = *reinterpret_cast<const f32x4*>(a.W_hh0 + (int64_t)grow(col) * H + kb * 4);
    if (TWO)
      *reinterpret_cast<f32x4*>(W1 + e * 4) =
          *reinterpret_cast<const f32x4*>(a.W_ih1 + (int64_t)grow(col) * H + kb * 4);
  }
  const int kw = wave % PKWN, rb0 = (wave / PKWN) * PRBW;    // k range, first row block
  const int kbase = kw * KW + KL * (lane >> 4);               // this lane's first k
  const int kb0 = kbase / 4;
  float wh[KL] = {};
  bf16x8 whb[NS] = {};
  const int k8_0 = (kw * KW) / 8 + (lane >> 4);              // bf16: this lane's first k block
  if (TWO && BF) {
#pragma unroll
    for (int st = 0; st < NS; ++st)
      whb[st] = *reinterpret_cast<const bf16x8*>(a.W1b + (int64_t)grow(lane & 15) * H + 8 * (k8_0 + 4 * st));
  } else if (TWO) {
    const float* sh = a.W_hh1 + (int64_t)grow(lane & 15) * H + kbase;
#pragma unroll
    for (int g = 0; g < GR; ++g) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(sh + 4 * g);
      wh[4 * g] = u[0]; wh[4 * g + 1] = u[1]; wh[4 * g + 2] = u[2]; wh[4 * g + 3] = u[3];
    }
  }
  __syncthreads();
  if (*status != 0) {
    fail();
    return;
  }

  float bias1[4] = {0.f, 0.f, 0.f, 0.f};
  if (TWO && eown)
#pragma unroll
    for (int g = 0; g < 4; ++g) bias1[g] = a.b_ih1[g * H + ej] + a.b_hh1[g * H + ej];
  const int64_t BH = (int64_t)B * H;
  CellOut out0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, out1 = out0;   // c carried from step to step
  // the previous iteration's outputs (layer 0 at step t0, layer 1 at step t0 - 1)
  auto store_outputs = [&](int t0) {
    if (!eown) return;
    if (TWO && t0 >= 1) {
      const int t1 = t0 - 1;
      const int64_t o = ((int64_t)eb * T + t1) * H + ej;
      cell_store(out1, a.c1 + o, a.h1 + o, a.g1 ? a.g1 + ((int64_t)eb * T + t1) * 4 * H + ej : nullptr, H);
    }
    if (t0 < T) {
      const int64_t o = ((int64_t)eb * T + t0) * H + ej;
      cell_store(out0, a.c0 + o, a.h0 + (int64_t)eb * a.h0_ldb + (int64_t)t0 * a.h0_ldt + ej,
                 a.g0 ? a.g0 + ((int64_t)eb * T + t0) * 4 * H + ej : nullptr, H);
    }
  };

  if constexpr (TWO && LAG2) {
    // Two-step wavefront: iteration t runs layer 0 at step t and layer 1 at step t - 2, so
    // layer 1's input product W_ih1 h0_(t-1) (for its step t - 1, done in iteration t + 1)
    // reads rows released one barrier earlier and runs between this workgroup's arrival at
    // barrier t and the release: a third of the MFMA work under the barrier's latency, for a
    // second (L2-hot) read of h0_(t-1).  After the release: W_hh0 h0_(t-1) and W_hh1 h1_(t-3).
    auto store_outputs2 = [&](int t0) {
      if (!eown) return;
      if (t0 >= 2 && t0 - 2 < T) {
        const int t1 = t0 - 2;
        const int64_t o = ((int64_t)eb * T + t1) * H + ej;
        cell_store(out1, a.c1 + o, a.h1 + o, a.g1 ? a.g1 + ((int64_t)eb * T + t1) * 4 * H + ej : nullptr, H);
      }
      if (t0 < T) {
        const int64_t o = ((int64_t)eb * T + t0) * H + ej;
        cell_store(out0, a.c0 + o, a.h0 + (int64_t)eb * a.h0_ldb + (int64_t)t0 * a.h0_ldt + ej,
                   a.g0 ? a.g0 + ((int64_t)eb * T + t0) * 4 * H + ej : nullptr, H);
      }
    };
    const int last2 = T + 1;
    f32x4 acc1[PRBW] = {};                                            // layer 1's carried input product
    for (int t = 0; t <= last2; ++t) {
      const bool l0 = t < T, l1 = t >= 2;
      if (t >= 1) store_outputs2(t - 1);
      float gxv[4] = {0.f, 0.f, 0.f, 0.f};
      if (eown && l0) {
        const float* g = a.gx0 + (int64_t)eb * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
        for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + ej];
      }
      f32x4 acc0[PRBW] = {};
      const int th0 = t >= 1 ? t - 1 : 0, th1 = t >= 3 ? t - 3 : 0;
      const bool pl0 = l0 && t >= 1, ps1 = t >= 3;
      if constexpr (BF) {
        const __bf16* hk0b = a.hk0b + (int64_t)th0 * BH;
        const __bf16* hk1b = a.hk1b + (int64_t)th1 * BH;
        if (pl0 && ps1) gemm_wave_bf<NS, false, true, true>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
        else if (pl0) gemm_wave_bf<NS, false, true, false>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
        else if (ps1) gemm_wave_bf<NS, false, false, true>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
      } else {
        const float* hk0 = a.hk0 + (int64_t)th0 * BH;
        const float* hk1 = a.hk1 + (int64_t)th1 * BH;
        if (pl0 && ps1) gemm_wave<KL, false, true, true>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
        else if (pl0) gemm_wave<KL, false, true, false>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
        else if (ps1) gemm_wave<KL, false, false, true>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
      }
      auto sum = [&](int g) {
        const float* r = red + eb * RED_LD + g * PU + eu;
        return ((r[0] + r[RED_SLOT]) + r[2 * RED_SLOT]) + r[3 * RED_SLOT];
      };
      auto reduce_put = [&](const f32x4 (&acc)[PRBW]) {
        if (kw < 4) put_tile(red + (kw & 3) * RED_SLOT, acc, rb0, lane);
#pragma unroll
        for (int ph = 1; ph < PKWN / 4; ++ph) {
          __syncthreads();
          if (kw / 4 == ph) add_tile(red + (kw & 3) * RED_SLOT, acc, rb0, lane);
        }
      };
      if (l1) {                                                       // layer 1 at step t - 2
        reduce_put(acc1);
        __syncthreads();
        if (wave < 4) {
          float pre[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) pre[g] = sum(g) + bias1[g];
          out1 = cell(pre, out1.c);
          handoff<BF>(out1.h, a.hk1 + (int64_t)(t - 2) * BH, a.hk1b + (int64_t)(t - 2) * BH, B, eb, ej, lane);
        }
        __syncthreads();
      }
      if (l0) {                                                       // layer 0 at step t
        reduce_put(acc0);
        __syncthreads();
        if (wave < 4) {
          float pre[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) pre[g] = sum(g) + gxv[g];
          out0 = cell(pre, out0.c);
          handoff<BF>(out0.h, a.hk0 + (int64_t)t * BH, a.hk0b + (int64_t)t * BH, B, eb, ej, lane);
        }
      }
      if (t == last2) break;
      grid_arrive(a, xcc_id, xcc_wgs, xcc_n, t);
      // under the barrier: layer 1's input product for its step t - 1 from h0_(t-1)
#pragma unroll
      for (int rb = 0; rb < PRBW; ++rb) acc1[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t >= 1 && t - 1 < T) {
        if constexpr (BF)
          gemm_wave_bf<NS, true, false, false>(a.hk0b + (int64_t)(t - 1) * BH, a.hk1b, whb, W0b, W1b, k8_0, B, rb0,
                                               lane, acc1, acc0);
        else
          gemm_wave<KL, true, false, false>(a.hk0 + (int64_t)(t - 1) * BH, a.hk1, wh, W0, W1, kb0, B, rb0, lane, acc1,
                                            acc0);
      }
      if (!grid_wait(a, xcc_id, status, t)) {
        fail();
        return;
      }
    }
    store_outputs2(last2);
    return;
  }
  const int last = TWO ? T : T - 1;                                 // final iteration
  for (int t = 0; t <= last; ++t) {
    const bool l0 = t < T, l1 = TWO && t >= 1;
    if (t >= 1) store_outputs(t - 1);
    // epilogue operands of this iteration (latency hidden under the products)
    float gxv[4] = {0.f, 0.f, 0.f, 0.f};
    if (eown && l0) {
      const float* g = a.gx0 + (int64_t)eb * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + ej];
    }
    f32x4 acc1[PRBW] = {}, acc0[PRBW] = {};
    const float* hk0 = a.hk0 + (int64_t)(t >= 1 ? t - 1 : 0) * BH;   // h0_{t-1}
    const float* hk1 = a.hk1 + (int64_t)(t >= 2 ? t - 2 : 0) * BH;   // h1_{t-2}
    const __bf16* hk0b = a.hk0b + (int64_t)(t >= 1 ? t - 1 : 0) * BH;
    const __bf16* hk1b = a.hk1b + (int64_t)(t >= 2 ? t - 2 : 0) * BH;
    if (t == 0) {                                                    // h0_{-1} = 0: no products
    } else if constexpr (BF) {
      if (!TWO) gemm_wave_bf<NS, false, true, false>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
      else if (t == 1) gemm_wave_bf<NS, true, true, false>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
      else if (t < T) gemm_wave_bf<NS, true, true, true>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
      else gemm_wave_bf<NS, true, false, true>(hk0b, hk1b, whb, W0b, W1b, k8_0, B, rb0, lane, acc1, acc0);
    } else {
      if (!TWO) gemm_wave<KL, false, true, false>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
      else if (t == 1) gemm_wave<KL, true, true, false>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
      else if (t < T) gemm_wave<KL, true, true, true>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);
      else gemm_wave<KL, true, false, true>(hk0, hk1, wh, W0, W1, kb0, B, rb0, lane, acc1, acc0);   // t == T
    }
    // the 4 waves' partial tiles summed through LDS in fixed order
    auto sum = [&](int layer, int g) {
      const float* r = red + layer * NSLOT * RED_SLOT + eb * RED_LD + g * PU + eu;
      return ((r[0] + r[RED_SLOT]) + r[2 * RED_SLOT]) + r[3 * RED_SLOT];
    };
    // more than 4 waves: wave w < 4 stores its tile into slot w, then waves 4..7 add into
    // slots 0..3, then waves 8..11, ... (fixed order)
    auto reduce_put = [&](float* slots, const f32x4 (&acc)[PRBW]) {
      if (kw < 4) put_tile(slots + (kw & 3) * RED_SLOT, acc, rb0, lane);
#pragma unroll
      for (int ph = 1; ph < PKWN / 4; ++ph) {
        __syncthreads();
        if (kw / 4 == ph) add_tile(slots + (kw & 3) * RED_SLOT, acc, rb0, lane);
      }
    };
    if (TWO) {
      reduce_put(red, acc1);
      __syncthreads();
      if (wave < 4 && l1) {                                        // layer 1 at step t - 1 (eown)
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) pre[g] = sum(0, g) + bias1[g];
        const int t1 = t - 1;
        out1 = cell(pre, out1.c);
        handoff<BF>(out1.h, a.hk1 + (int64_t)t1 * BH, a.hk1b + (int64_t)t1 * BH, B, eb, ej, lane);
      }
      __syncthreads();                                             // slots reused for layer 0
    }
    reduce_put(red, acc0);
    __syncthreads();
    if (wave < 4 && l0) {                                          // layer 0 at step t (eown)
      float pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) pre[g] = sum(0, g) + gxv[g];
      out0 = cell(pre, out0.c);
      handoff<BF>(out0.h, a.hk0 + (int64_t)t * BH, a.hk0b + (int64_t)t * BH, B, eb, ej, lane);
    }
    if (t < last && !grid_sync(a, xcc_id, xcc_wgs, xcc_n, census, status, t)) {
      fail();
      return;
    }
  }
  store_outputs(last);                                               // the final iteration's outputs
}

// ---------------------------------------------------------------- row-split stacked forward
// lstm_persist_kernel gives each workgroup all 64 batch rows x 16 gate columns, so every CU
// streams the whole h0_{t-1} and h1_{t-2} (512 KB fp32) out of L2 every step.  Here the two
// workgroups of a pair split the rows instead (32 rows each) and each owns twice the columns
// (8 units x 4 gates = 32): the same MFMA work per CU, half the per-CU h fill, twice the
// stationary weights — W_hh0's 32 rows in LDS (128 KB fp32, [k/4][32][4]), W_ih1's and W_hh1's
// as MFMA B fragments in VGPRs (128 per lane fp32, 64 bf16).  Wave w = k range w (128 k),
// 2 row blocks x 2 column blocks per wave; the 8 partial tiles summed through LDS in fixed order
// (the k order of lstm_persist_kernel: same sums), cell update by waves 0-3 (thread e: row
// e / 8, unit e % 8).  Iteration structure, barrier, hand-off and fault path are those of
// lstm_persist_kernel (both wavefront forms).
constexpr int RS_ROWS = 32;                 // batch rows per workgroup
constexpr int RS_U = 8;                     // hidden units per workgroup
constexpr int RS_C = 4 * RS_U;              // tile columns
constexpr int RS_RB = RS_ROWS / 16;         // 16-row blocks
constexpr int RS_CB = RS_C / 16;            // 16-column blocks
constexpr int RS_LD = RS_C + 1;             // padded partial-tile row
constexpr int RS_SLOT = RS_ROWS * RS_LD;
static_assert(PNW == 8 && PRH == 1, "row-split form: 8 waves, one k range each");

constexpr int RS_KEEP = 2 * 6 * 256;        // cell outputs kept between iterations: [layer][6][thread]

template <int HH, bool BF>
constexpr int rs_lds_bytes() {
  return (BF ? 2 : 4) * HH * RS_C + 4 * (NSLOT * RS_SLOT + RS_KEEP);
}
static_assert(rs_lds_bytes<1024, false>() <= 160 * 1024, "LDS budget (row split)");

using RsAcc = f32x4[RS_RB][RS_CB];

// fp32 products over this wave's k range.  S0: layer 1's input product (h0_{t-1}, W_ih1 from
// VGPRs), L0: layer 0's recurrent product (h0_{t-1}, W_hh0 from LDS), S1: layer 1's recurrent
// product (h1, W_hh1 from VGPRs).  Lane l: k slot l >> 4 covers k = kbase + 64... as in
// gemm_wave (KL consecutive k per slot), A row r0 + 16 rb + (l & 15), B column 16 cb + (l & 15).
template <int KL, bool S0, bool L0, bool S1>
__device__ __forceinline__ void rs_gemm(const float* __restrict__ hk0_t, const float* __restrict__ hk1_t,
                                        const float (&wi)[RS_CB][KL], const float (&wh)[RS_CB][KL],
                                        const float* W0, int kb0, int B, int r0, int lane, RsAcc& acc1,
                                        RsAcc& acc0) {
  const __amdgpu_buffer_rsrc_t q0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hk0_t), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t q1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hk1_t), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t off0 = (uint32_t)((kb0 * B + r0 + (lane & 15)) * 16);
  const uint32_t gstride = (uint32_t)B * 16;
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int g, int rb) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off0 + g * gstride + rb * 256, 0, 16));
  };
  f32x4 a0[RS_RB], a1[RS_RB];
#pragma unroll
  for (int rb = 0; rb < RS_RB; ++rb) {
    if (S0 || L0) a0[rb] = ld(q0, 0, rb);
    if (S1) a1[rb] = ld(q1, 0, rb);
  }
  const float* w0p = W0 + (kb0 * RS_C + (lane & 15)) * 4;
#pragma unroll
  for (int g = 0; g < KL / 4; ++g) {
    f32x4 x0[RS_RB], x1[RS_RB];
#pragma unroll
    for (int rb = 0; rb < RS_RB; ++rb) {
      x0[rb] = a0[rb];
      x1[rb] = a1[rb];
    }
    if (g + 1 < KL / 4) {
#pragma unroll
      for (int rb = 0; rb < RS_RB; ++rb) {
        if (S0 || L0) a0[rb] = ld(q0, g + 1, rb);
        if (S1) a1[rb] = ld(q1, g + 1, rb);
      }
    }
    f32x4 bv0[RS_CB] = {};
    if (L0)
#pragma unroll
      for (int cb = 0; cb < RS_CB; ++cb) bv0[cb] = *reinterpret_cast<const f32x4*>(w0p + (g * RS_C + 16 * cb) * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
        for (int cb = 0; cb < RS_CB; ++cb) {
          if (S0) acc1[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[rb][q], wi[cb][4 * g + q], acc1[rb][cb], 0, 0, 0);
          if (S1) acc1[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[rb][q], wh[cb][4 * g + q], acc1[rb][cb], 0, 0, 0);
          if (L0) acc0[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[rb][q], bv0[cb][q], acc0[rb][cb], 0, 0, 0);
        }
  }
}

// bf16 products (v_mfma_f32_16x16x32_bf16), operand maps of gemm_wave_bf: lane l supplies the
// 8 k of block k8_0 + 4 st of row r0 + 16 rb + (l & 15); B fragments W_hh0 [H/8][32][8] (LDS),
// W_ih1 / W_hh1 (VGPRs)
template <int NS, bool S0, bool L0, bool S1>
__device__ __forceinline__ void rs_gemm_bf(const __bf16* __restrict__ hk0_t, const __bf16* __restrict__ hk1_t,
                                           const bf16x8 (&wi)[RS_CB][NS], const bf16x8 (&wh)[RS_CB][NS],
                                           const __bf16* W0, int k8_0, int B, int r0, int lane, RsAcc& acc1,
                                           RsAcc& acc0) {
  const __amdgpu_buffer_rsrc_t q0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(hk0_t), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t q1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(hk1_t), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t off0 = (uint32_t)((k8_0 * B + r0 + (lane & 15)) * 16);
  const uint32_t sstride = (uint32_t)B * 64;
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int st, int rb) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off0 + st * sstride + rb * 256, 0, 16));
  };
  bf16x8 a0[RS_RB], a1[RS_RB];
#pragma unroll
  for (int rb = 0; rb < RS_RB; ++rb) {
    if (S0 || L0) a0[rb] = ld(q0, 0, rb);
    if (S1) a1[rb] = ld(q1, 0, rb);
  }
  const __bf16* w0p = W0 + (k8_0 * RS_C + (lane & 15)) * 8;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    bf16x8 x0[RS_RB], x1[RS_RB];
#pragma unroll
    for (int rb = 0; rb < RS_RB; ++rb) {
      x0[rb] = a0[rb];
      x1[rb] = a1[rb];
    }
    if (st + 1 < NS) {
#pragma unroll
      for (int rb = 0; rb < RS_RB; ++rb) {
        if (S0 || L0) a0[rb] = ld(q0, st + 1, rb);
        if (S1) a1[rb] = ld(q1, st + 1, rb);
      }
    }
    bf16x8 bv0[RS_CB] = {};
    if (L0)
#pragma unroll
      for (int cb = 0; cb < RS_CB; ++cb)
        bv0[cb] = *reinterpret_cast<const bf16x8*>(w0p + (st * 4 * RS_C + 16 * cb) * 8);
#pragma unroll
    for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < RS_CB; ++cb) {
        if (S0) acc1[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0[rb], wi[cb][st], acc1[rb][cb], 0, 0, 0);
        if (S1) acc1[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[rb], wh[cb][st], acc1[rb][cb], 0, 0, 0);
        if (L0) acc0[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0[rb], bv0[cb], acc0[rb][cb], 0, 0, 0);
      }
  }
}

// partial tile (acc[rb][cb], C/D map col = lane & 15, row = 4 (lane >> 4) + r) -> LDS slot
template <bool ADD>
__device__ __forceinline__ void rs_tile(float* slot, const RsAcc& acc, int lane) {
#pragma unroll
  for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < RS_CB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* p = slot + (16 * rb + 4 * (lane >> 4) + r) * RS_LD + 16 * cb + (lane & 15);
        if (ADD) *p += acc[rb][cb][r];
        else *p = acc[rb][cb][r];
      }
}

template <int HH, bool BF, bool LAG2>
__global__ __launch_bounds__(PNT, 1) void lstm2_rs_kernel(PArgs a) {
  constexpr int H = HH, KW = HH / PNW, KL = KW / 4, NS = KW / 32;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* W0 = lds;                                          // fp32 [H/4][32][4]
  __bf16* W0b = reinterpret_cast<__bf16*>(lds);             // bf16 [H/8][32][8]
  float* red = lds + (BF ? HH * RS_C / 2 : HH * RS_C);      // NSLOT partial-tile slots
  int* status = reinterpret_cast<int*>(red + RS_C);         // pad column of slot 0's row 0
  // the epilogue threads' cell outputs (c, h, i, f, g, o of both layers) wait in LDS for the
  // next iteration's stores instead of holding 12 VGPRs across the products
  float* keep = red + NSLOT * RS_SLOT;
  int xcc_id = 0, xcc_wgs = 0, xcc_n = 0;
  int census[16] = {};
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware ownership (see lstm_persist_kernel): block b runs on XCD b % 8; that XCD's 32
  // workgroups own 16 consecutive unit blocks of 8 units, two row halves each
  const int nxb = (int)gridDim.x / 8, slot = (int)blockIdx.x / 8;
  const int j0 = ((int)blockIdx.x % 8 * (nxb / 2) + slot / 2) * RS_U;
  const int r0 = (slot & 1) * RS_ROWS;
  auto grow = [&](int col) { return (col >> 3) * H + j0 + (col & 7); };   // tile column -> gate row
  // epilogue ownership: thread e < 256 owns (batch row r0 + e / 8, unit j0 + e % 8)
  const int er = tid >> 3, eu = tid & 7, eb = r0 + er, ej = j0 + eu;
  const bool eown = tid < 4 * 64 && eb < B;
  auto fail = [&]() {
    const float nan = __builtin_nanf("");
    if (eown)
      for (int t = 0; t < T; ++t) {
        a.h0[(int64_t)eb * a.h0_ldb + (int64_t)t * a.h0_ldt + ej] = nan;
        a.c0[((int64_t)eb * T + t) * H + ej] = nan;
        a.h1[((int64_t)eb * T + t) * H + ej] = nan;
        a.c1[((int64_t)eb * T + t) * H + ej] = nan;
      }
    if (tid == 0)
      __hip_atomic_fetch_or(&g_avc_fault, kFaultLstm2Persist, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  if (tid == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 15;
    add_rlx(a.bar + (BAR_CENSUS + xcc) * L, 1);
    add_rlx(a.bar + BAR_START * L, 1);
    const bool ok = wait_ge(a.bar + BAR_START * L, gridDim.x, a.bar + BAR_ERR * L, a.timeout_ticks);
    int nx = 0;
    for (int x = 0; x < 16; ++x) {
      census[x] = ld_rlx(a.bar + (BAR_CENSUS + x) * L);
      nx += census[x] > 0;
    }
    xcc_id = (int)xcc;
    xcc_wgs = ld_rlx(a.bar + (BAR_CENSUS + xcc) * L);
    xcc_n = nx;
    *status = ok ? 0 : 1;
  }
  // ---- weights: W_hh0 -> LDS (k-blocked), W_ih1 / W_hh1 -> VGPRs (B fragments)
  if (BF) {
    for (int e = tid; e < (H / 8) * RS_C; e += PNT) {
      const int kb = e / RS_C, col = e % RS_C;
      *reinterpret_cast<bf16x8*>(W0b + e * 8) = *reinterpret_cast<const bf16x8*>(a.W0b + (int64_t)grow(col) * H + kb * 8);
    }
  } else {
    for (int e = tid; e < (H / 4) * RS_C; e += PNT) {
      const int kb = e / RS_C, col = e % RS_C;
      *reinterpret_cast<f32x4*>(W0 + e * 4) = *reinterpret_cast<const f32x4*>(a.W_hh0 + (int64_t)grow(col) * H + kb * 4);
    }
  }
  const int kw = wave;
  const int kbase = kw * KW + KL * (lane >> 4), kb0 = kbase / 4;
  const int k8_0 = (kw * KW) / 8 + (lane >> 4);
  float wi[RS_CB][BF ? 1 : KL], wh[RS_CB][BF ? 1 : KL];
  bf16x8 wib[RS_CB][BF ? NS : 1], whb[RS_CB][BF ? NS : 1];
#pragma unroll
  for (int cb = 0; cb < RS_CB; ++cb) {
    const int64_t row = (int64_t)grow(16 * cb + (lane & 15)) * H;
    if constexpr (BF) {
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        wib[cb][st] = *reinterpret_cast<const bf16x8*>(a.Wi1b + row + 8 * (k8_0 + 4 * st));
        whb[cb][st] = *reinterpret_cast<const bf16x8*>(a.W1b + row + 8 * (k8_0 + 4 * st));
      }
    } else {
#pragma unroll
      for (int g = 0; g < KL / 4; ++g) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(a.W_ih1 + row + kbase + 4 * g);
        const f32x4 v = *reinterpret_cast<const f32x4*>(a.W_hh1 + row + kbase + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          wi[cb][4 * g + q] = u[q];
          wh[cb][4 * g + q] = v[q];
        }
      }
    }
  }
  if (tid < 256) {                                               // c_{-1} = 0 for both layers
    keep[tid] = 0.f;
    keep[6 * 256 + tid] = 0.f;
  }
  __syncthreads();
  if (*status != 0) {
    fail();
    return;
  }

  float bias1[4] = {0.f, 0.f, 0.f, 0.f};
  if (eown)
#pragma unroll
    for (int g = 0; g < 4; ++g) bias1[g] = a.b_ih1[g * H + ej] + a.b_hh1[g * H + ej];
  const int64_t BH = (int64_t)B * H;
  float* keep_t = keep + (tid & 255);
  auto cell_keep = [&](int layer, const float (&pre)[4]) {      // waves 0-3: returns h
    float* k = keep_t + layer * 6 * 256;
    const CellOut r = cell(pre, k[0]);
    k[0] = r.c; k[256] = r.h; k[512] = r.i; k[768] = r.f; k[1024] = r.g; k[1280] = r.o;
    return r.h;
  };
  auto kept = [&](int layer) {
    const float* k = keep_t + layer * 6 * 256;
    return CellOut{k[0], k[256], k[512], k[768], k[1024], k[1280]};
  };
  // outputs of layer 0 at step t0 and layer 1 at step t1 (either may be out of range)
  auto store = [&](int t0, int t1) {
    if (!eown) return;
    if (t1 >= 0 && t1 < T) {
      const int64_t o = ((int64_t)eb * T + t1) * H + ej;
      cell_store(kept(1), a.c1 + o, a.h1 + o, a.g1 ? a.g1 + ((int64_t)eb * T + t1) * 4 * H + ej : nullptr, H);
    }
    if (t0 >= 0 && t0 < T) {
      const int64_t o = ((int64_t)eb * T + t0) * H + ej;
      cell_store(kept(0), a.c0 + o, a.h0 + (int64_t)eb * a.h0_ldb + (int64_t)t0 * a.h0_ldt + ej,
                 a.g0 ? a.g0 + ((int64_t)eb * T + t0) * 4 * H + ej : nullptr, H);
    }
  };
  auto sum = [&](int g) {
    const float* r = red + er * RS_LD + g * RS_U + eu;
    return ((r[0] + r[RS_SLOT]) + r[2 * RS_SLOT]) + r[3 * RS_SLOT];
  };
  // waves 0-3 store their tiles into slots 0-3, then waves 4-7 add into them (fixed order)
  auto reduce_put = [&](const RsAcc& acc) {
    if (kw < 4) rs_tile<false>(red + kw * RS_SLOT, acc, lane);
    __syncthreads();
    if (kw >= 4) rs_tile<true>(red + (kw - 4) * RS_SLOT, acc, lane);
  };
  // one product call: which of the three products run is a template choice
  auto products = [&](int th0, int th1, bool s0, bool l0, bool s1, RsAcc& acc1, RsAcc& acc0) {
    if constexpr (BF) {
      const __bf16* p0 = a.hk0b + (int64_t)th0 * BH;
      const __bf16* p1 = a.hk1b + (int64_t)th1 * BH;
      if (s0 && l0 && s1) rs_gemm_bf<NS, true, true, true>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (s0 && l0) rs_gemm_bf<NS, true, true, false>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (s0 && s1) rs_gemm_bf<NS, true, false, true>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (l0 && s1) rs_gemm_bf<NS, false, true, true>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (s0) rs_gemm_bf<NS, true, false, false>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (l0) rs_gemm_bf<NS, false, true, false>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
      else if (s1) rs_gemm_bf<NS, false, false, true>(p0, p1, wib, whb, W0b, k8_0, B, r0, lane, acc1, acc0);
    } else {
      const float* p0 = a.hk0 + (int64_t)th0 * BH;
      const float* p1 = a.hk1 + (int64_t)th1 * BH;
      if (s0 && l0 && s1) rs_gemm<KL, true, true, true>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (s0 && l0) rs_gemm<KL, true, true, false>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (s0 && s1) rs_gemm<KL, true, false, true>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (l0 && s1) rs_gemm<KL, false, true, true>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (s0) rs_gemm<KL, true, false, false>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (l0) rs_gemm<KL, false, true, false>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
      else if (s1) rs_gemm<KL, false, false, true>(p0, p1, wi, wh, W0, kb0, B, r0, lane, acc1, acc0);
    }
  };
  auto zero = [](RsAcc& acc) {
#pragma unroll
    for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < RS_CB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // iteration t: layer 0 at step t; layer 1 at step t - LAG (LAG = 2: its input product for
  // step t - 1 runs between this workgroup's arrival at barrier t and the release)
  constexpr int LAG = LAG2 ? 2 : 1;
  const int last = T - 1 + LAG;
  RsAcc acc1c;                                  // LAG2: layer 1's carried input product
  zero(acc1c);
  for (int t = 0; t <= last; ++t) {
    const bool l0 = t < T, l1 = t >= LAG;
    if (t >= 1) store(t - 1, t - 1 - LAG);
    float gxv[4] = {0.f, 0.f, 0.f, 0.f};
    if (eown && l0) {
      const float* g = a.gx0 + (int64_t)eb * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + ej];
    }
    RsAcc acc0, acc1;
    zero(acc0);
    if (LAG2) {
#pragma unroll
      for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
        for (int cb = 0; cb < RS_CB; ++cb) acc1[rb][cb] = acc1c[rb][cb];
    } else {
      zero(acc1);
    }
    // h0_{t-1} feeds layer 0 (t >= 1) and, one-step form, layer 1's input product (1 <= t <= T);
    // h1_{t-1-LAG} feeds layer 1's recurrent product (t - 1 - LAG >= 0, layer 1 running)
    const bool pl0 = l0 && t >= 1, ps0 = !LAG2 && l1, ps1 = l1 && t - 1 - LAG >= 0;
    products(t >= 1 ? t - 1 : 0, t - 1 - LAG >= 0 ? t - 1 - LAG : 0, ps0, pl0, ps1, acc1, acc0);
    if (l1) {                                                      // layer 1 at step t - LAG
      reduce_put(acc1);
      __syncthreads();
      if (wave < 4) {
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) pre[g] = sum(g) + bias1[g];
        handoff<BF>(cell_keep(1, pre), a.hk1 + (int64_t)(t - LAG) * BH, a.hk1b + (int64_t)(t - LAG) * BH, B, eb, ej,
                    lane);
      }
      __syncthreads();                                             // slots reused for layer 0
    }
    if (l0) {                                                      // layer 0 at step t
      reduce_put(acc0);
      __syncthreads();
      if (wave < 4) {
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) pre[g] = sum(g) + gxv[g];
        handoff<BF>(cell_keep(0, pre), a.hk0 + (int64_t)t * BH, a.hk0b + (int64_t)t * BH, B, eb, ej, lane);
      }
    }
    if (t == last) break;
    if constexpr (LAG2) {
      grid_arrive(a, xcc_id, xcc_wgs, xcc_n, t);
      zero(acc1c);                                                 // under the barrier:
      if (t >= 1 && t - 1 < T) {                                   // layer 1's input product
        RsAcc dummy;                                               // for its step t - 1
        products(t - 1, 0, true, false, false, acc1c, dummy);
      }
      if (!grid_wait(a, xcc_id, status, t)) {
        fail();
        return;
      }
    } else if (!grid_sync(a, xcc_id, xcc_wgs, xcc_n, census, status, t)) {
      fail();
      return;
    }
  }
  store(last, last - LAG);
}

int g_cus = -1;

// one workgroup of the <HH, TWO> kernel must fit on a CU, and every workgroup must be resident
// at once: no more workgroups (HH / PU) than CUs
template <int HH, bool TWO, bool BF = false>
bool persist_fits() {
  static int per = -1;
  if (per < 0) {
    per = 0;
    const void* k = reinterpret_cast<const void*>(lstm_persist_kernel<HH, TWO, BF>);
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<HH, TWO, BF>()) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lstm_persist_kernel<HH, TWO, BF>, PNT,
                                                     lds_bytes<HH, TWO, BF>()) != hipSuccess)
      per = 0;
    int per2 = 0;                         // the two-step wavefront form must fit the same way
    const void* k2 = reinterpret_cast<const void*>(lstm_persist_kernel<HH, TWO, BF, true>);
    if (TWO && (hipFuncSetAttribute(k2, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<HH, TWO, BF>()) !=
                    hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, lstm_persist_kernel<HH, TWO, BF, true>, PNT,
                                                             lds_bytes<HH, TWO, BF>()) != hipSuccess ||
                per2 < 1))
      per = 0;
  }
  if (g_cus < 0) {
    int dev = 0;
    hipDeviceProp_t p;
    g_cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
                ? p.multiProcessorCount : 0;
  }
  return per >= 1 && HH / PU <= g_cus;
}

// The two-step wavefront of the stacked forward (LAG2 above): the fp32 default (20.7-21.0 ->
// 18.1-18.2 us per wavefront step, 15.39 -> 14.99 ms per training step, alternating on one box:
// profiles/r03/ab_lstm2_lag2.txt); not under bf16, whose 8x cheaper products leave the
// barrier nothing to hide and the second h0 read costs (10.5 -> 14.1 us).  AVC_LSTM2_LAG2=0 /
// =1 forces it off / on for both; read per launch (one per forward), so tests compare both.
// Under the row split (lstm2_rs_kernel, half the h fill per CU) the two-step form wins for
// bf16 too: 8.2-8.3 -> 7.3 us per wavefront step (profiles/r04/lstm2_rs_ab.txt).
bool lag2_on(bool bf, bool rs = false) {
  const char* e = getenv("AVC_LSTM2_LAG2");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return rs || !bf;
}

// The row-split stacked forward (lstm2_rs_kernel), the default: AVC_LSTM2_RS=0 selects
// lstm_persist_kernel instead (read per launch); it runs only where one workgroup per CU fits
// and B is two row halves.  fp32 15.8-15.9 -> 15.0-15.1 us per wavefront step, 14.66 -> 14.57
// ms per training step (profiles/r04/lstm2_rs_ab.txt); bit-identical outputs.
template <bool BF>
bool rs_fits() {
  static int per = -1;
  if (per < 0) {
    per = 1;
    for (int lag = 0; lag < 2 && per > 0; ++lag) {
      const void* k = lag ? reinterpret_cast<const void*>(lstm2_rs_kernel<1024, BF, true>)
                          : reinterpret_cast<const void*>(lstm2_rs_kernel<1024, BF, false>);
      int n = 0;
      if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, rs_lds_bytes<1024, BF>()) != hipSuccess ||
          (lag ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, lstm2_rs_kernel<1024, BF, true>, PNT,
                                                             rs_lds_bytes<1024, BF>())
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, lstm2_rs_kernel<1024, BF, false>, PNT,
                                                             rs_lds_bytes<1024, BF>())) != hipSuccess ||
          n < 1)
        per = 0;
    }
  }
  return per >= 1 && 2 * 1024 / RS_U <= g_cus;
}

bool rs_on() {
  const char* e = getenv("AVC_LSTM2_RS");
  return !(e && e[0] == '0');
}

template <int HH, bool TWO, bool BF = false>
void launch_persist(PArgs& a, void* workspace, hipStream_t stream) {
  a.bar = static_cast<int*>(workspace);
  a.hk0 = reinterpret_cast<float*>(static_cast<char*>(workspace) + BAR_BYTES);
  a.hk1 = TWO ? a.hk0 + (int64_t)a.T * a.B * HH : nullptr;
  a.hk0b = reinterpret_cast<__bf16*>(a.hk0);
  a.hk1b = TWO ? a.hk0b + (int64_t)a.T * a.B * HH : nullptr;
  // 1 s of s_memrealtime (100 MHz) per wait: a safety net, never a schedule
  a.timeout_ticks = g_timeout_ticks > 0 ? g_timeout_ticks : 100000000;
  if constexpr (TWO && HH == 1024) {
    if (rs_on() && a.B == 2 * RS_ROWS && rs_fits<BF>()) {
      const dim3 grid(2 * HH / RS_U);
      if (lag2_on(BF, true))
        hipLaunchKernelGGL((lstm2_rs_kernel<HH, BF, true>), grid, dim3(PNT), (rs_lds_bytes<HH, BF>()), stream, a);
      else
        hipLaunchKernelGGL((lstm2_rs_kernel<HH, BF, false>), grid, dim3(PNT), (rs_lds_bytes<HH, BF>()), stream, a);
      return;
    }
  }
  if (TWO && lag2_on(BF))
    hipLaunchKernelGGL((lstm_persist_kernel<HH, TWO, BF, true>), dim3(HH / PU), dim3(PNT), (lds_bytes<HH, TWO, BF>()),
                       stream, a);
  else
    hipLaunchKernelGGL((lstm_persist_kernel<HH, TWO, BF>), dim3(HH / PU), dim3(PNT), (lds_bytes<HH, TWO, BF>()), stream,
                       a);
}

// ================================================================ XCD-local recurrences
// Decoder lstm1 (nn.LSTM(2*dim_neck + dim_emb, 512), model_vc_mel.py:90,111) as ONE
// persistent launch whose synchronisation never leaves an XCD.  The batch rows of a step are
// independent sequences, so XCD x (its 32 CUs, its own L2) owns batch rows 8x .. 8x+7 for the
// whole sequence: its 32 workgroups (slot s = 0..31, one per CU) hold a replica of W_hh's
// columns for units 16s .. 16s+15 (4 gates x 16 units x H = 128 KB fp32, in VGPRs as MFMA A
// fragments), and per step only the 8 rows of h_{t-1} (16 KB) move, written and read inside
// the XCD's L2: plain stores (kept in L2), sc1 loads (L1 bypassed, L2-served), and a per-XCD
// step counter advanced by workgroup-scope atomics — executed in that L2, the coherence point
// of every CU of the XCD — instead of a chip-wide barrier (lstm2_persist's costs ~2.8 us, a
// launch boundary ~1.5 us).  Workgroups learn their XCD from HW_REG_XCC_ID and take slots
// from a per-XCD counter, so any dispatch order works; a group that does not get exactly 32
// workgroups (another partition mode, a second process's kernels) times out into the fault
// path below (NaN over the outputs, device fault word, autovc_fault_status).
// Products: v_mfma_f32_16x16x4_f32 with A = 16 gate columns x 4 k (W, registers) and B = 4 k
// x 16 batch lanes, of which the group's 8 rows are real (the other 8 read a zero row):
// 128 MFMAs per wave per step (wave w = gate w), k split as 4 lane groups x 128 consecutive k.
constexpr int XRB = 8;                 // batch rows per XCD group
constexpr int XNX = 8;                 // groups = XCDs
constexpr int XSL = 32;                // workgroups (slots) per group
constexpr int XNT = 256;               // 4 waves
// barrier block (ints, one 128-B line per word): census and step counters per XCD, error word
constexpr int XC_CENSUS = 0, XC_STEP = 16, XC_ERR = 32, XC_LINES = 33;
constexpr int64_t XC_BYTES = XC_LINES * L * 4;
constexpr int XC_PAD_LDS = 96 * 1024;  // dynamic LDS that keeps one workgroup per CU

struct XArgs {
  int B, T;
  const float* gx;
  int64_t gx_ldb, gx_ldt;
  const float* W;            // W_hh (4H, H)
  const __bf16* Wb;          // its RNE bf16 copy (BF)
  float *h, *c, *g;          // h (b*h_ldb + t*h_ldt), c (B,T,H), gates (B,T,4H) or null
  int64_t h_ldb, h_ldt;
  int* bar;
  int timeout_ticks;
};

__device__ __forceinline__ int add_l2(int* p, int v) {
  // every adder and poller of this word runs on ONE XCD: the add is performed in its L2
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// BF: the recurrent product on bf16 copies (autovc_lstm_fwd_bf16's numerics: RNE W_hh and h,
// fp32 accumulation, fp32 cell math and outputs) with v_mfma_f32_16x16x32_bf16: 16 MFMAs per
// wave per step instead of 128.
template <int HH, bool BF>
__global__ __launch_bounds__(XNT, 1) void lstm_xcd_fwd_kernel(XArgs a) {
  constexpr int U = HH / XSL;            // units per slot
  constexpr int KG = HH / 4;             // k per MFMA lane group
  constexpr int HS = HH + 4;             // LDS row stride of the staged h rows (bank spread)
  static_assert(U == 16, "one 16-column MFMA tile per gate");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int HSB = HH + 8;            // bf16 row stride
  float* hs = lds;                        // [XRB + 1][HS], row XRB = zeros
  __bf16* hsb = reinterpret_cast<__bf16*>(lds);   // BF: [XRB + 1][HSB]
  float* pre = lds + (XRB + 1) * HS;      // [4 gates][U][XRB + 1]
  __shared__ int s_info[3];               // xcc, slot, status
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T;
  if (tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    const int xcc = (int)(x & 15);
    const int slot = add_rlx(a.bar + (XC_CENSUS + xcc) * L, 1);
    s_info[0] = xcc;
    s_info[1] = slot;
    s_info[2] = (xcc < XNX && slot < XSL) ? 0 : 1;
    if (s_info[2]) st_rlx(a.bar + XC_ERR * L, 1);
  }
  for (int i = tid; i < HS; i += XNT) hs[XRB * HS + i] = 0.f;
  if (BF)
    for (int i = tid; i < HSB; i += XNT) hsb[XRB * HSB + i] = (__bf16)0.f;
  __syncthreads();
  const int xcc = s_info[0] < XNX ? s_info[0] : 0, slot = s_info[1] < XSL ? s_info[1] : 0;
  const int r0 = XRB * xcc, u0 = U * slot;
  // cell ownership: threads 0..127 own (row tid / 16, unit tid % 16) for the whole sequence
  const int cb = tid >> 4, cu = tid & 15;
  const bool cown = tid < XRB * U;
  auto fail = [&]() {
    const float nan = __builtin_nanf("");
    if (cown)
      for (int t = 0; t < T; ++t) {
        a.h[(int64_t)(r0 + cb) * a.h_ldb + (int64_t)t * a.h_ldt + u0 + cu] = nan;
        a.c[((int64_t)(r0 + cb) * T + t) * HH + u0 + cu] = nan;
      }
    if (tid == 0) __hip_atomic_fetch_or(&g_avc_fault, kFaultLstmXcdFwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (s_info[2]) {
    if (s_info[0] < XNX && s_info[1] < XSL) fail();   // an in-range slot of a failed group
    if (tid == 0) __hip_atomic_fetch_or(&g_avc_fault, kFaultLstmXcdFwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // W fragments: wave = gate, lane -> column u0 + lane % 16, k = 128 (lane / 16) + q
  float wf[BF ? 1 : KG];
  bf16x8 wb[BF ? KG / 8 : 1];
  if constexpr (BF) {
    // k of MFMA q, lane group g, element e: KG g + 8 q + e (A and B alike)
    const __bf16* src = a.Wb + (int64_t)(wave * HH + u0 + (lane & 15)) * HH + KG * (lane >> 4);
#pragma unroll
    for (int q = 0; q < KG / 8; ++q) wb[q] = *reinterpret_cast<const bf16x8*>(src + 8 * q);
  } else {
    const float* src = a.W + (int64_t)(wave * HH + u0 + (lane & 15)) * HH + KG * (lane >> 4);
#pragma unroll
    for (int q = 0; q < KG; q += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + q);
      wf[q] = v[0]; wf[q + 1] = v[1]; wf[q + 2] = v[2]; wf[q + 3] = v[3];
    }
  }
  // B rows of this lane: its batch row of the staged h, or the zero row
  const int hsel = ((lane & 15) < XRB) ? (lane & 15) : XRB;
  [[maybe_unused]] const float* hrow = hs + hsel * HS + KG * (lane >> 4);
  [[maybe_unused]] const __bf16* hrowb = hsb + hsel * HSB + KG * (lane >> 4);
  float cst = 0.f;                        // cell state (cown)
  float cell_out[5];
  float gxv[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_gx = [&](int t) {
    const float* g = a.gx + (int64_t)(r0 + cb) * a.gx_ldb + (int64_t)t * a.gx_ldt + u0 + cu;
#pragma unroll
    for (int q = 0; q < 4; ++q) gxv[q] = g[q * HH];
  };
  if (cown) load_gx(0);
  int* step_ctr = a.bar + (XC_STEP + xcc) * L;
  for (int t = 0; t < T; ++t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (t > 0) {
      // ---- XCD barrier: all 32 slots stored h_{t-1}
      if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_rlx(step_ctr) < XSL * t) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)a.timeout_ticks || ld_rlx(a.bar + XC_ERR * L)) {
            st_rlx(a.bar + XC_ERR * L, 1);
            ok = 0;
            break;
          }
        }
        s_info[2] = ok ? 0 : 1;
      }
      __syncthreads();
      if (s_info[2]) {
        fail();
        return;
      }
      // ---- stage h_{t-1} of the group's 8 rows (sc1 loads: L1 bypassed, L2-served)
      {
        // wave-instruction i of wave w moves 1 KB chunk 4w + i of the 8 rows (whole lines per
        // instruction): row (4w + i) / (HH / 256), floats 256 ((4w + i) % (HH / 256)) + 4 lane
        constexpr int NI = XRB * HH / 256 / 4;     // b128 loads per lane
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            a.h + (int64_t)r0 * a.h_ldb + (int64_t)(t - 1) * a.h_ldt, (short)0, 0x7fffffff, 0x00020000);
        f32x4 v[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int ch = NI * wave + i, row = ch / (HH / 256), k = 256 * (ch % (HH / 256)) + 4 * lane;
          v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               r, (uint32_t)(((int64_t)row * a.h_ldb + k) * 4), 0, 16));
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int ch = NI * wave + i, row = ch / (HH / 256), k = 256 * (ch % (HH / 256)) + 4 * lane;
          if constexpr (BF)
            *reinterpret_cast<bf16x4*>(hsb + row * HSB + k) =
                bf16x4{(__bf16)v[i][0], (__bf16)v[i][1], (__bf16)v[i][2], (__bf16)v[i][3]};
          else
            *reinterpret_cast<f32x4*>(hs + row * HS + k) = v[i];
        }
      }
      __syncthreads();
      if constexpr (BF) {
#pragma unroll
        for (int q = 0; q < KG / 8; ++q)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[q], *reinterpret_cast<const bf16x8*>(hrowb + 8 * q), acc,
                                                        0, 0, 0);
      } else {
#pragma unroll
        for (int q = 0; q < KG; q += 4) {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(hrow + q);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q], bv[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q + 1], bv[1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q + 2], bv[2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q + 3], bv[3], acc, 0, 0, 0);
        }
      }
    }
    if ((lane & 15) < XRB) {
      // C[unit 4 (lane / 16) + r][batch lane % 16] of gate `wave`
#pragma unroll
      for (int r = 0; r < 4; ++r) pre[(wave * U + 4 * (lane >> 4) + r) * (XRB + 1) + (lane & 15)] = acc[r];
    }
    __syncthreads();
    if (cown) {
      float p[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = pre[(q * U + cu) * (XRB + 1) + cb] + gxv[q];
      const float i_ = avc_sigmoid_fast(p[0]), f_ = avc_sigmoid_fast(p[1]), g_ = avc_tanh_fast(p[2]);
      const float o_ = avc_sigmoid_fast(p[3]);
      cst = f_ * cst + i_ * g_;
      const float hn = o_ * avc_tanh_fast(cst);
      a.h[(int64_t)(r0 + cb) * a.h_ldb + (int64_t)t * a.h_ldt + u0 + cu] = hn;
      cell_out[0] = cst; cell_out[1] = i_; cell_out[2] = f_; cell_out[3] = g_; cell_out[4] = o_;
    }
    // ---- arrive once h_t (only it) is in the XCD's L2; c / gates and the next gx loads
    // go out after the arrive, under the next step's wait
    if (t + 1 < T) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) add_l2(step_ctr, 1);
    }
    if (cown) {
      const int64_t bt = (int64_t)(r0 + cb) * T + t;
      a.c[bt * HH + u0 + cu] = cell_out[0];
      if (a.g) {
        float* gs = a.g + bt * 4 * HH + u0 + cu;
        gs[0] = cell_out[1]; gs[HH] = cell_out[2]; gs[2 * HH] = cell_out[3]; gs[3 * HH] = cell_out[4];
      }
      if (t + 1 < T) load_gx(t + 1);
    }
  }
}

// Backward of the same layer (BPTT, reverse time), same XCD split, in one launch: slot s of
// XCD x owns units 16s .. 16s+15 of batch rows 8x .. 8x+7 — the cells whose gate gradients
// it writes and the 16 columns of dh_rec(t) = dG_{t+1} W_hh (K = 4H = 2048) it reduces.
// W_hh's 16 columns stay in registers as MFMA A fragments (from the (H, 4H) transpose the
// per-step path reads too); each wave takes a quarter of K and stages its slice of the
// group's 8 dG_{t+1} rows (written by the XCD's 32 slots into its L2) through LDS with
// coalesced sc1 loads, the 4 partial tiles are summed in LDS in fixed order, then the cell
// math of lstm.hip pw_finish.  BF: the product on the bf16 copies (autovc_lstm_bwd_bf16's
// numerics: RNE W_hh^T and dG, fp32 accumulation) — the exchange moves the bf16 dG rows
// (half the bytes), 16 MFMAs per wave per step instead of 128.
// (Round 3 measured the fp32 form alone at 4.2 vs 9.3 us per step but slower in the training
// step of that schedule; profiles/r06/ab_lstm1_xcd_bwd.txt re-measures it in this one.)
struct XBArgs {
  int B, T;
  const float* dh;           // dh_out (b*d_ldb + t*d_ldt), may be null
  int64_t d_ldb, d_ldt;
  const float* gates;        // (B,T,4H) i, f, g, o
  const float* c;            // (B,T,H)
  const float* WT;           // W_hh^T (H, 4H) fp32
  const __bf16* WTb;         // its RNE bf16 copy (BF)
  float* dG;                 // (B,T,4H)
  __bf16* dGb;               // (B,T,4H) bf16 copy (BF: required, the exchanged operand)
  int* bar;
  int timeout_ticks;
};

template <int HH, bool BF>
__global__ __launch_bounds__(XNT, 1) void lstm_xcd_bwd_kernel(XBArgs a) {
  constexpr int U = HH / XSL;            // units per slot (16)
  constexpr int K4 = 4 * HH;             // recurrent K
  constexpr int KW = K4 / 4;             // k per wave
  constexpr int KG = KW / 4;             // k per MFMA lane group (consecutive)
  static_assert(U == 16, "tile shape");
  // slab row stride in elements (bank spread).  fp32: the wave's K quarter arrives in two
  // rounds of half the k (each lane group's 128 k as two 64-k chunks), so the slab holds 256 k
  // per row: 41 KB of LDS per workgroup instead of 77, room for a GEMM workgroup beside it
  constexpr int SS = BF ? KW + 8 : KW / 2 + 4;
  using E = typename std::conditional<BF, __bf16, float>::type;
  static_assert(4 * U * (XRB + 1) * 4 + 4 * (XRB + 1) * SS * (int)sizeof(E) <= XC_PAD_LDS, "LDS budget");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* part = lds;                      // [4 waves][U][XRB + 1]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  E* slab = reinterpret_cast<E*>(lds + 4 * U * (XRB + 1)) + wave * (XRB + 1) * SS;   // row XRB = 0
  __shared__ int s_info[3];
  const int T = a.T;
  if (tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    const int xcc = (int)(x & 15);
    const int slot = add_rlx(a.bar + (XC_CENSUS + xcc) * L, 1);
    s_info[0] = xcc;
    s_info[1] = slot;
    s_info[2] = (xcc < XNX && slot < XSL) ? 0 : 1;
    if (s_info[2]) st_rlx(a.bar + XC_ERR * L, 1);
  }
  for (int i = lane; i < SS; i += 64) slab[XRB * SS + i] = (E)0.f;
  __syncthreads();
  const int xcc = s_info[0] < XNX ? s_info[0] : 0, slot = s_info[1] < XSL ? s_info[1] : 0;
  const int r0 = XRB * xcc, u0 = U * slot;
  const int cb = tid >> 4, cu = tid & 15;
  const bool cown = tid < XRB * U;
  const int64_t cell0 = (int64_t)(r0 + cb) * T;     // (b, t) row base of this cell's batch row
  auto fail = [&]() {
    const float nan = __builtin_nanf("");
    if (cown)
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a.dG[(cell0 + t) * K4 + q * HH + u0 + cu] = nan;
          if (a.dGb) a.dGb[(cell0 + t) * K4 + q * HH + u0 + cu] = (__bf16)nan;
        }
    if (tid == 0) __hip_atomic_fetch_or(&g_avc_fault, kFaultLstmXcdBwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (s_info[2]) {
    if (s_info[0] < XNX && s_info[1] < XSL) fail();
    if (tid == 0) __hip_atomic_fetch_or(&g_avc_fault, kFaultLstmXcdBwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // A fragments: lane -> unit u0 + lane % 16, k = KW wave + KG (lane / 16) + q (B alike)
  const int kbase = KW * wave + KG * (lane >> 4);
  float wf[BF ? 1 : KG];
  bf16x8 wb[BF ? KG / 8 : 1];
  if constexpr (BF) {
    const __bf16* src = a.WTb + (int64_t)(u0 + (lane & 15)) * K4 + kbase;
#pragma unroll
    for (int q = 0; q < KG / 8; ++q) wb[q] = *reinterpret_cast<const bf16x8*>(src + 8 * q);
  } else {
    const float* src = a.WT + (int64_t)(u0 + (lane & 15)) * K4 + kbase;
#pragma unroll
    for (int q = 0; q < KG; q += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + q);
      wf[q] = v[0]; wf[q + 1] = v[1]; wf[q + 2] = v[2]; wf[q + 3] = v[3];
    }
  }
  const bool bvalid = (lane & 15) < XRB;
  const E* brow = slab + (bvalid ? (lane & 15) : XRB) * SS + (BF ? KG : KG / 2) * (lane >> 4);
  // pointwise operands of step t (prefetched one step ahead)
  f32x4 gt = {0.f, 0.f, 0.f, 0.f};
  float cc = 0.f, cpv = 0.f, dho = 0.f, dcs = 0.f;
  auto load_pw = [&](int t) {
    const float* g = a.gates + (cell0 + t) * K4 + u0 + cu;
#pragma unroll
    for (int q = 0; q < 4; ++q) gt[q] = g[q * HH];
    cc = a.c[(cell0 + t) * HH + u0 + cu];
    cpv = t > 0 ? a.c[(cell0 + t - 1) * HH + u0 + cu] : 0.f;
    dho = a.dh ? a.dh[(int64_t)(r0 + cb) * a.d_ldb + (int64_t)t * a.d_ldt + u0 + cu] : 0.f;
  };
  if (cown) load_pw(T - 1);
  int* step_ctr = a.bar + (XC_STEP + xcc) * L;
  for (int s = 0; s < T; ++s) {
    const int t = T - 1 - s;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      // ---- XCD barrier: all 32 slots stored dG_{t+1}
      if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_rlx(step_ctr) < XSL * s) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)a.timeout_ticks || ld_rlx(a.bar + XC_ERR * L)) {
            st_rlx(a.bar + XC_ERR * L, 1);
            ok = 0;
            break;
          }
        }
        s_info[2] = ok ? 0 : 1;
      }
      __syncthreads();
      if (s_info[2]) {
        fail();
        return;
      }
      // ---- this wave's K quarter of the group's dG_{t+1} rows -> its LDS slab: coalesced sc1
      // loads (whole lines per instruction: L1 is bypassed, so scattered fragment loads would
      // re-fetch every line), then the products dh_rec = dG_{t+1} W_hh from LDS
      if constexpr (!BF) {
        // load i = 8 h + r: row r, round h; lane group g = lane / 16 takes the 16 float4 of its
        // chunk k = KG g + 64 h + 4 (lane % 16) .. +3 (256 contiguous bytes per lane group)
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.dG + ((int64_t)r0 * T + t + 1) * K4 + KW * wave), (short)0, 0x7fffffff, 0x00020000);
        f32x4 v[2 * XRB];
        const int kl = KG * (lane >> 4) + 4 * (lane & 15);
#pragma unroll
        for (int i = 0; i < 2 * XRB; ++i) {
          const int row = i % XRB, h = i / XRB;
          v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               r, (uint32_t)(((int64_t)row * T * K4 + kl + 64 * h) * 4), 0, 16));
        }
        float* sl = reinterpret_cast<float*>(slab) + (KG / 2) * (lane >> 4) + 4 * (lane & 15);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int row = 0; row < XRB; ++row) *reinterpret_cast<f32x4*>(sl + row * SS) = v[h * XRB + row];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int q = 0; q < KG / 2; q += 4) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(brow + q);
            const int w0 = (KG / 2) * h + q;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[w0], bv[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[w0 + 1], bv[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[w0 + 2], bv[2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[w0 + 3], bv[3], acc, 0, 0, 0);
          }
          // (the next round's writes follow this wave's own slab reads in program order)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
        }
      } else {
        constexpr int CPR = KW * (int)sizeof(E) / 16;    // 16-B chunks per row slice
        constexpr int NL = XRB * CPR / 64;               // b128 loads per lane
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<__bf16*>(a.dGb + ((int64_t)r0 * T + t + 1) * K4 + KW * wave), (short)0, 0x7fffffff, 0x00020000);
        f32x4 v[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int ci = i * 64 + lane, row = ci / CPR, k16 = ci % CPR;
          v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               r, (uint32_t)((int64_t)row * T * K4 * (int)sizeof(E) + 16 * k16), 0,
                                               16));
        }
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int ci = i * 64 + lane, row = ci / CPR, k16 = ci % CPR;
          *reinterpret_cast<f32x4*>(slab + row * SS + k16 * (16 / (int)sizeof(E))) = v[i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
      if constexpr (BF) {
#pragma unroll
        for (int q = 0; q < KG / 8; ++q)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[q], *reinterpret_cast<const bf16x8*>(brow + 8 * q), acc, 0,
                                                        0, 0);
      }
    }
    // C[unit 4 (lane / 16) + r][batch lane % 16]: the 4 waves' K quarters, summed in order
    if (bvalid)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(wave * U + 4 * (lane >> 4) + r) * (XRB + 1) + (lane & 15)] = acc[r];
    __syncthreads();
    float dgo[4];
    if (cown) {
#pragma clang fp contract(off)
      const float dh = dho + (((part[(0 * U + cu) * (XRB + 1) + cb] + part[(1 * U + cu) * (XRB + 1) + cb]) +
                               part[(2 * U + cu) * (XRB + 1) + cb]) + part[(3 * U + cu) * (XRB + 1) + cb]);
      const float i_ = gt[0], f_ = gt[1], g_ = gt[2], o_ = gt[3];
      const float tc = tanhf(cc);
      const float dc = dcs + dh * o_ * (1.f - tc * tc);
      dgo[0] = dc * g_ * i_ * (1.f - i_);
      dgo[1] = dc * cpv * f_ * (1.f - f_);
      dgo[2] = dc * i_ * (1.f - g_ * g_);
      dgo[3] = dh * tc * o_ * (1.f - o_);
      dcs = dc * f_;
      // the exchanged copy first (fp32: dG, BF: dGb); the other after the arrive
      if constexpr (BF) {
        __bf16* db = a.dGb + (cell0 + t) * K4 + u0 + cu;
#pragma unroll
        for (int q = 0; q < 4; ++q) db[q * HH] = (__bf16)dgo[q];
      } else {
        float* d = a.dG + (cell0 + t) * K4 + u0 + cu;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q * HH] = dgo[q];
      }
    }
    if (s + 1 < T) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) add_l2(step_ctr, 1);
    }
    if (cown) {
      if constexpr (BF) {
        float* d = a.dG + (cell0 + t) * K4 + u0 + cu;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q * HH] = dgo[q];
      }
      if (s + 1 < T) load_pw(t - 1);
    }
  }
}

int g_xcd_ok = -1;
// dynamic LDS of the backward launch: just over half a CU's 160 KB (one workgroup per CU) while
// leaving room for one X6 / fp32 GEMM workgroup beside it (12.43 vs 12.69-12.71 ms/step with the
// forward's 96 KB pad: profiles/r06/ab_lstm1_xcd_bwd_x6.txt)
// (With the fp32 slab halved the kernel needs 39.7 KB; requesting only that — so that the side
// GEMM workgroups co-reside — measured the same step, 12.51-12.53 vs 12.52-12.55 ms:
// profiles/r06/ab_xcd_bwd_lds.txt.)
constexpr int kXcdBwdLds = 82432;
int xcd_bwd_lds() { return kXcdBwdLds; }

bool xcd_fits() {
  if (g_xcd_ok < 0) {
    int dev = 0, per = 0;
    hipDeviceProp_t p;
    const void* k = reinterpret_cast<const void*>(lstm_xcd_fwd_kernel<512, false>);
    const int lb = XC_PAD_LDS;
    g_xcd_ok = hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess &&
               p.multiProcessorCount == XNX * XSL &&
               hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lb) == hipSuccess &&
               hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lstm_xcd_fwd_kernel<512, false>, XNT, lb) == hipSuccess &&
               per >= 1 &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_xcd_fwd_kernel<512, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lb) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_xcd_bwd_kernel<512, false>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lb) == hipSuccess &&
               hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lstm_xcd_bwd_kernel<512, false>, XNT, lb) ==
                   hipSuccess &&
               per >= 1 &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_xcd_bwd_kernel<512, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lb) == hipSuccess;
  }
  return g_xcd_ok == 1;
}


}  // namespace

extern "C" int autovc_lstm_xcd_supported(int B, int H) {
  return (B == XRB * XNX && H == 512 && xcd_fits()) ? 1 : 0;
}

extern "C" int64_t autovc_lstm_xcd_workspace_bytes(void) { return XC_BYTES; }

extern "C" int autovc_lstm_fwd_xcd_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                       const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                       float* gates, void* workspace, hipStream_t stream) {
  static const char* fn = "autovc_lstm_fwd_xcd_f32";
  AVC_CHECK_ARG(T > 0 && autovc_lstm_xcd_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs B=64, H=512, 8 XCDs x 32 CUs)", fn, B, H);
  AVC_CHECK_ARG(gx && W_hh && h && c_all && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh) && AVC_ALIGNED16(workspace), "%s: W_hh / workspace must be 16-byte aligned", fn);
  XArgs a;
  a.B = B; a.T = T; a.gx = gx; a.gx_ldb = gx_ldb; a.gx_ldt = gx_ldt; a.W = W_hh; a.Wb = nullptr;
  a.h = h; a.c = c_all; a.g = gates; a.h_ldb = h_ldb; a.h_ldt = h_ldt;
  a.bar = static_cast<int*>(workspace);
  a.timeout_ticks = g_timeout_ticks > 0 ? g_timeout_ticks : 100000000;
  AVC_HIP(avc::zero_async(workspace, XC_BYTES, stream), fn);
  hipLaunchKernelGGL((lstm_xcd_fwd_kernel<512, false>), dim3(XNX * XSL), dim3(XNT), XC_PAD_LDS, stream, a);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int autovc_lstm_fwd_xcd_bf16(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                        const uint16_t* W_hh_b, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                        float* gates, void* workspace, hipStream_t stream) {
  static const char* fn = "autovc_lstm_fwd_xcd_bf16";
  AVC_CHECK_ARG(T > 0 && autovc_lstm_xcd_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs B=64, H=512, 8 XCDs x 32 CUs)", fn, B, H);
  AVC_CHECK_ARG(gx && W_hh_b && h && c_all && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_b) && AVC_ALIGNED16(workspace), "%s: W_hh_b / workspace must be 16-byte aligned",
                fn);
  XArgs a;
  a.B = B; a.T = T; a.gx = gx; a.gx_ldb = gx_ldb; a.gx_ldt = gx_ldt; a.W = nullptr;
  a.Wb = reinterpret_cast<const __bf16*>(W_hh_b);
  a.h = h; a.c = c_all; a.g = gates; a.h_ldb = h_ldb; a.h_ldt = h_ldt;
  a.bar = static_cast<int*>(workspace);
  a.timeout_ticks = g_timeout_ticks > 0 ? g_timeout_ticks : 100000000;
  AVC_HIP(avc::zero_async(workspace, XC_BYTES, stream), fn);
  hipLaunchKernelGGL((lstm_xcd_fwd_kernel<512, true>), dim3(XNX * XSL), dim3(XNT), XC_PAD_LDS, stream, a);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int autovc_lstm_bwd_xcd_f32(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                                       const float* gates, const float* c_all, const float* WT, float* dG,
                                       void* workspace, hipStream_t stream) {
  static const char* fn = "autovc_lstm_bwd_xcd_f32";
  AVC_CHECK_ARG(T > 0 && autovc_lstm_xcd_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs B=64, H=512, 8 XCDs x 32 CUs)", fn, B, H);
  AVC_CHECK_ARG(gates && c_all && WT && dG && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(WT) && AVC_ALIGNED16(dG) && AVC_ALIGNED16(workspace),
                "%s: WT / dG / workspace must be 16-byte aligned", fn);
  XBArgs a;
  a.B = B; a.T = T; a.dh = dh_out; a.d_ldb = d_ldb; a.d_ldt = d_ldt; a.gates = gates; a.c = c_all;
  a.WT = WT; a.WTb = nullptr; a.dG = dG; a.dGb = nullptr;
  a.bar = static_cast<int*>(workspace);
  a.timeout_ticks = g_timeout_ticks > 0 ? g_timeout_ticks : 100000000;
  AVC_HIP(avc::zero_async(workspace, XC_BYTES, stream), fn);
  hipLaunchKernelGGL((lstm_xcd_bwd_kernel<512, false>), dim3(XNX * XSL), dim3(XNT), xcd_bwd_lds(), stream, a);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int autovc_lstm_bwd_xcd_bf16(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                                        const float* gates, const float* c_all, const uint16_t* WT_b, float* dG,
                                        uint16_t* dGb, void* workspace, hipStream_t stream) {
  static const char* fn = "autovc_lstm_bwd_xcd_bf16";
  AVC_CHECK_ARG(T > 0 && autovc_lstm_xcd_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs B=64, H=512, 8 XCDs x 32 CUs)", fn, B, H);
  AVC_CHECK_ARG(gates && c_all && WT_b && dG && dGb && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(WT_b) && AVC_ALIGNED16(dGb) && AVC_ALIGNED16(workspace),
                "%s: WT_b / dGb / workspace must be 16-byte aligned", fn);
  XBArgs a;
  a.B = B; a.T = T; a.dh = dh_out; a.d_ldb = d_ldb; a.d_ldt = d_ldt; a.gates = gates; a.c = c_all;
  a.WT = nullptr; a.WTb = reinterpret_cast<const __bf16*>(WT_b); a.dG = dG; a.dGb = reinterpret_cast<__bf16*>(dGb);
  a.bar = static_cast<int*>(workspace);
  a.timeout_ticks = g_timeout_ticks > 0 ? g_timeout_ticks : 100000000;
  AVC_HIP(avc::zero_async(workspace, XC_BYTES, stream), fn);
  hipLaunchKernelGGL((lstm_xcd_bwd_kernel<512, true>), dim3(XNX * XSL), dim3(XNT), xcd_bwd_lds(), stream, a);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int64_t autovc_lstm2_persist_workspace_bytes(int B, int T, int H) {
  if (B <= 0 || T <= 0 || H != 1024) return -1;
  return BAR_BYTES + 2 * (int64_t)T * B * H * 4;
}

extern "C" int autovc_lstm2_persist_supported(int B, int H) {
  return (H == 1024 && B == PB && persist_fits<1024, true>()) ? 1 : 0;
}

extern "C" int autovc_lstm2_fwd_persist_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                            const float* W_hh0, const float* b_ih1, const float* b_hh1,
                                            const float* W_ih1, const float* W_hh1, float* h0, float* c0,
                                            float* gates0, float* h1, float* c1, float* gates1, void* workspace,
                                            hipStream_t stream) {
  static const char* fn = "autovc_lstm2_fwd_persist_f32";
  AVC_CHECK_ARG(T > 0 && autovc_lstm2_persist_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs H=1024, B=%d, one CU per workgroup)", fn,
                B, H, PB);
  AVC_CHECK_ARG(gx0 && W_hh0 && b_ih1 && b_hh1 && W_ih1 && W_hh1 && h0 && c0 && h1 && c1 && workspace,
                "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh0) && AVC_ALIGNED16(W_ih1) && AVC_ALIGNED16(W_hh1) && AVC_ALIGNED16(workspace),
                "%s: weights / workspace must be 16-byte aligned", fn);
  PArgs a;
  a.B = B; a.T = T; a.H = H;
  a.gx0 = gx0; a.gx_ldb = gx_ldb; a.gx_ldt = gx_ldt;
  a.W_hh0 = W_hh0; a.b_ih1 = b_ih1; a.b_hh1 = b_hh1; a.W_ih1 = W_ih1; a.W_hh1 = W_hh1;
  a.h0 = h0; a.c0 = c0; a.g0 = gates0; a.h1 = h1; a.c1 = c1; a.g1 = gates1;
  a.h0_ldb = (int64_t)T * H; a.h0_ldt = H;
  AVC_HIP(avc::zero_async(workspace, BAR_BYTES, stream), fn);
  launch_persist<1024, true>(a, workspace, stream);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int autovc_lstm2_fwd_persist_bf16(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                             const uint16_t* W_hh0_b, const float* b_ih1, const float* b_hh1,
                                             const uint16_t* W_ih1_b, const uint16_t* W_hh1_b, float* h0, float* c0,
                                             float* gates0, float* h1, float* c1, float* gates1, void* workspace,
                                             hipStream_t stream) {
  static const char* fn = "autovc_lstm2_fwd_persist_bf16";
  AVC_CHECK_ARG(T > 0 && H == 1024 && B == PB && (persist_fits<1024, true, true>()),
                "%s: unsupported shape B=%d H=%d on this device (needs H=1024, B=%d, one CU per workgroup)", fn,
                B, H, PB);
  AVC_CHECK_ARG(gx0 && W_hh0_b && b_ih1 && b_hh1 && W_ih1_b && W_hh1_b && h0 && c0 && h1 && c1 && workspace,
                "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh0_b) && AVC_ALIGNED16(W_ih1_b) && AVC_ALIGNED16(W_hh1_b) &&
                AVC_ALIGNED16(workspace), "%s: weights / workspace must be 16-byte aligned", fn);
  PArgs a = {};
  a.B = B; a.T = T; a.H = H;
  a.gx0 = gx0; a.gx_ldb = gx_ldb; a.gx_ldt = gx_ldt;
  a.b_ih1 = b_ih1; a.b_hh1 = b_hh1;
  a.W0b = reinterpret_cast<const __bf16*>(W_hh0_b);
  a.Wi1b = reinterpret_cast<const __bf16*>(W_ih1_b);
  a.W1b = reinterpret_cast<const __bf16*>(W_hh1_b);
  a.h0 = h0; a.c0 = c0; a.g0 = gates0; a.h1 = h1; a.c1 = c1; a.g1 = gates1;
  a.h0_ldb = (int64_t)T * H; a.h0_ldt = H;
  AVC_HIP(avc::zero_async(workspace, BAR_BYTES, stream), fn);
  launch_persist<1024, true, true>(a, workspace, stream);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

extern "C" int64_t autovc_lstm_persist_workspace_bytes(int B, int T, int H) {
  if (B <= 0 || T <= 0 || (H != 512 && H != 1024)) return -1;
  return BAR_BYTES + (int64_t)T * B * H * 4;
}

extern "C" int autovc_lstm_persist_supported(int B, int H) {
  if (B != PB) return 0;
  if (H == 512) return persist_fits<512, false>() ? 1 : 0;
  if (H == 1024) return persist_fits<1024, false>() ? 1 : 0;
  return 0;
}

extern "C" int autovc_lstm_fwd_persist_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                           const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                           float* gates, void* workspace, hipStream_t stream) {
  static const char* fn = "autovc_lstm_fwd_persist_f32";
  AVC_CHECK_ARG(T > 0 && autovc_lstm_persist_supported(B, H),
                "%s: unsupported shape B=%d H=%d on this device (needs H=512 or 1024, B=%d)", fn, B, H, PB);
  AVC_CHECK_ARG(gx && W_hh && h && c_all && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh) && AVC_ALIGNED16(workspace), "%s: weights / workspace must be 16-byte aligned",
                fn);
  PArgs a = {};
  a.B = B; a.T = T; a.H = H;
  a.gx0 = gx; a.gx_ldb = gx_ldb; a.gx_ldt = gx_ldt;
  a.W_hh0 = W_hh;
  a.h0 = h; a.c0 = c_all; a.g0 = gates;
  a.h0_ldb = h_ldb; a.h0_ldt = h_ldt;
  AVC_HIP(avc::zero_async(workspace, BAR_BYTES, stream), fn);
  if (H == 512) launch_persist<512, false>(a, workspace, stream);
  else launch_persist<1024, false>(a, workspace, stream);
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}

// 0 = the last call's barriers completed, else a timeout was recorded (synchronises)
extern "C" int autovc_lstm2_persist_status(const void* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(workspace != nullptr, "autovc_lstm2_persist_status: null workspace");
  int err = 0;
  AVC_HIP(hipMemcpyAsync(&err, static_cast<const int*>(workspace) + BAR_ERR * L, sizeof(int), hipMemcpyDeviceToHost,
                         stream), "autovc_lstm2_persist_status");
  AVC_HIP(hipStreamSynchronize(stream), "autovc_lstm2_persist_status");
  return err;
}

// test hook: the spin budget of the persistent launches in s_memrealtime ticks (0 = 1 s)
extern "C" int autovc_lstm_persist_set_timeout_ticks(int ticks) {
  AVC_CHECK_ARG(ticks >= 0, "autovc_lstm_persist_set_timeout_ticks: ticks must be >= 0");
  g_timeout_ticks = ticks;
  return avc::kOk;
}

// The device fault word (one bit per persistent kernel family whose barrier timed out) after
// everything queued on `stream`; synchronises the stream.  clear != 0 resets it.
extern "C" int autovc_fault_status(hipStream_t stream, int clear, int* out) {
  AVC_CHECK_ARG(out != nullptr, "autovc_fault_status: null out");
  int v = 0;
  AVC_HIP(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_avc_fault), sizeof(int), 0, hipMemcpyDeviceToHost, stream),
          "autovc_fault_status");
  AVC_HIP(hipStreamSynchronize(stream), "autovc_fault_status");
  if (clear && v) {
    const int zero = 0;
    AVC_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_avc_fault), &zero, sizeof(int), 0, hipMemcpyHostToDevice, stream),
            "autovc_fault_status");
    AVC_HIP(hipStreamSynchronize(stream), "autovc_fault_status");
  }
  *out = v;
  return avc::kOk;
}


