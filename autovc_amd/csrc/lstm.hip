// LSTM recurrences (torch nn.LSTM semantics, used at model_vc_mel.py:61,90,104) on gfx950.
//
//   gates_t = gx_t + h_{t-1} W_hh^T            (gx_t = x_t W_ih^T + b_ih + b_hh: one GEMM
//                                               over all frames, done before the recurrence)
//   i,f,o = sigmoid, g = tanh;  c_t = f c_{t-1} + i g;  h_t = o tanh(c_t);  h_{-1} = c_{-1} = 0
//   torch gate order [i | f | g | o] along the 4H axis.
//
// Two regimes:
//  * large H (decoder lstm1 H=512, lstm2 H=1024): one launch per time step on the
//    caller's stream (a kernel boundary, ~1.5 us, is cheaper than a grid barrier on
//    MI355X: MI355X_MICROARCH.md price list "boundary" vs "barrier-xcd").  Each step is a
//    small-M GEMM (64 batch x 4H gate rows x H) cut into 32x32 output tiles = 256
//    workgroups for H=1024: a tile is 32 batch rows x (8 hidden units x 4 gates), so the
//    cell update is fused into the epilogue.  Operands are register-staged into a
//    double-buffered, XOR-swizzled LDS tile (see tile_gemm) and each wave's 16x16
//    quadrant runs on v_mfma_f32_16x16x4_f32 (exact fp32).
//    Backward = per step the same tile kernel computing split-K partials of
//    dh_rec = dG_t W_hh (through the pre-transposed W_hh^T) + a pointwise kernel.
//  * small H (encoder BLSTM, H=32): the whole sequence in one launch, one workgroup per
//    (direction, 2 batch rows), a quad of lanes per (row, unit) splitting the 32-deep dot
//    products, W_hh slices held in registers, per-step operands prefetched 8 steps ahead.
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int kThreads = 256;
constexpr int TB = 32;          // batch rows per tile
constexpr int TN = 32;          // output columns per tile
constexpr int UT = TN / 4;      // hidden units per forward tile (x 4 gates)

// Register-staged tile GEMM: the 32 x 32 output tile of a workgroup,
//   C[r][n] = sum_k A_r[k] * B_n[k]   (A rows: batch, B rows: weight rows; K contiguous),
// over chunks of KCH k.  Each thread prefetches its PER float4 of the next D chunks into
// VGPRs (plain global_load_dwordx4: far cheaper to issue than LDS-DMA, which capped the
// first version at ~25 GB/s per CU — tools/lstm_step_bench.hip), writes the current
// chunk to one of two LDS buffers (XOR-swizzled 16-B slots: conflict-free ds_read_b128),
// one barrier per chunk.  NW = 4 waves: one 16x16 quadrant each; NW = 8: quadrant x
// k-half, the halves summed through LDS at the end.  v_mfma_f32_16x16x4_f32 throughout.
template <int KCH, int NW, int D>
struct Tile {
  static constexpr int SLOTS = KCH / 4;             // float4 slots per row per chunk
  static constexpr int NT = 64 * NW;
  static constexpr int PER = TB * SLOTS / NT;       // float4 per thread per operand per chunk
  static constexpr int CF = (TB + TN) * KCH;        // floats per LDS chunk buffer
  static constexpr int SUB = KCH / 16 / (NW / 4);   // 16-k sub-blocks per wave per chunk
  static constexpr int RED = 4 * 16 * 17;
  static constexpr int LDS_FLOATS = 2 * CF + RED;
  static_assert(PER * NT == TB * SLOTS && TB == TN, "staging map covers the tile exactly");
};

// swizzled float4 position of slot sl in row r
__device__ __forceinline__ int swz(int sl, int r) { return (sl & ~15) | ((sl & 15) ^ (r & 15)); }

// Two K segments: k < K1 reads the rows of (arow_of, brow_of), the next K2 those of
// (arow2_of, brow2_of) — the stacked-layer step concatenates [input ; recurrent] this way
// (K2 = 0: one segment).
// BF: the rows hold bf16 (row pointers and K1/K2 still in 4-byte units: a 16-byte slot is
// 8 bf16), and a 16-k sub-block of fp32 slots becomes one 32-k v_mfma_f32_16x16x32_bf16 —
// lane group g's slot is exactly that instruction's k = 8g .. 8g+7 operand.  The staging,
// swizzle and reduction are byte-for-byte those of the fp32 tile.
template <int KCH, int NW, int D, bool BF = false, class AR, class BR, class AR2, class BR2>
__device__ __forceinline__ f32x4 tile_gemm2(float* lds, AR arow_of, BR brow_of, int K1, AR2 arow2_of, BR2 brow2_of,
                                            int K2) {
  using C = Tile<KCH, NW, D>;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* arow[C::PER];
  const float* brow[C::PER];
  const float* arow2[C::PER];
  const float* brow2[C::PER];
  int srow[C::PER], spos[C::PER];
#pragma unroll
  for (int i = 0; i < C::PER; ++i) {
    const int e = tid + i * C::NT;
    const int r = e / C::SLOTS, sl = e % C::SLOTS;
    srow[i] = r;
    spos[i] = swz(sl, r);
    arow[i] = (K1 ? arow_of(r) : arow2_of(r)) + 4 * sl;
    brow[i] = (K1 ? brow_of(r) : brow2_of(r)) + 4 * sl;
    arow2[i] = (K2 ? arow2_of(r) : arow[i] - 4 * sl) + 4 * sl;
    brow2[i] = (K2 ? brow2_of(r) : brow[i] - 4 * sl) + 4 * sl;
  }
  const int nc1 = K1 / KCH, nc = (K1 + K2) / KCH;
  auto at = [&](const float* const* p1, const float* const* p2, int i, int cl) {
    return cl < nc1 ? p1[i] + cl * KCH : p2[i] + (cl - nc1) * KCH;
  };
  // Loads run D chunks ahead.  They are issued unconditionally (past the last chunk the
  // address is clamped to the last chunk, an L2 hit) so the k loop is straight-line code
  // and hipcc can wait with vmcnt(4 (D-1)) for the oldest chunk only: a conditional load
  // makes it wait vmcnt(0) at the join, which silently degrades D > 1 to D = 1.
  f32x4 sa[D][C::PER], sb[D][C::PER];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int cl = min(d, nc - 1);
#pragma unroll
    for (int i = 0; i < C::PER; ++i) {
      sa[d][i] = *reinterpret_cast<const f32x4*>(at(arow, arow2, i, cl));
      sb[d][i] = *reinterpret_cast<const f32x4*>(at(brow, brow2, i, cl));
    }
  }
  const int q = w & 3, kh = w >> 2, g = lane >> 4;
  const int ra = (q >> 1) * 16 + (lane & 15), rb = (q & 1) * 16 + (lane & 15);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nc; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      float* L = lds + (c & 1) * C::CF;
#pragma unroll
      for (int i = 0; i < C::PER; ++i) {
        *reinterpret_cast<f32x4*>(L + srow[i] * KCH + 4 * spos[i]) = sa[d][i];
        *reinterpret_cast<f32x4*>(L + (TB + srow[i]) * KCH + 4 * spos[i]) = sb[d][i];
      }
      __syncthreads();   // chunk c visible; buffer (c+1)&1 no longer read (last read at c-1)
      const int cn = min(c + D, nc - 1);
#pragma unroll
      for (int i = 0; i < C::PER; ++i) {
        sa[d][i] = *reinterpret_cast<const f32x4*>(at(arow, arow2, i, cn));
        sb[d][i] = *reinterpret_cast<const f32x4*>(at(brow, brow2, i, cn));
      }
      if (c < nc) {
        f32x4 av[C::SUB], bv[C::SUB];
#pragma unroll
        for (int s = 0; s < C::SUB; ++s) {
          const int sl = (kh * C::SUB + s) * 4 + g;
          av[s] = *reinterpret_cast<const f32x4*>(L + ra * KCH + 4 * swz(sl, ra));
          bv[s] = *reinterpret_cast<const f32x4*>(L + (TB + rb) * KCH + 4 * swz(sl, rb));
        }
        // MFMA local k index (lane>>4) <-> actual k = 16*sub + 4g + jj: same map for A and B
        if constexpr (BF) {
#pragma unroll
          for (int s = 0; s < C::SUB; ++s) {
            const bf16x8 ab = __builtin_bit_cast(bf16x8, av[s]), bb = __builtin_bit_cast(bf16x8, bv[s]);
            if (s & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc1, 0, 0, 0);
            else acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc0, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int s = 0; s < C::SUB; ++s)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              if (s & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s][jj], bv[s][jj], acc1, 0, 0, 0);
              else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s][jj], bv[s][jj], acc0, 0, 0, 0);
            }
        }
      }
    }
  }
  f32x4 acc = acc0 + acc1;
  if (NW == 8) {
    float* red = lds + 2 * C::CF;
    if (kh == 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(q * 16 + 4 * g + r) * 17 + (lane & 15)] = acc[r];
    __syncthreads();
    if (kh == 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += red[(q * 16 + 4 * g + r) * 17 + (lane & 15)];
  }
  return acc;  // valid in waves 0..3 (quadrant q = wave)
}

template <int KCH, int NW, int D, bool BF = false, class AR, class BR>
__device__ __forceinline__ f32x4 tile_gemm(float* lds, AR arow_of, BR brow_of, int K) {
  return tile_gemm2<KCH, NW, D, BF>(lds, arow_of, brow_of, K, arow_of, brow_of, 0);
}

// configuration used by the product kernels (chosen with tools/lstm_step_bench.hip): k chunk,
// waves per workgroup, chunks of loads in flight
constexpr int KCH = 64, NWV = 8, DPF = 2;
using TileP = Tile<KCH, NWV, DPF>;
// the fused backward steps' tile (tools/lstm_bwd_tile_sweep.sh builds variants: AVC_BKCH / AVC_BNW /
// AVC_BD override it)
#ifndef AVC_BKCH
#define AVC_BKCH 64
#endif
#ifndef AVC_BNW
#define AVC_BNW 8
#endif
#ifndef AVC_BD
#define AVC_BD 2
#endif
constexpr int BKCH = AVC_BKCH, BNW = AVC_BNW, BD = AVC_BD;

struct StepArgs {
  int B, T, H;
  const float* gx; int64_t gx_ldb, gx_ldt;   // gx[b*gx_ldb + t*gx_ldt + r]
  const float* W;                            // W_hh (4H, H)
  float* h; int64_t h_ldb, h_ldt;            // h out/in: h[b*h_ldb + t*h_ldt + j]
  float* c;                                  // (B, T, H) cell states
  float* gates;                              // (B, T, 4H) post-activation gates or null
  const float* gx2;                          // second bias added to gx (same strides) or null
  // bf16 recurrences (precision "bf16"): W_hh rounded to bf16 (4H, H) and a bf16 copy of
  // h, (B, T, H) contiguous, written by the epilogue and read by the next step's product
  const __bf16* Wb;
  __bf16* hb;
};

// One forward time step of a large-H layer, block (blockIdx.x, blockIdx.y) of grid
// (H / 8, ceil(B / 32)).  Gate pre-activations = gx_t + [xin_t ; h_{t-1}] [W_in ; W]^T:
// K_in = 0 for a layer whose input projection gx was precomputed by one GEMM over all
// frames; K_in = I for the upper layer of a stacked pair, whose input is the lower layer's
// h_t of this same launch wavefront (gx then holds only b_ih + b_hh, strides 0).
// ABL != 0 only in the ablation build of tools/lstm_step_bench.hip (bit 0: every block
// reads the same W_hh rows, bit 1: every lane reads the same h row) — never launched here.
// BF: the recurrent (and stacked-input) products on bf16 copies (StepArgs::Wb / hb, the
// input rows xin / W_in bf16 too), cell math and all fp32 outputs unchanged.
template <int ABL, int KCH_, int NW_, int D_, bool BF = false>
__device__ __forceinline__ void fwd_step_body(const StepArgs& a, int t, int tp, const void* xin, int64_t x_ldb,
                                              int64_t x_ldt, const void* W_in, int K_in) {
  using C = Tile<KCH_, NW_, D_>;
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int H = a.H;
  const int j0 = blockIdx.x * UT, b0 = blockIdx.y * TB;
  // epilogue operands (input-gate pre-activations, previous cell) prefetched before the
  // recurrent product so their latency hides under it
  const int bl = (threadIdx.x & 255) >> 3, u = threadIdx.x & 7;
  const int b = b0 + bl, j = j0 + u;
  const bool own = threadIdx.x < 256 && b < a.B;
  float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f;
  if (own) {
    const float* g = a.gx + (int64_t)b * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
    for (int q = 0; q < 4; ++q) gxv[q] = g[q * H + j];
    if (a.gx2) {
      const float* g2 = a.gx2 + (int64_t)b * a.gx_ldb + (int64_t)t * a.gx_ldt;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] += g2[q * H + j];
    }
    if (tp >= 0) cp = a.c[(int64_t)b * a.T * H + (int64_t)tp * H + j];
  }
  // K in 4-byte units (bf16 rows: half the elements)
  const int K_rec = tp >= 0 ? (BF ? H / 2 : H) : 0;
  const int K_in_u = BF ? K_in / 2 : K_in;
  auto arow_of = [&](int r) {
    const int b = (ABL & 2) ? 0 : min(b0 + r, a.B - 1);  // rows past B: any valid row, result unused
    if constexpr (BF) return reinterpret_cast<const float*>(a.hb + ((int64_t)b * a.T + max(tp, 0)) * H);
    else return (const float*)(a.h + (int64_t)b * a.h_ldb + (int64_t)max(tp, 0) * a.h_ldt);
  };
  auto brow_of = [&](int r) {  // tile column r = gate*8 + unit
    const int64_t row = (r >> 3) * H + ((ABL & 1) ? 0 : j0) + (r & 7);
    if constexpr (BF) return reinterpret_cast<const float*>(a.Wb + row * H);
    else return a.W + row * H;
  };
  auto xrow_of = [&](int r) {
    const int64_t off = (int64_t)min(b0 + r, a.B - 1) * x_ldb + (int64_t)t * x_ldt;
    if constexpr (BF) return reinterpret_cast<const float*>(static_cast<const __bf16*>(xin) + off);
    else return static_cast<const float*>(xin) + off;
  };
  auto wrow_of = [&](int r) {
    const int64_t off = (int64_t)((r >> 3) * H + j0 + (r & 7)) * K_in;
    if constexpr (BF) return reinterpret_cast<const float*>(static_cast<const __bf16*>(W_in) + off);
    else return static_cast<const float*>(W_in) + off;
  };
  float pre[4];
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (K_in_u + K_rec > 0)
      acc = tile_gemm2<KCH_, NW_, D_, BF>(smem, xrow_of, wrow_of, K_in_u, arow_of, brow_of, K_rec);
    __syncthreads();
    float* tile = smem;                                      // [32][33] after the chunk buffers are drained
    if (w < 4) {
      const int wi = w >> 1, wn = w & 1;
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(wi * 16 + 4 * (lane >> 4) + r) * (TN + 1) + wn * 16 + (lane & 15)] = acc[r];
    }
    __syncthreads();
    if (!own) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = tile[bl * (TN + 1) + q * UT + u];
  }
  const float i_ = avc_sigmoid(pre[0] + gxv[0]), f_ = avc_sigmoid(pre[1] + gxv[1]);
  const float g_ = tanhf(pre[2] + gxv[2]), o_ = avc_sigmoid(pre[3] + gxv[3]);
  const float cn = f_ * cp + i_ * g_;
  a.c[(int64_t)b * a.T * H + (int64_t)t * H + j] = cn;
  const float hn = o_ * tanhf(cn);
  a.h[(int64_t)b * a.h_ldb + (int64_t)t * a.h_ldt + j] = hn;
  if (BF) a.hb[((int64_t)b * a.T + t) * H + j] = (__bf16)hn;
  if (a.gates) {
    float* gs = a.gates + ((int64_t)b * a.T + t) * 4 * H;
    gs[0 * H + j] = i_; gs[1 * H + j] = f_; gs[2 * H + j] = g_; gs[3 * H + j] = o_;
  }
}

template <int ABL = 0, int KCH_ = KCH, int NW_ = NWV, int D_ = DPF, bool BF = false>
__global__ __launch_bounds__(64 * NW_) void lstm_fwd_step_kernel(StepArgs a, int t, int tp) {
  fwd_step_body<ABL, KCH_, NW_, D_, BF>(a, t, tp, nullptr, 0, 0, nullptr, 0);
}

// Two stacked layers (nn.LSTM num_layers=2, decoder lstm2) as one launch per wavefront
// step: blockIdx.z = 0 runs layer 0 at step t, z = 1 runs layer 1 at step t - 1 on the
// layer-0 output h0_{t-1} written by the previous launch.  T + 1 launches instead of 2T,
// both layers' blocks co-resident on every CU (2 blocks/CU), and no separate input
// projection GEMM for layer 1 (it is the first K segment of its step).
struct Stack2Args {
  StepArgs l0, l1;
  const float* W_ih1;   // (4H, H)
  const __bf16* W_ih1b; // its bf16 copy (BF)
};

template <int KCH_ = KCH, int NW_ = NWV, int D_ = DPF, bool BF = false>
__global__ __launch_bounds__(64 * NW_) void lstm2_fwd_step_kernel(Stack2Args a, int t) {
  if (blockIdx.z == 0) {
    if (t < a.l0.T) fwd_step_body<0, KCH_, NW_, D_, BF>(a.l0, t, t - 1, nullptr, 0, 0, nullptr, 0);
  } else if (t >= 1) {
    if constexpr (BF)
      fwd_step_body<0, KCH_, NW_, D_, true>(a.l1, t - 1, t - 2, a.l0.hb, (int64_t)a.l0.T * a.l0.H, a.l0.H,
                                            a.W_ih1b, a.l1.H);
    else
      fwd_step_body<0, KCH_, NW_, D_>(a.l1, t - 1, t - 2, a.l0.h, a.l0.h_ldb, a.l0.h_ldt, a.W_ih1, a.l1.H);
  }
}

// Backward pointwise for one step of a large-H layer: thread per (b, j).
//   dh = dh_out[t] + sum_s P[s]           (P: split-K partials of dG_{t'} W_hh, t' = later step)
//   dc = dc_state + dh o (1 - tanh(c)^2);  dG = [dc g i(1-i), dc c_prev f(1-f), dc i (1-g^2),
//   dh tanh(c) o(1-o)];  dc_state <- dc f
struct BwdArgs {
  int B, T, H;
  const float* dh_out; int64_t d_ldb, d_ldt;  // dL/dh from above (may be null)
  const float* gates;                          // (B,T,4H)
  const float* c;                              // (B,T,H)
  float* dG;                                   // (B,T,4H) out
  float* dc_state;                             // (B,H)
  float* P; int S;                             // (S,B,H) partials or null
  __bf16* dGb;                                 // bf16 copy of dG (bf16 recurrences) or null
  int prio;                                    // fused steps: raise the waves' issue priority
};

// The fused backward steps run at wave priority 3 (s_setprio): beside the gradient side
// stream's GEMM waves — older, and so ahead in the SIMD's issue arbitration at equal priority —
// the latency-bound step's waves issue first.  fp32 step 14.30-14.35 vs 14.37-14.41 ms, bf16
// 9.01-9.03 alike (profiles/r05/ab_lstm_prio.txt).
int lstm_prio() { return 1; }
__device__ __forceinline__ void step_priority(int prio) {
  if (__builtin_amdgcn_readfirstlane(prio)) __builtin_amdgcn_s_setprio(3);
}

// Pointwise pass of one backward step: thread per (b, j).  Every operand is loaded
// unconditionally before first use (optional operands are template switches, the previous
// cell is read at a clamped step and masked): a load behind a runtime condition makes
// hipcc wait vmcnt(0) per load, serialising a dozen HBM round trips.
// Thread = 4 consecutive units of one batch row (float4 loads / stores), grid (H/256, B)
// of 64-thread blocks: no 64-bit index division, and the bf16 dG copy comes from registers.
// 16-byte load through L2 only (sc1: the vector L1 is bypassed) — the partial slabs of the
// fused backward below, written by other workgroups of the same launch with sc1 stores
// (cdna_hip_programming.md §6 Guideline 16, the write-through counter form)
__device__ __forceinline__ f32x4 ld4_sc1(const float* base, int64_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(off * 4), 0, 16));
}
__device__ __forceinline__ void st4_sc1(float* base, int64_t off, f32x4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                         (uint32_t)(off * 4), 0, 16);
}

// The pointwise pass of 4 consecutive units (b, j..j+3), in two halves: pw_load issues the
// loads that do not depend on this step's partials (saved gates and cells, dh from above, the
// carried cell gradient), pw_finish reads the S partials, sums them after dh in slab order and
// writes dG (and its bf16 copy) and the new carry.  SC1: the partials were stored write-through
// by other workgroups of the running launch and are read through L2.
struct PwIn {
  f32x4 i, f, g, o, cc, cpr, dh, dcs;
};

template <bool FIRST, bool HAS_DH>
__device__ __forceinline__ PwIn pw_load(const BwdArgs& a, int t, int tp, int b, int j) {
  const int H = a.H;
  auto ld4 = [](const float* p) { return *reinterpret_cast<const f32x4*>(p); };
  const float* gs = a.gates + ((int64_t)b * a.T + t) * 4 * H + j;
  PwIn in;
  in.i = ld4(gs); in.f = ld4(gs + H); in.g = ld4(gs + 2 * H); in.o = ld4(gs + 3 * H);
  in.cc = ld4(a.c + ((int64_t)b * a.T + t) * H + j);
  in.cpr = ld4(a.c + ((int64_t)b * a.T + (tp >= 0 ? tp : t)) * H + j);
  in.dh = f32x4{0.f, 0.f, 0.f, 0.f};
  in.dcs = f32x4{0.f, 0.f, 0.f, 0.f};
  if (HAS_DH) in.dh = ld4(a.dh_out + (int64_t)b * a.d_ldb + (int64_t)t * a.d_ldt + j);
  if (!FIRST) in.dcs = ld4(a.dc_state + (int64_t)b * H + j);
  return in;
}

// Contraction off: the fused step and the launch pair inline this into different code, and
// with mul-add fusion left to the compiler they rounded layer 0's cell gradient differently
// (1 ulp); spelled out, both paths are bit-identical.
template <int S, bool FIRST, bool SC1>
__device__ __forceinline__ void pw_finish(const BwdArgs& a, const PwIn& in, int t, int tp, int b, int j) {
#pragma clang fp contract(off)
  const int H = a.H;
  const int64_t BH = (int64_t)a.B * H, bj = (int64_t)b * H + j;
  auto ld4 = [](const float* p) { return *reinterpret_cast<const f32x4*>(p); };
  f32x4 dh = in.dh;
  const f32x4 dcs = in.dcs;
  const f32x4 i_ = in.i, f_ = in.f, g_ = in.g, o_ = in.o, cc = in.cc, cpr = in.cpr;
  f32x4 p[S];
  if (!FIRST) {
#pragma unroll
    for (int s = 0; s < S; ++s) p[s] = SC1 ? ld4_sc1(a.P, (int64_t)s * BH + bj) : ld4(a.P + (int64_t)s * BH + bj);
#pragma unroll
    for (int s = 0; s < S; ++s) dh += p[s];
  }
  f32x4 di, df, dg, dO, dcn;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float cp = tp >= 0 ? cpr[e] : 0.f;
    const float tc = tanhf(cc[e]);
    const float dc = dcs[e] + dh[e] * o_[e] * (1.f - tc * tc);
    di[e] = dc * g_[e] * i_[e] * (1.f - i_[e]);
    df[e] = dc * cp * f_[e] * (1.f - f_[e]);
    dg[e] = dc * i_[e] * (1.f - g_[e] * g_[e]);
    dO[e] = dh[e] * tc * o_[e] * (1.f - o_[e]);
    dcn[e] = dc * f_[e];
  }
  float* d = a.dG + ((int64_t)b * a.T + t) * 4 * H + j;
  *reinterpret_cast<f32x4*>(d) = di;
  *reinterpret_cast<f32x4*>(d + H) = df;
  *reinterpret_cast<f32x4*>(d + 2 * H) = dg;
  *reinterpret_cast<f32x4*>(d + 3 * H) = dO;
  if (a.dGb) {
    __bf16* db = a.dGb + ((int64_t)b * a.T + t) * 4 * H + j;
    auto cv = [](f32x4 v) { return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]}; };
    *reinterpret_cast<bf16x4*>(db) = cv(di);
    *reinterpret_cast<bf16x4*>(db + H) = cv(df);
    *reinterpret_cast<bf16x4*>(db + 2 * H) = cv(dg);
    *reinterpret_cast<bf16x4*>(db + 3 * H) = cv(dO);
  }
  *reinterpret_cast<f32x4*>(a.dc_state + bj) = dcn;
}

template <int S, bool FIRST, bool HAS_DH, bool SC1 = false>
__device__ __forceinline__ void bwd_pointwise_elem(const BwdArgs& a, int t, int tp, int b, int j) {
  const PwIn in = pw_load<FIRST, HAS_DH>(a, t, tp, b, j);
  pw_finish<S, FIRST, SC1>(a, in, t, tp, b, j);
}

template <int S, bool FIRST, bool HAS_DH>
__device__ __forceinline__ void bwd_pointwise_body(const BwdArgs& a, int t, int tp) {
  const int j = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (j >= a.H) return;
  bwd_pointwise_elem<S, FIRST, HAS_DH>(a, t, tp, blockIdx.y, j);
}

template <int S, bool FIRST, bool HAS_DH>
__global__ __launch_bounds__(64) void lstm_bwd_pointwise_kernel(BwdArgs a, int t, int tp) {
  bwd_pointwise_body<S, FIRST, HAS_DH>(a, t, tp);
}

// Both layers of a stacked pair (decoder lstm2) in one launch of the backward wavefront
// (see autovc_lstm2_bwd_f32): blockIdx.z = 0 is layer 1 at step t1 (dh from above + its
// S recurrent partials), z = 1 is layer 0 at step t0 = t1 + 1, whose dh is the sum of 2S
// partials: S of its own recurrence and S of layer 1's input gradient dG1_t0 W_ih1.
template <int S>
__global__ __launch_bounds__(64) void lstm2_bwd_pointwise_kernel(BwdArgs a1, BwdArgs a0, int t1, int t0) {
  if (blockIdx.z == 0) {
    if (t1 < 0) return;
    if (t1 == a1.T - 1) bwd_pointwise_body<S, true, true>(a1, t1, t1 - 1);
    else bwd_pointwise_body<S, false, true>(a1, t1, t1 - 1);
  } else {
    if (t0 >= a0.T) return;
    bwd_pointwise_body<2 * S, false, false>(a0, t0, t0 - 1);
  }
}

template <int S>
void launch_pointwise(dim3 grid, hipStream_t st, const BwdArgs& a, int t, int tp, bool first) {
  if (first) {
    if (a.dh_out) hipLaunchKernelGGL((lstm_bwd_pointwise_kernel<S, true, true>), grid, dim3(64), 0, st, a, t, tp);
    else hipLaunchKernelGGL((lstm_bwd_pointwise_kernel<S, true, false>), grid, dim3(64), 0, st, a, t, tp);
  } else {
    if (a.dh_out) hipLaunchKernelGGL((lstm_bwd_pointwise_kernel<S, false, true>), grid, dim3(64), 0, st, a, t, tp);
    else hipLaunchKernelGGL((lstm_bwd_pointwise_kernel<S, false, false>), grid, dim3(64), 0, st, a, t, tp);
  }
}

void launch_pointwise_any(int /*blocks*/, hipStream_t st, const BwdArgs& a, int t, int tp, bool first) {
  const dim3 grid((a.H / 4 + 63) / 64, a.B);
  switch (a.S) {
    case 1: launch_pointwise<1>(grid, st, a, t, tp, first); break;
    case 2: launch_pointwise<2>(grid, st, a, t, tp, first); break;
    case 4: launch_pointwise<4>(grid, st, a, t, tp, first); break;
    default: launch_pointwise<8>(grid, st, a, t, tp, first); break;
  }
}

// Split-K recurrent product P[s][b][j] = sum_{r in split s} dG[b][t][r] W^T[j][r]
// (the split-s part of dh_rec for the next step back), grid = (H/32, ceil(B/32), S).
// The S partials are summed, in fixed order, by the next step's pointwise kernel.  (A
// fused variant — last-arriving split block runs the pointwise pass behind an agent-scope
// release/acquire ticket — measured 13.8 us per step against 9.2 + 4.0 us for the two
// launches: the serial partial read + fences cost more than the kernel boundary.)
// BF: dG / WT are the bf16 copies (passed as raw pointers, row lengths in bf16 elements).
template <int KCH_, int NW_, int D_, bool BF>
__device__ __forceinline__ void bwd_rec_body(int B, int T, int H, const float* dG, int t, const float* WT, float* P,
                                             int j0) {
  using C = Tile<KCH_, NW_, D_>;
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b0 = blockIdx.y * TB, s = blockIdx.z, S = gridDim.z;
  // row length / split offsets in 4-byte units
  const int K4 = BF ? 2 * H : 4 * H, ks = K4 / S, kb = s * ks;
  auto arow_of = [&](int r) { return dG + ((int64_t)min(b0 + r, B - 1) * T + t) * K4 + kb; };
  auto brow_of = [&](int r) { return WT + (int64_t)(j0 + r) * K4 + kb; };
  {
    const f32x4 acc = tile_gemm<KCH_, NW_, D_, BF>(smem, arow_of, brow_of, ks);
    if (w >= 4) return;
    const int wi = w >> 1, wn = w & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = b0 + wi * 16 + 4 * (lane >> 4) + r;
      if (b < B) P[((int64_t)s * B + b) * H + j0 + wn * 16 + (lane & 15)] = acc[r];
    }
  }
}

template <int KCH_ = KCH, int NW_ = NWV, int D_ = DPF, bool BF = false>
__global__ __launch_bounds__(64 * NW_) void lstm_bwd_rec_kernel(int B, int T, int H, const float* dG, int t,
                                                               const float* WT, float* P) {
  bwd_rec_body<KCH_, NW_, D_, BF>(B, T, H, dG, t, WT, P, blockIdx.x * TN);
}

// Recurrent products of one backward wavefront launch of a stacked pair, grid
// (3 H/32, ceil(B/32), S): x-tiles [0, H/32) = dG1_t1 W_hh1 (layer 1's own recurrence,
// -> P1), [H/32, 2H/32) = dG1_t1 W_ih1 (its input gradient = layer 0's dh at t1, -> the
// upper S slabs of PQ0), [2H/32, 3H/32) = dG0_t0 W_hh0 (-> the lower S slabs of PQ0).
// W*T are the (H, 4H) transposes.  Out-of-range steps (t1 < 0, t0 >= T) exit.
// BF: dG* / W*T are the bf16 copies (autovc_lstm2_bwd_bf16).
template <int KCH_ = KCH, int NW_ = NWV, int D_ = DPF, bool BF = false>
__global__ __launch_bounds__(64 * NW_) void lstm2_bwd_rec_kernel(int B, int T, int H, const float* dG1,
                                                                const float* dG0, int t1, int t0,
                                                                const float* WT1, const float* WIT1,
                                                                const float* WT0, float* P1, float* PQ0) {
  const int nt = H / TN, prod = blockIdx.x / nt, j0 = (blockIdx.x % nt) * TN;
  const int64_t slabs = (int64_t)gridDim.z * B * H;
  if (prod < 2) {
    if (t1 < 0) return;
    if (prod == 0) bwd_rec_body<KCH_, NW_, D_, BF>(B, T, H, dG1, t1, WT1, P1, j0);
    else bwd_rec_body<KCH_, NW_, D_, BF>(B, T, H, dG1, t1, WIT1, PQ0 + slabs, j0);
  } else {
    if (t0 >= T) return;
    bwd_rec_body<KCH_, NW_, D_, BF>(B, T, H, dG0, t0, WT0, PQ0, j0);
  }
}

// ---------------------------------------------------------------- fused backward step
// One launch per backward step instead of a product launch + a pointwise launch: every
// split-K job of an output tile (32 batch rows x 32 units) stores its partial write-through
// (sc1), waits for its stores (vmcnt(0)), and one lane draws a ticket on the tile's counter
// (relaxed agent-scope fetch_add); the job that draws the last ticket reads every partial of
// the tile through L2 (sc1 loads) in slab order and runs the pointwise pass of the tile's
// 32 x 32 (b, j) — the placement-independent counter hand-off of cdna_hip_programming.md
// §6 Guideline 16 (its write-through form: no release or acquire fence).  The products, the
// partial values, the order of the sums and the pointwise arithmetic are those of the
// two-launch path, so dG is bit-identical to it (tests/test_lstm_bwd_fused_gpu.py).  The
// grid keeps the product kernels' (x = column tile, y = row tile, z = split) layout with x
// a multiple of 8, so a tile's jobs share blockIdx % 8 (one XCD under the observed
// round-robin placement: speed only).  The counter is reset by the last arriver; the call
// zeroes it once.
struct FusedTile {
  int* cnt;            // arrival counters, one per output tile (layer-1 tiles, then layer 0)
};

// the job's half of the hand-off: its 32 x 32 partial (waves 0..3 hold it after tile_gemm),
// transposed through LDS so that each of 256 threads stores one 16-byte row piece
// P[b][j0 + 4q .. +3] write-through; returns true in every thread of the last-arriving job
__device__ __forceinline__ bool fused_arrive(float* smem, const f32x4& acc, bool zero, float* P, int B, int H,
                                             int b0, int j0, int* cnt, int njobs) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __syncthreads();                                          // tile_gemm's LDS buffers are free
  float* tile = smem;                                       // [32][33]
  if (w < 4) {
    const int wi = w >> 1, wn = w & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      tile[(wi * 16 + 4 * (lane >> 4) + r) * (TN + 1) + wn * 16 + (lane & 15)] = zero ? 0.f : acc[r];
  }
  __syncthreads();
  if (tid < 256) {
    const int row = tid >> 3, q = tid & 7, b = b0 + row;
    if (b < B) {
      const float* src = tile + row * (TN + 1) + 4 * q;
      const f32x4 v = {src[0], src[1], src[2], src[3]};
      st4_sc1(P, (int64_t)b * H + j0 + 4 * q, v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // this wave's partial is written through
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + TB * (TN + 1));  // one LDS array only (no second __shared__)
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == njobs - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // ready for the next launch
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// the last arriver's pointwise pass: 256 threads x 4 units = the tile's 32 rows x 32 units.
// (Issuing the partial-independent loads in every job before its hand-off, so that they
// arrive under the write-through and the ticket, measured slower: the non-last jobs' extra
// fill cost more than the tail it hid — lstm2 23.07 vs 22.36 us per step, lstm1 8.13 vs 7.52.)
template <int NP, bool HAS_DH>
__device__ __forceinline__ void fused_pointwise(const BwdArgs& a, int t, int tp, int b0, int j0) {
  const int tid = threadIdx.x;
  if (tid >= 256) return;
  const int b = b0 + (tid >> 3), j = j0 + 4 * (tid & 7);
  if (b < a.B) bwd_pointwise_elem<NP, false, HAS_DH, true>(a, t, tp, b, j);
}

// single layer (decoder lstm1): grid (H/32, ceil(B/32), S); launch for processed step t
// (products dG_t W_hh -> partials of step tn) runs the pointwise pass of step tn (previous
// cell at tnp, -1 = none)
template <int KCH_, int NW_, int D_, bool BF, int S, bool HAS_DH>
__global__ __launch_bounds__(64 * NW_) void lstm_bwd_fused_kernel(BwdArgs a, const float* dG, int t, int tn, int tnp,
                                                                 const float* WT, FusedTile f) {
  using C = Tile<KCH_, NW_, D_>;
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  step_priority(a.prio);
  const int B = a.B, T = a.T, H = a.H;
  const int j0 = blockIdx.x * TN, b0 = blockIdx.y * TB, s = blockIdx.z;
  const int K4 = BF ? 2 * H : 4 * H, ks = K4 / S, kb = s * ks;
  auto arow_of = [&](int r) { return dG + ((int64_t)min(b0 + r, B - 1) * T + t) * K4 + kb; };
  auto brow_of = [&](int r) { return WT + (int64_t)(j0 + r) * K4 + kb; };
  const f32x4 acc = tile_gemm<KCH_, NW_, D_, BF>(smem, arow_of, brow_of, ks);
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  if (fused_arrive(smem, acc, false, a.P + (int64_t)s * B * H, B, H, b0, j0, f.cnt + tile, S))
    fused_pointwise<S, HAS_DH>(a, tn, tnp, b0, j0);
}

// stacked pair (decoder lstm2): grid (3 H/32, ceil(B/32), S) as lstm2_bwd_rec_kernel's.
// Launch for (t1, t0 = t1 + 1): layer-1 tiles (product 0, S jobs) finish layer 1's step
// t1 - 1; layer-0 tiles (products 2 and 1: 2S jobs, slab order = the two-launch path's) finish
// layer 0's step t1.  t0 = T: product 2 has no step and contributes zero slabs; t1 = 0: the
// layer-1 jobs have nothing left to finish and exit.
template <int KCH_, int NW_, int D_, bool BF, int S>
__global__ __launch_bounds__(64 * NW_) void lstm2_bwd_fused_kernel(BwdArgs a1, BwdArgs a0, const float* dG1,
                                                                  const float* dG0, int t1, int t0,
                                                                  const float* WT1, const float* WIT1,
                                                                  const float* WT0, FusedTile f) {
  using C = Tile<KCH_, NW_, D_>;
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  step_priority(a1.prio);
  const int B = a1.B, T = a1.T, H = a1.H;
  const int nt = H / TN, prod = blockIdx.x / nt, ct = blockIdx.x % nt, j0 = ct * TN;
  const int b0 = blockIdx.y * TB, s = blockIdx.z;
  if (prod == 0 && t1 == 0) return;
  const int K4 = BF ? 2 * H : 4 * H, ks = K4 / S, kb = s * ks;
  const float* dG = prod == 2 ? dG0 : dG1;
  const int t = prod == 2 ? t0 : t1;
  const float* WT = prod == 0 ? WT1 : (prod == 1 ? WIT1 : WT0);
  const bool none = t >= T;                                  // product 2 of the first launch
  auto arow_of = [&](int r) { return dG + ((int64_t)min(b0 + r, B - 1) * T + min(t, T - 1)) * K4 + kb; };
  auto brow_of = [&](int r) { return WT + (int64_t)(j0 + r) * K4 + kb; };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // timing-only ablation builds (tools/lstm_bwd_ablate.sh; wrong results by design):
  // AVC_ABL_EMPTY returns at once (launch boundary), AVC_ABL_NOMFMA skips the products,
  // AVC_ABL_NOARRIVE returns after them, AVC_ABL_NOTAIL skips the last arriver's pointwise pass
#ifdef AVC_ABL_EMPTY
  return;
#endif
#ifndef AVC_ABL_NOMFMA
  if (!none) acc = tile_gemm<KCH_, NW_, D_, BF>(smem, arow_of, brow_of, ks);
#endif
#ifdef AVC_ABL_NOARRIVE
  if (acc[0] == 12345.f) a1.P[0] = acc[1];
  return;
#endif
  const int64_t slab = (int64_t)B * H;
  const int ntile = gridDim.y * nt, tile = blockIdx.y * nt + ct;
  if (prod == 0) {
    if (fused_arrive(smem, acc, false, a1.P + s * slab, B, H, b0, j0, f.cnt + tile, S)) {
#ifndef AVC_ABL_NOTAIL
      fused_pointwise<S, true>(a1, t1 - 1, t1 - 2, b0, j0);
#endif
    }
  } else {
    // layer 0's slabs: [S of its own recurrence (product 2) | S of dG1 W_ih1 (product 1)]
    float* P = a0.P + (prod == 2 ? s : S + s) * slab;
    if (fused_arrive(smem, acc, none, P, B, H, b0, j0, f.cnt + ntile + tile, 2 * S)) {
#ifndef AVC_ABL_NOTAIL
      fused_pointwise<2 * S, false>(a0, t1, t1 - 1, b0, j0);
#endif
    }
  }
}

// Wide-tile recurrent products of the stacked backward (splits = 8): a workgroup owns all
// 64 batch rows x 64 output columns over 4H / 8 of K, so every weight row is fetched once
// per step instead of once per 32-row batch tile, and the per-CU operand bytes for the
// step's 3 x 64 x H outputs halve ((64 + 64) / (64 x 64) against (32 + 32) / (32 x 32) per
// output and k).  8 waves: wave w computes the 32 x 32 block (w & 3) of the tile over the
// k-half w >> 2 of each chunk as 2 x 2 v_mfma_f32_16x16x4_f32 (bf16: 16x16x32) tiles (four
// LDS fragment reads per 16 MFMAs instead of two per 4); the halves are summed through LDS.
// Staging, swizzle and prefetch are tile_gemm2's.
constexpr int TBW = 64, TNW = 64;
template <int KCH_, int D_, bool BF>
__device__ __forceinline__ void bwd_rec_body_wide(int B, int T, int H, const float* dG, int t, const float* WT,
                                                  float* P, int j0) {
  constexpr int NT = 512, SLOTS = KCH_ / 4, PER = TBW * SLOTS / NT, CF = (TBW + TNW) * KCH_;
  constexpr int SUB = KCH_ / 32;                           // 16-k sub-blocks per wave per chunk
  static_assert(PER * NT == TBW * SLOTS && TBW == TNW && SUB >= 1, "wide staging map");
  __shared__ __attribute__((aligned(16))) float lds[2 * CF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blockIdx.y * TBW, s = blockIdx.z, S = gridDim.z;
  const int K4 = BF ? 2 * H : 4 * H, ks = K4 / S, kb = s * ks;
  const float* arow[PER];
  const float* brow[PER];
  int srow[PER], spos[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + i * NT, r = e / SLOTS, sl = e % SLOTS;
    srow[i] = r;
    spos[i] = swz(sl, r);
    arow[i] = dG + ((int64_t)min(b0 + r, B - 1) * T + t) * K4 + kb + 4 * sl;
    brow[i] = WT + (int64_t)(j0 + r) * K4 + kb + 4 * sl;
  }
  const int nc = ks / KCH_;
  f32x4 sa[D_][PER], sb[D_][PER];
#pragma unroll
  for (int d = 0; d < D_; ++d) {
    const int cl = min(d, nc - 1);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      sa[d][i] = *reinterpret_cast<const f32x4*>(arow[i] + cl * KCH_);
      sb[d][i] = *reinterpret_cast<const f32x4*>(brow[i] + cl * KCH_);
    }
  }
  const int q = w & 3, kh = w >> 2, g = lane >> 4;
  const int ra0 = (q >> 1) * 32 + (lane & 15), rb0 = (q & 1) * 32 + (lane & 15);
  f32x4 acc[2][2] = {};
  for (int c0 = 0; c0 < nc; c0 += D_) {
#pragma unroll
    for (int d = 0; d < D_; ++d) {
      const int c = c0 + d;
      float* L = lds + (c & 1) * CF;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        *reinterpret_cast<f32x4*>(L + srow[i] * KCH_ + 4 * spos[i]) = sa[d][i];
        *reinterpret_cast<f32x4*>(L + (TBW + srow[i]) * KCH_ + 4 * spos[i]) = sb[d][i];
      }
      __syncthreads();
      const int cn = min(c + D_, nc - 1);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        sa[d][i] = *reinterpret_cast<const f32x4*>(arow[i] + cn * KCH_);
        sb[d][i] = *reinterpret_cast<const f32x4*>(brow[i] + cn * KCH_);
      }
      if (c < nc) {
#pragma unroll
        for (int sub = 0; sub < SUB; ++sub) {
          const int sl = (kh * SUB + sub) * 4 + g;
          f32x4 av[2], bv[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int ra = ra0 + 16 * i, rb = rb0 + 16 * i;
            av[i] = *reinterpret_cast<const f32x4*>(L + ra * KCH_ + 4 * swz(sl, ra));
            bv[i] = *reinterpret_cast<const f32x4*>(L + (TBW + rb) * KCH_ + 4 * swz(sl, rb));
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jn = 0; jn < 2; ++jn) {
              if constexpr (BF) {
                acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[i]),
                                                                     __builtin_bit_cast(bf16x8, bv[jn]), acc[i][jn],
                                                                     0, 0, 0);
              } else {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                  acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][jj], bv[jn][jj], acc[i][jn], 0, 0, 0);
              }
            }
        }
      }
    }
  }
  // k-halves: waves 4..7 leave their blocks in the (now idle) chunk buffers, waves 0..3 add
  __syncthreads();
  float* red = lds + q * 1024;
  if (kh == 1)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) *reinterpret_cast<f32x4*>(red + ((2 * i + jn) * 64 + lane) * 4) = acc[i][jn];
  __syncthreads();
  if (kh == 1) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const f32x4 o = *reinterpret_cast<const f32x4*>(red + ((2 * i + jn) * 64 + lane) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = b0 + (q >> 1) * 32 + 16 * i + 4 * g + r;
        if (b < B) P[((int64_t)s * B + b) * H + j0 + (q & 1) * 32 + 16 * jn + (lane & 15)] = acc[i][jn][r] + o[r];
      }
    }
}

// grid (3 H / 64, ceil(B / 64), S): x-tiles as lstm2_bwd_rec_kernel's, 64 columns each
template <int KCH_ = KCH, int D_ = DPF, bool BF = false>
__global__ __launch_bounds__(512) void lstm2_bwd_rec_wide_kernel(int B, int T, int H, const float* dG1,
                                                                 const float* dG0, int t1, int t0,
                                                                 const float* WT1, const float* WIT1,
                                                                 const float* WT0, float* P1, float* PQ0) {
  const int nt = H / TNW, prod = blockIdx.x / nt, j0 = (blockIdx.x % nt) * TNW;
  const int64_t slabs = (int64_t)gridDim.z * B * H;
  if (prod < 2) {
    if (t1 < 0) return;
    if (prod == 0) bwd_rec_body_wide<KCH_, D_, BF>(B, T, H, dG1, t1, WT1, P1, j0);
    else bwd_rec_body_wide<KCH_, D_, BF>(B, T, H, dG1, t1, WIT1, PQ0 + slabs, j0);
  } else {
    if (t0 >= T) return;
    bwd_rec_body_wide<KCH_, D_, BF>(B, T, H, dG0, t0, WT0, PQ0, j0);
  }
}

// ------------------------------------------------------------------ small H (BLSTM)
// Whole sequence, both directions in one launch.  grid = (ceil(B/2), ndir); block 256 =
// 2 batch rows x 32 units x 4 k-quarters.  gx: (B,T,ndir*4H) [dir-major blocks]; h out:
// (B,T,ndir*H).
constexpr int SH = 32;

// Latency layout: a step of the H = 32 recurrence is a 32-deep dot product per gate, so
// each (batch row, unit) gets a quad of lanes that split k (or, backward, the 4 gate
// blocks) four ways and combine with two DPP quad adds; a workgroup holds SB2 = 2 batch
// rows (256 threads, one wave per SIMD), so per-step VALU work per SIMD is a quarter of
// a thread-per-(b, j) layout, and B / 2 x ndir workgroups spread over as many CUs.
// Per-step operands (input-gate pre-activations; in backward the saved gates, cells and
// dh from above) are prefetched PD steps ahead into a register ring: the recurrence is a
// fraction of a microsecond per step, a load issued in its own step a full HBM round trip.
// The loop runs over T rounded up to PD with clamped addresses, so every load is
// unconditional and hipcc counts its waits precisely; steps past T store nothing.
constexpr int PD = 8, SB2 = 2, KQ = SH / 4;

__global__ __launch_bounds__(kThreads) void blstm_fwd_kernel(int B, int T, const float* gx, const float* Whh_f,
                                                            const float* Whh_b, float* hout, float* call,
                                                            float* gates, int ndir) {
  __shared__ __attribute__((aligned(16))) float hs[2][SB2][SH];
  const int dir = blockIdx.y;
  const int ks = threadIdx.x & 3, j = (threadIdx.x >> 2) & 31, bl = threadIdx.x >> 7;
  const int b = blockIdx.x * SB2 + bl;
  const int bc = min(b, B - 1);          // rows past B load a valid row, store nothing
  const float* W = dir ? Whh_b : Whh_f;
  float wr[4][KQ];                       // W_hh[q*SH + j][ks*KQ + kk]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < KQ; k += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(W + (q * SH + j) * SH + ks * KQ + k);
      wr[q][k] = v[0]; wr[q][k + 1] = v[1]; wr[q][k + 2] = v[2]; wr[q][k + 3] = v[3];
    }
  if (threadIdx.x < SB2 * SH) hs[0][threadIdx.x / SH][threadIdx.x % SH] = 0.f;
  __syncthreads();
  const int G = ndir * 4 * SH, HO = ndir * SH;
  // lane ks brings gate ks's input pre-activation; the quad sum adds it exactly once
  auto gsrc = [&](int s) {
    const int tt = min(s, T - 1);
    return gx + ((int64_t)bc * T + (dir ? T - 1 - tt : tt)) * G + dir * 4 * SH + ks * SH + j;
  };
  float gq[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) gq[d] = *gsrc(d);
  float c = 0.f;
  int cur = 0;
  const bool own = b < B;
  for (int s0 = 0; s0 < T; s0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int s = s0 + d;
      const int t = dir ? T - 1 - s : s;
      float acc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = q == ks ? gq[d] : 0.f;
      gq[d] = *gsrc(s + PD);
      const float* hr = &hs[cur][bl][ks * KQ];
      const f32x4 h0 = *reinterpret_cast<const f32x4*>(hr), h1 = *reinterpret_cast<const f32x4*>(hr + 4);
#pragma unroll
      for (int k = 0; k < KQ; ++k) {
        const float hv = k < 4 ? h0[k] : h1[k - 4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = fmaf(hv, wr[q][k], acc[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = avc_quad_xor_add<2>(avc_quad_xor_add<1>(acc[q]));
      const float i_ = avc_sigmoid_fast(acc[0]), f_ = avc_sigmoid_fast(acc[1]), g_ = avc_tanh_fast(acc[2]);
      const float o_ = avc_sigmoid_fast(acc[3]);
      c = f_ * c + i_ * g_;
      const float h = o_ * avc_tanh_fast(c);
      if (ks == 0) hs[cur ^ 1][bl][j] = h;
      if (own && s < T) {
        const int64_t o = ((int64_t)b * T + t) * HO + dir * SH + j;
        if (ks == 0) hout[o] = h;
        if (call && ks == 1) call[o] = c;
        if (gates) gates[((int64_t)b * T + t) * G + dir * 4 * SH + ks * SH + j] =
            ks == 0 ? i_ : ks == 1 ? f_ : ks == 2 ? g_ : o_;
      }
      cur ^= 1;
      __syncthreads();
    }
  }
}

// Backward of blstm_fwd_kernel: per direction, walk the sequence in reverse processing
// order.  dG: (B,T,ndir*4H).  dh_out: (B,T,ndir*H) or null (HAS_DH).  The quad of
// (b, j) computes the pointwise step redundantly, lane ks stores gate ks of dG, and the
// recurrent dh_rec[b][j] = sum_r dG[b][r] W[r][j] splits r by gate block (lane ks: rows
// ks*SH .. +SH, W_hh column j of that block in registers), summed by two DPP quad adds.
// dG_t goes through a double-buffered LDS row: one barrier per step.
template <bool HAS_DH>
__global__ __launch_bounds__(kThreads) void blstm_bwd_kernel(int B, int T, const float* dh_out, const float* gates,
                                                            const float* call, const float* Whh_f,
                                                            const float* Whh_b, float* dG, int ndir) {
  __shared__ __attribute__((aligned(16))) float dgs[2][SB2][4 * SH];
  const int dir = blockIdx.y;
  const int ks = threadIdx.x & 3, j = (threadIdx.x >> 2) & 31, bl = threadIdx.x >> 7;
  const int b = blockIdx.x * SB2 + bl;
  const int bc = min(b, B - 1);
  const float* W = dir ? Whh_b : Whh_f;
  float wc[SH];                          // W_hh[ks*SH + i][j]
#pragma unroll
  for (int i = 0; i < SH; ++i) wc[i] = W[(ks * SH + i) * SH + j];
  const int G = ndir * 4 * SH, HO = ndir * SH;
  // backward walk step s (0 = the forward's last step) -> time index
  auto tim = [&](int s) { const int ss = min(s, T - 1); return dir ? ss : T - 1 - ss; };
  struct Ops { float g[4], cc, cp, dh; };
  auto fetch = [&](Ops& o, int s) {
    const int t = tim(s);
    const int64_t bt = (int64_t)bc * T + t;
    const float* gs = gates + bt * G + dir * 4 * SH + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) o.g[q] = gs[q * SH];
    o.cc = call[bt * HO + dir * SH + j];
    const int tp = dir ? min(t + 1, T - 1) : max(t - 1, 0);   // previous step in forward order
    o.cp = call[((int64_t)bc * T + tp) * HO + dir * SH + j];
    o.dh = HAS_DH ? dh_out[bt * HO + dir * SH + j] : 0.f;
  };
  Ops ring[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) fetch(ring[d], d);
  float dcs = 0.f, dhr = 0.f;
  const bool own = b < B;
  int cur = 0;
  for (int s0 = 0; s0 < T; s0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int s = s0 + d;
      const Ops o = ring[d];
      fetch(ring[d], s + PD);
      const int t = tim(s);
      const float i_ = o.g[0], f_ = o.g[1], g_ = o.g[2], o_ = o.g[3];
      const float dh = dhr + o.dh;
      const float cp = s == T - 1 ? 0.f : o.cp;   // the forward's first step: c_prev = 0
      const float tc = avc_tanh_fast(o.cc);
      const float dc = dcs + dh * o_ * (1.f - tc * tc);
      const float di = dc * g_ * i_ * (1.f - i_);
      const float df = dc * cp * f_ * (1.f - f_);
      const float dg = dc * i_ * (1.f - g_ * g_);
      const float dO = dh * tc * o_ * (1.f - o_);
      dcs = dc * f_;
      const float mine = ks == 0 ? di : ks == 1 ? df : ks == 2 ? dg : dO;
      if (own && s < T) dG[((int64_t)b * T + t) * G + dir * 4 * SH + ks * SH + j] = mine;
      dgs[cur][bl][ks * SH + j] = own ? mine : 0.f;
      __syncthreads();
      const float* dr = &dgs[cur][bl][ks * SH];
      float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < SH; i += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(dr + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) part[e] = fmaf(v[e], wc[i + e], part[e]);
      }
      dhr = avc_quad_xor_add<2>(avc_quad_xor_add<1>((part[0] + part[1]) + (part[2] + part[3])));
      cur ^= 1;
    }
  }
}

bool lstm_shape_ok(int B, int H) { return B > 0 && H > 0 && H % 64 == 0; }

// the fused backward step (one launch per step) is the default; AVC_LSTM_BWD_FUSED=0 or
// autovc_lstm_bwd_set_fused(0) selects the product + pointwise launch pair (A/B and the
// bit-identity test); set_fused(-1) returns to the environment's choice
int g_bwd_fused = -1;
bool bwd_fused() {
  static const bool env = [] {
    const char* e = getenv("AVC_LSTM_BWD_FUSED");
    return !(e && e[0] == '0');
  }();
  return g_bwd_fused < 0 ? env : g_bwd_fused != 0;
}

int64_t ceil4(int64_t n) { return (n + 3) / 4 * 4; }
int64_t bwd_tiles(int B, int H) { return (int64_t)((B + TB - 1) / TB) * (H / TN); }

template <bool BF, int S>
void launch_lstm_fused_s(hipStream_t st, const BwdArgs& a, const float* dG, int t, int tn, int tnp, const float* WT,
                         FusedTile f) {
  const dim3 grid(a.H / TN, (a.B + TB - 1) / TB, S);
  if (a.dh_out)
    hipLaunchKernelGGL((lstm_bwd_fused_kernel<BKCH, BNW, BD, BF, S, true>), grid, dim3(64 * BNW), 0, st, a, dG, t, tn,
                       tnp, WT, f);
  else
    hipLaunchKernelGGL((lstm_bwd_fused_kernel<BKCH, BNW, BD, BF, S, false>), grid, dim3(64 * BNW), 0, st, a, dG, t, tn,
                       tnp, WT, f);
}

template <bool BF>
void launch_lstm_fused(hipStream_t st, const BwdArgs& a, const float* dG, int t, int tn, int tnp, const float* WT,
                       FusedTile f) {
  switch (a.S) {
    case 1: launch_lstm_fused_s<BF, 1>(st, a, dG, t, tn, tnp, WT, f); break;
    case 2: launch_lstm_fused_s<BF, 2>(st, a, dG, t, tn, tnp, WT, f); break;
    case 4: launch_lstm_fused_s<BF, 4>(st, a, dG, t, tn, tnp, WT, f); break;
    default: launch_lstm_fused_s<BF, 8>(st, a, dG, t, tn, tnp, WT, f); break;
  }
}

template <bool BF>
void launch_lstm2_fused(hipStream_t st, int S, const BwdArgs& a1, const BwdArgs& a0, const float* dG1,
                        const float* dG0, int t1, int t0, const float* w1, const float* wi, const float* w0,
                        FusedTile f) {
  const dim3 grid(3 * a1.H / TN, (a1.B + TB - 1) / TB, S);
  if (S == 4)
    hipLaunchKernelGGL((lstm2_bwd_fused_kernel<BKCH, BNW, BD, BF, 4>), grid, dim3(64 * BNW), 0, st, a1, a0, dG1, dG0,
                       t1, t0, w1, wi, w0, f);
  else
    hipLaunchKernelGGL((lstm2_bwd_fused_kernel<BKCH, BNW, BD, BF, 2>), grid, dim3(64 * BNW), 0, st, a1, a0, dG1, dG0,
                       t1, t0, w1, wi, w0, f);
}

// k-chunk of the tile GEMM: the tuned KCH when it divides K, else 64
template <int ABL = 0>
void launch_fwd_step(dim3 grid, hipStream_t st, const StepArgs& a, int t, int tp) {
  if (a.H % KCH == 0)
    hipLaunchKernelGGL((lstm_fwd_step_kernel<ABL, KCH, NWV, DPF>), grid, dim3(64 * NWV), 0, st, a, t, tp);
  else
    hipLaunchKernelGGL((lstm_fwd_step_kernel<ABL, 64, NWV, DPF>), grid, dim3(64 * NWV), 0, st, a, t, tp);
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" int autovc_lstm_fwd_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                   const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                   float* gates, int reverse, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && lstm_shape_ok(B, H), "autovc_lstm_fwd_f32: bad dims B=%d T=%d H=%d (H must be a multiple of 64)", B, T, H);
  AVC_CHECK_ARG(gx && W_hh && h && c_all, "autovc_lstm_fwd_f32: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh) && AVC_ALIGNED16(h) && (h_ldb % 4 == 0) && (h_ldt % 4 == 0),
                "autovc_lstm_fwd_f32: W_hh / h must be 16-byte aligned with strides %% 4 == 0");
  StepArgs a{B, T, H, gx, gx_ldb, gx_ldt, W_hh, h, h_ldb, h_ldt, c_all, gates, nullptr};
  const dim3 grid(H / UT, (B + TB - 1) / TB);
  for (int s = 0; s < T; ++s) {
    const int t = reverse ? T - 1 - s : s;
    const int tp = s == 0 ? -1 : (reverse ? t + 1 : t - 1);
    launch_fwd_step(grid, stream, a, t, tp);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_fwd_f32");
  return avc::kOk;
}

extern "C" int autovc_lstm2_fwd_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                    const float* W_hh0, const float* b_ih1, const float* b_hh1,
                                    const float* W_ih1, const float* W_hh1, float* h0, float* c0, float* gates0,
                                    float* h1, float* c1, float* gates1, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && lstm_shape_ok(B, H) && H % KCH == 0,
                "autovc_lstm2_fwd_f32: bad dims B=%d T=%d H=%d (H must be a multiple of %d)", B, T, H, KCH);
  AVC_CHECK_ARG(gx0 && W_hh0 && b_ih1 && b_hh1 && W_ih1 && W_hh1 && h0 && c0 && h1 && c1,
                "autovc_lstm2_fwd_f32: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh0) && AVC_ALIGNED16(W_ih1) && AVC_ALIGNED16(W_hh1) && AVC_ALIGNED16(h0) &&
                AVC_ALIGNED16(h1), "autovc_lstm2_fwd_f32: weights / h must be 16-byte aligned");
  Stack2Args a{StepArgs{B, T, H, gx0, gx_ldb, gx_ldt, W_hh0, h0, (int64_t)T * H, H, c0, gates0, nullptr},
               StepArgs{B, T, H, b_ih1, 0, 0, W_hh1, h1, (int64_t)T * H, H, c1, gates1, b_hh1}, W_ih1};
  const dim3 grid(H / UT, (B + TB - 1) / TB, 2);
  for (int t = 0; t <= T; ++t)
    hipLaunchKernelGGL((lstm2_fwd_step_kernel<KCH, NWV, DPF>), grid, dim3(64 * NWV), 0, stream, a, t);
  AVC_CHECK_LAUNCH("autovc_lstm2_fwd_f32");
  return avc::kOk;
}

// [S partial slabs | dc carry | fused-step tile counters]
extern "C" int64_t autovc_lstm_bwd_workspace_floats(int B, int H, int splits) {
  return (int64_t)splits * B * H + (int64_t)B * H + ceil4(bwd_tiles(B, H));
}

extern "C" int autovc_lstm_bwd_set_fused(int on) {
  AVC_CHECK_ARG(on >= -1 && on <= 1, "autovc_lstm_bwd_set_fused: -1, 0 or 1");
  g_bwd_fused = on;
  return avc::kOk;
}

namespace {
// the backward steps of one large-H layer in processing order: the first pointwise pass, then
// per step either one fused launch or the product + pointwise pair
template <bool BF>
int lstm_bwd_steps(const BwdArgs& a, int reverse, const float* dGsrc, const float* WT, float* workspace,
                   hipStream_t stream, const char* fn) {
  const int B = a.B, T = a.T, H = a.H;
  const bool fused = bwd_fused();
  FusedTile f{reinterpret_cast<int*>(workspace + (int64_t)(a.S + 1) * B * H)};
  if (fused && T > 1) AVC_HIP(avc::zero_async(f.cnt, 4 * ceil4(bwd_tiles(B, H)), stream), fn);
  const int64_t BH = (int64_t)B * H;
  const int pw_blocks = (int)((BH + 255) / 256);
  const dim3 rgrid(H / TN, (B + TB - 1) / TB, a.S);
  auto step_t = [&](int s) { return reverse ? T - 1 - s : s; };
  auto step_tp = [&](int s) { return s == 0 ? -1 : (reverse ? step_t(s) + 1 : step_t(s) - 1); };
  for (int s = T - 1; s >= 0; --s) {
    const int t = step_t(s);
    if (!fused || s == T - 1) launch_pointwise_any(pw_blocks, stream, a, t, step_tp(s), s == T - 1);
    if (s == 0) continue;
    if (fused)
      launch_lstm_fused<BF>(stream, a, dGsrc, t, step_t(s - 1), step_tp(s - 1), WT, f);
    else
      hipLaunchKernelGGL((lstm_bwd_rec_kernel<KCH, NWV, DPF, BF>), rgrid, dim3(64 * NWV), 0, stream, B, T, H, dGsrc,
                         t, WT, a.P);
  }
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}
}  // namespace

extern "C" int autovc_lstm_bwd_f32(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                                   const float* gates, const float* c_all, const float* W_hh_T, float* dG,
                                   int reverse, int splits, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && lstm_shape_ok(B, H), "autovc_lstm_bwd_f32: bad dims");
  AVC_CHECK_ARG((splits == 1 || splits == 2 || splits == 4 || splits == 8) && (4 * H) % (64 * splits) == 0,
                "autovc_lstm_bwd_f32: splits must be 1, 2, 4 or 8 and 4H must split into multiples of 64");
  AVC_CHECK_ARG(gates && c_all && W_hh_T && dG && workspace, "autovc_lstm_bwd_f32: null pointer");
  AVC_CHECK_ARG(!dh_out || (d_ldb % 4 == 0 && d_ldt % 4 == 0 && AVC_ALIGNED16(dh_out)),
                "autovc_lstm_bwd_f32: dh_out must be 16-byte aligned with strides %% 4 == 0");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_T) && AVC_ALIGNED16(dG), "autovc_lstm_bwd_f32: W_hh_T/dG alignment");
  float* P = workspace;
  float* dcs = workspace + (int64_t)splits * B * H;
  BwdArgs a{B, T, H, dh_out, d_ldb, d_ldt, gates, c_all, dG, dcs, P, splits};
  a.prio = lstm_prio();
  return lstm_bwd_steps<false>(a, reverse, dG, W_hh_T, workspace, stream, "autovc_lstm_bwd_f32");
}

// [P1: S slabs | PQ0: 2S slabs | dc carry layer 1 | dc carry layer 0 | fused-step tile counters]
extern "C" int64_t autovc_lstm2_bwd_workspace_floats(int B, int H, int splits) {
  return (int64_t)(3 * splits + 2) * B * H + ceil4(2 * bwd_tiles(B, H));
}

namespace {
// the stacked backward wavefront: launch pair s = 0..T of autovc_lstm2_bwd_f32, or (fused)
// the first pointwise pass and T fused launches
template <bool BF>
int lstm2_bwd_steps(const BwdArgs& a1, const BwdArgs& a0, int splits, const float* d1, const float* d0,
                    const float* w1, const float* wi, const float* w0, float* workspace, hipStream_t stream,
                    const char* fn) {
  const int B = a1.B, T = a1.T, H = a1.H;
  const int64_t BH = (int64_t)B * H;
  const bool wide = splits == 8;
  const bool fused = bwd_fused() && !wide;
  float* dcs0 = workspace + (int64_t)(3 * splits + 1) * BH;
  FusedTile f{reinterpret_cast<int*>(workspace + (int64_t)(3 * splits + 2) * BH)};
  if (fused) {
    // layer 0's carried cell gradient and the tile counters (contiguous); product 2 of the
    // first launch writes zero slabs itself
    AVC_HIP(avc::zero_async(dcs0, 4 * (BH + ceil4(2 * bwd_tiles(B, H))), stream), fn);
  } else {
    // layer 0's first processed step has no recurrent partials and no carried cell gradient
    AVC_HIP(avc::zero_async(a0.P, sizeof(float) * splits * BH, stream), fn);
    AVC_HIP(avc::zero_async(dcs0, sizeof(float) * BH, stream), fn);
  }
  const dim3 pgrid((H / 4 + 63) / 64, B, 2);
  const dim3 rgrid = wide ? dim3(3 * H / TNW, (B + TBW - 1) / TBW, splits) : dim3(3 * H / TN, (B + TB - 1) / TB, splits);
  for (int s = 0; s <= T; ++s) {
    const int t1 = T - 1 - s, t0 = T - s;
    if (!fused || s == 0) {
      if (splits == 8) hipLaunchKernelGGL((lstm2_bwd_pointwise_kernel<8>), pgrid, dim3(64), 0, stream, a1, a0, t1, t0);
      else if (splits == 4) hipLaunchKernelGGL((lstm2_bwd_pointwise_kernel<4>), pgrid, dim3(64), 0, stream, a1, a0, t1, t0);
      else hipLaunchKernelGGL((lstm2_bwd_pointwise_kernel<2>), pgrid, dim3(64), 0, stream, a1, a0, t1, t0);
    }
    if (s == T) break;
    if (fused)
      launch_lstm2_fused<BF>(stream, splits, a1, a0, d1, d0, t1, t0, w1, wi, w0, f);
    else if (wide)
      hipLaunchKernelGGL((lstm2_bwd_rec_wide_kernel<KCH, DPF, BF>), rgrid, dim3(512), 0, stream, B, T, H, d1, d0, t1,
                         t0, w1, wi, w0, a1.P, a0.P);
    else
      hipLaunchKernelGGL((lstm2_bwd_rec_kernel<KCH, NWV, DPF, BF>), rgrid, dim3(64 * NWV), 0, stream, B, T, H, d1, d0,
                         t1, t0, w1, wi, w0, a1.P, a0.P);
  }
  AVC_CHECK_LAUNCH(fn);
  return avc::kOk;
}
}  // namespace

// Backward of two stacked layers (decoder lstm2) as a one-step-lagged wavefront, the
// mirror of autovc_lstm2_fwd_f32: launch pair s = 0..T runs layer 1 at t1 = T-1-s and
// layer 0 at t0 = T-s.  Layer 1's input gradient dG1_t W_ih1 (layer 0's dh_t) is a third
// product of the recurrent launch instead of a GEMM over all frames after layer 1 ends,
// and layer 0 starts one step behind layer 1 instead of T steps.  Same per-element sums
// as the unstacked path except that layer 0's dh_t adds its 2S partials in one order.
extern "C" int autovc_lstm2_bwd_f32(int B, int T, int H, const float* dh1_out, int64_t d_ldb, int64_t d_ldt,
                                    const float* gates1, const float* c1, const float* gates0, const float* c0,
                                    const float* W_hh1_T, const float* W_ih1_T, const float* W_hh0_T, float* dG1,
                                    float* dG0, int splits, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && lstm_shape_ok(B, H), "autovc_lstm2_bwd_f32: bad dims");
  AVC_CHECK_ARG((splits == 2 || splits == 4 || splits == 8) && (4 * H) % (KCH * splits) == 0 &&
                    (splits < 8 || H % TNW == 0),
                "autovc_lstm2_bwd_f32: splits must be 2, 4 or 8 with 4H a multiple of %d x splits", KCH);
  AVC_CHECK_ARG(dh1_out && gates1 && c1 && gates0 && c0 && W_hh1_T && W_ih1_T && W_hh0_T && dG1 && dG0 && workspace,
                "autovc_lstm2_bwd_f32: null pointer");
  AVC_CHECK_ARG(d_ldb % 4 == 0 && d_ldt % 4 == 0 && AVC_ALIGNED16(dh1_out) && AVC_ALIGNED16(W_hh1_T) &&
                AVC_ALIGNED16(W_ih1_T) && AVC_ALIGNED16(W_hh0_T) && AVC_ALIGNED16(dG1) && AVC_ALIGNED16(dG0),
                "autovc_lstm2_bwd_f32: operands must be 16-byte aligned with strides %% 4 == 0");
  const int64_t BH = (int64_t)B * H;
  float* P1 = workspace;
  float* PQ0 = P1 + splits * BH;            // [S slabs of layer 0's recurrence | S slabs of dG1 W_ih1]
  float* dcs1 = PQ0 + 2 * splits * BH;
  float* dcs0 = dcs1 + BH;
  BwdArgs a1{B, T, H, dh1_out, d_ldb, d_ldt, gates1, c1, dG1, dcs1, P1, splits};
  BwdArgs a0{B, T, H, nullptr, 0, 0, gates0, c0, dG0, dcs0, PQ0, 2 * splits};
  a1.prio = a0.prio = lstm_prio();
  // splits 8: the wide-tile products (64 x 64 per workgroup, never fused); 2 / 4: 32 x 32 tiles
  return lstm2_bwd_steps<false>(a1, a0, splits, dG1, dG0, W_hh1_T, W_ih1_T, W_hh0_T, workspace, stream,
                                "autovc_lstm2_bwd_f32");
}

extern "C" int autovc_blstm_fwd_f32(int B, int T, int H, int ndir, const float* gx, const float* W_hh_f,
                                    const float* W_hh_b, float* h, float* c_all, float* gates, hipStream_t stream) {
  AVC_CHECK_ARG(H == SH, "autovc_blstm_fwd_f32: small-H kernel is built for H=%d (got %d)", SH, H);
  AVC_CHECK_ARG(B > 0 && T > 0 && (ndir == 1 || ndir == 2), "autovc_blstm_fwd_f32: bad dims");
  AVC_CHECK_ARG(gx && W_hh_f && h && c_all && (ndir == 1 || W_hh_b), "autovc_blstm_fwd_f32: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_f) && (ndir == 1 || AVC_ALIGNED16(W_hh_b)), "autovc_blstm_fwd_f32: W alignment");
  hipLaunchKernelGGL(blstm_fwd_kernel, dim3((B + SB2 - 1) / SB2, ndir), dim3(kThreads), 0, stream, B, T, gx,
                     W_hh_f, W_hh_b, h, c_all, gates, ndir);
  AVC_CHECK_LAUNCH("autovc_blstm_fwd_f32");
  return avc::kOk;
}

extern "C" int autovc_blstm_bwd_f32(int B, int T, int H, int ndir, const float* dh_out, const float* gates,
                                    const float* c_all, const float* W_hh_f, const float* W_hh_b, float* dG,
                                    hipStream_t stream) {
  AVC_CHECK_ARG(H == SH, "autovc_blstm_bwd_f32: small-H kernel is built for H=%d (got %d)", SH, H);
  AVC_CHECK_ARG(B > 0 && T > 0 && (ndir == 1 || ndir == 2), "autovc_blstm_bwd_f32: bad dims");
  AVC_CHECK_ARG(gates && c_all && W_hh_f && dG && (ndir == 1 || W_hh_b), "autovc_blstm_bwd_f32: null pointer");
  if (dh_out)
    hipLaunchKernelGGL(blstm_bwd_kernel<true>, dim3((B + SB2 - 1) / SB2, ndir), dim3(kThreads), 0, stream, B, T,
                       dh_out, gates, c_all, W_hh_f, W_hh_b, dG, ndir);
  else
    hipLaunchKernelGGL(blstm_bwd_kernel<false>, dim3((B + SB2 - 1) / SB2, ndir), dim3(kThreads), 0, stream, B, T,
                       dh_out, gates, c_all, W_hh_f, W_hh_b, dG, ndir);
  AVC_CHECK_LAUNCH("autovc_blstm_bwd_f32");
  return avc::kOk;
}

// ------------------------------------------------------------------ measurement
// Same launches as autovc_lstm_fwd_f32, each bracketed by hipExtLaunchKernelGGL's own
// start/stop events (timestamps taken by the dispatch itself, so the inter-kernel gap is
// excluded); synchronises and writes the mean per-launch kernel time in microseconds to
// *avg_us (host).  Used by bench.py for the roofline of the recurrent kernel.
extern "C" int autovc_lstm_fwd_timed_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                         const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                         float* gates, hipStream_t stream, float* avg_us) {
  AVC_CHECK_ARG(T > 1 && lstm_shape_ok(B, H) && avg_us, "autovc_lstm_fwd_timed_f32: bad args");
  AVC_CHECK_ARG(gx && W_hh && h && c_all, "autovc_lstm_fwd_timed_f32: null pointer");
  StepArgs a{B, T, H, gx, gx_ldb, gx_ldt, W_hh, h, h_ldb, h_ldt, c_all, gates, nullptr};
  const dim3 grid(H / UT, (B + TB - 1) / TB);
  hipEvent_t* ev = new hipEvent_t[2 * T];
  for (int i = 0; i < 2 * T; ++i) AVC_HIP(hipEventCreate(&ev[i]), "autovc_lstm_fwd_timed_f32/event");
  for (int s = 0; s < T; ++s) {
    const int tp = s == 0 ? -1 : s - 1;
    if (H % KCH == 0)
      hipExtLaunchKernelGGL((lstm_fwd_step_kernel<0, KCH, NWV, DPF>), grid, dim3(64 * NWV), 0, stream, ev[2 * s],
                            ev[2 * s + 1], 0, a, s, tp);
    else
      hipExtLaunchKernelGGL((lstm_fwd_step_kernel<0, 64, NWV, DPF>), grid, dim3(64 * NWV), 0, stream, ev[2 * s],
                            ev[2 * s + 1], 0, a, s, tp);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_fwd_timed_f32");
  AVC_HIP(hipStreamSynchronize(stream), "autovc_lstm_fwd_timed_f32/sync");
  double tot = 0.0;
  int n = 0;
  for (int s = 1; s < T; ++s) {  // step 0 has no recurrent product: excluded from the mean
    float ms = 0.f;
    AVC_HIP(hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]), "autovc_lstm_fwd_timed_f32/elapsed");
    tot += ms;
    ++n;
  }
  for (int i = 0; i < 2 * T; ++i) (void)hipEventDestroy(ev[i]);
  delete[] ev;
  *avg_us = (float)(tot / n * 1000.0);
  return avc::kOk;
}

// ------------------------------------------------------------------ bf16 recurrences
// precision "bf16" (BASELINE config 3): the recurrent products read bf16 copies of W
// (RNE-rounded by the caller) and of h / dG (written by the step epilogues); cell math,
// c, gates, h and dG stay fp32.  h is (B, T, H) contiguous.
namespace {
bool bf16_shape_ok(int B, int H) { return B > 0 && H > 0 && H % 128 == 0; }
}

extern "C" int autovc_lstm_fwd_bf16(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                    const uint16_t* W_hh_b, float* h, uint16_t* h_b, float* c_all, float* gates,
                                    int reverse, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && bf16_shape_ok(B, H), "autovc_lstm_fwd_bf16: bad dims B=%d T=%d H=%d (H %% 128 != 0)", B, T, H);
  AVC_CHECK_ARG(gx && W_hh_b && h && h_b && c_all, "autovc_lstm_fwd_bf16: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_b) && AVC_ALIGNED16(h_b), "autovc_lstm_fwd_bf16: bf16 operands must be 16-byte aligned");
  StepArgs a{B, T, H, gx, gx_ldb, gx_ldt, nullptr, h, (int64_t)T * H, H, c_all, gates, nullptr,
             reinterpret_cast<const __bf16*>(W_hh_b), reinterpret_cast<__bf16*>(h_b)};
  const dim3 grid(H / UT, (B + TB - 1) / TB);
  for (int s = 0; s < T; ++s) {
    const int t = reverse ? T - 1 - s : s;
    const int tp = s == 0 ? -1 : (reverse ? t + 1 : t - 1);
    hipLaunchKernelGGL((lstm_fwd_step_kernel<0, KCH, NWV, DPF, true>), grid, dim3(64 * NWV), 0, stream, a, t, tp);
  }
  AVC_CHECK_LAUNCH("autovc_lstm_fwd_bf16");
  return avc::kOk;
}

extern "C" int autovc_lstm2_fwd_bf16(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                     const uint16_t* W_hh0_b, const float* b_ih1, const float* b_hh1,
                                     const uint16_t* W_ih1_b, const uint16_t* W_hh1_b, float* h0, uint16_t* h0_b,
                                     float* c0, float* gates0, float* h1, uint16_t* h1_b, float* c1, float* gates1,
                                     hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && bf16_shape_ok(B, H), "autovc_lstm2_fwd_bf16: bad dims B=%d T=%d H=%d", B, T, H);
  AVC_CHECK_ARG(gx0 && W_hh0_b && b_ih1 && b_hh1 && W_ih1_b && W_hh1_b && h0 && h0_b && c0 && h1 && h1_b && c1,
                "autovc_lstm2_fwd_bf16: null pointer");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh0_b) && AVC_ALIGNED16(W_ih1_b) && AVC_ALIGNED16(W_hh1_b) && AVC_ALIGNED16(h0_b) &&
                AVC_ALIGNED16(h1_b), "autovc_lstm2_fwd_bf16: bf16 operands must be 16-byte aligned");
  Stack2Args a{StepArgs{B, T, H, gx0, gx_ldb, gx_ldt, nullptr, h0, (int64_t)T * H, H, c0, gates0, nullptr,
                        reinterpret_cast<const __bf16*>(W_hh0_b), reinterpret_cast<__bf16*>(h0_b)},
               StepArgs{B, T, H, b_ih1, 0, 0, nullptr, h1, (int64_t)T * H, H, c1, gates1, b_hh1,
                        reinterpret_cast<const __bf16*>(W_hh1_b), reinterpret_cast<__bf16*>(h1_b)},
               nullptr, reinterpret_cast<const __bf16*>(W_ih1_b)};
  const dim3 grid(H / UT, (B + TB - 1) / TB, 2);
  for (int t = 0; t <= T; ++t)
    hipLaunchKernelGGL((lstm2_fwd_step_kernel<KCH, NWV, DPF, true>), grid, dim3(64 * NWV), 0, stream, a, t);
  AVC_CHECK_LAUNCH("autovc_lstm2_fwd_bf16");
  return avc::kOk;
}

extern "C" int autovc_lstm_bwd_bf16(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                                    const float* gates, const float* c_all, const uint16_t* W_hh_T_b, float* dG,
                                    uint16_t* dG_b, int reverse, int splits, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && bf16_shape_ok(B, H), "autovc_lstm_bwd_bf16: bad dims");
  AVC_CHECK_ARG((splits == 1 || splits == 2 || splits == 4 || splits == 8) && (2 * H) % (KCH * splits) == 0,
                "autovc_lstm_bwd_bf16: splits must be 1, 2, 4 or 8 with 2H/splits a multiple of %d", KCH);
  AVC_CHECK_ARG(gates && c_all && W_hh_T_b && dG && dG_b && workspace, "autovc_lstm_bwd_bf16: null pointer");
  AVC_CHECK_ARG(!dh_out || (d_ldb % 4 == 0 && d_ldt % 4 == 0 && AVC_ALIGNED16(dh_out)),
                "autovc_lstm_bwd_bf16: dh_out must be 16-byte aligned with strides %% 4 == 0");
  AVC_CHECK_ARG(AVC_ALIGNED16(W_hh_T_b) && AVC_ALIGNED16(dG_b), "autovc_lstm_bwd_bf16: alignment");
  float* P = workspace;
  float* dcs = workspace + (int64_t)splits * B * H;
  BwdArgs a{B, T, H, dh_out, d_ldb, d_ldt, gates, c_all, dG, dcs, P, splits, reinterpret_cast<__bf16*>(dG_b)};
  a.prio = lstm_prio();
  return lstm_bwd_steps<true>(a, reverse, reinterpret_cast<const float*>(dG_b), reinterpret_cast<const float*>(W_hh_T_b),
                              workspace, stream, "autovc_lstm_bwd_bf16");
}

// autovc_lstm2_bwd_f32 with the recurrent products on bf16 copies (precision "bf16"): the
// pointwise passes also write dG1_b / dG0_b, which the next launch's products read; W*T_b are
// RNE bf16 copies of the (H, 4H) transposes.  Cell backward, dG, partials fp32.
extern "C" int autovc_lstm2_bwd_bf16(int B, int T, int H, const float* dh1_out, int64_t d_ldb, int64_t d_ldt,
                                     const float* gates1, const float* c1, const float* gates0, const float* c0,
                                     const uint16_t* W_hh1_T_b, const uint16_t* W_ih1_T_b, const uint16_t* W_hh0_T_b,
                                     float* dG1, uint16_t* dG1_b, float* dG0, uint16_t* dG0_b, int splits,
                                     float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(T > 0 && bf16_shape_ok(B, H), "autovc_lstm2_bwd_bf16: bad dims");
  AVC_CHECK_ARG((splits == 2 || splits == 4 || splits == 8) && (2 * H) % (KCH * splits) == 0 &&
                    (splits < 8 || H % TNW == 0),
                "autovc_lstm2_bwd_bf16: splits must be 2, 4 or 8 with 2H a multiple of %d x splits", KCH);
  AVC_CHECK_ARG(dh1_out && gates1 && c1 && gates0 && c0 && W_hh1_T_b && W_ih1_T_b && W_hh0_T_b && dG1 && dG1_b &&
                dG0 && dG0_b && workspace, "autovc_lstm2_bwd_bf16: null pointer");
  AVC_CHECK_ARG(d_ldb % 4 == 0 && d_ldt % 4 == 0 && AVC_ALIGNED16(dh1_out) && AVC_ALIGNED16(W_hh1_T_b) &&
                AVC_ALIGNED16(W_ih1_T_b) && AVC_ALIGNED16(W_hh0_T_b) && AVC_ALIGNED16(dG1_b) && AVC_ALIGNED16(dG0_b),
                "autovc_lstm2_bwd_bf16: operands must be 16-byte aligned with strides %% 4 == 0");
  const int64_t BH = (int64_t)B * H;
  float* P1 = workspace;
  float* PQ0 = P1 + splits * BH;
  float* dcs1 = PQ0 + 2 * splits * BH;
  float* dcs0 = dcs1 + BH;
  BwdArgs a1{B, T, H, dh1_out, d_ldb, d_ldt, gates1, c1, dG1, dcs1, P1, splits, reinterpret_cast<__bf16*>(dG1_b)};
  BwdArgs a0{B, T, H, nullptr, 0, 0, gates0, c0, dG0, dcs0, PQ0, 2 * splits, reinterpret_cast<__bf16*>(dG0_b)};
  a1.prio = a0.prio = lstm_prio();
  return lstm2_bwd_steps<true>(a1, a0, splits, reinterpret_cast<const float*>(dG1_b),
                               reinterpret_cast<const float*>(dG0_b), reinterpret_cast<const float*>(W_hh1_T_b),
                               reinterpret_cast<const float*>(W_ih1_T_b), reinterpret_cast<const float*>(W_hh0_T_b),
                               workspace, stream, "autovc_lstm2_bwd_bf16");
}

// The product's decoder-lstm2 launch (autovc_lstm2_fwd_f32's two-layer wavefront) with every
// launch bracketed by its dispatch events; *avg_us (host) = mean over launches 2..T-1 (both
// layers carry a recurrent product there).  bench.py's roofline of the dominant LSTM kernel.
extern "C" int autovc_lstm2_fwd_timed_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                          const float* W_hh0, const float* b_ih1, const float* b_hh1,
                                          const float* W_ih1, const float* W_hh1, float* h0, float* c0,
                                          float* gates0, float* h1, float* c1, float* gates1, hipStream_t stream,
                                          float* avg_us) {
  AVC_CHECK_ARG(T > 3 && lstm_shape_ok(B, H) && H % KCH == 0 && avg_us, "autovc_lstm2_fwd_timed_f32: bad args");
  AVC_CHECK_ARG(gx0 && W_hh0 && b_ih1 && b_hh1 && W_ih1 && W_hh1 && h0 && c0 && h1 && c1,
                "autovc_lstm2_fwd_timed_f32: null pointer");
  Stack2Args a{StepArgs{B, T, H, gx0, gx_ldb, gx_ldt, W_hh0, h0, (int64_t)T * H, H, c0, gates0, nullptr},
               StepArgs{B, T, H, b_ih1, 0, 0, W_hh1, h1, (int64_t)T * H, H, c1, gates1, b_hh1}, W_ih1};
  const dim3 grid(H / UT, (B + TB - 1) / TB, 2);
  hipEvent_t* ev = new hipEvent_t[2 * (T + 1)];
  for (int i = 0; i < 2 * (T + 1); ++i) AVC_HIP(hipEventCreate(&ev[i]), "autovc_lstm2_fwd_timed_f32/event");
  for (int t = 0; t <= T; ++t)
    hipExtLaunchKernelGGL((lstm2_fwd_step_kernel<KCH, NWV, DPF>), grid, dim3(64 * NWV), 0, stream, ev[2 * t],
                          ev[2 * t + 1], 0, a, t);
  AVC_CHECK_LAUNCH("autovc_lstm2_fwd_timed_f32");
  AVC_HIP(hipStreamSynchronize(stream), "autovc_lstm2_fwd_timed_f32/sync");
  double tot = 0.0;
  int n = 0;
  for (int t = 2; t < T; ++t) {
    float ms = 0.f;
    AVC_HIP(hipEventElapsedTime(&ms, ev[2 * t], ev[2 * t + 1]), "autovc_lstm2_fwd_timed_f32/elapsed");
    tot += ms;
    ++n;
  }
  for (int i = 0; i < 2 * (T + 1); ++i) (void)hipEventDestroy(ev[i]);
  delete[] ev;
  *avg_us = (float)(tot / n * 1000.0);
  return avc::kOk;
}
