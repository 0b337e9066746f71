// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32), with an implicit
// im2col operand mode for AutoVC's Conv1d(k=5, pad=2) layers.
//
//   C[M,N] (row-major, ldc) = sum_k A(m,k) * B(k,n)  (+ bias1[n] + bias2[n]) (+ C_old)
//
// Operand storage ("RK" = row index r, K contiguous; "CK" = K rows, r contiguous):
//   A: a_trans=0 -> A(m,k) = A[m*lda + k]     a_trans=1 -> A(m,k) = A[k*lda + m]
//   B: b_trans=0 -> B(k,n) = B[n*ldb + k]     b_trans=1 -> B(k,n) = B[k*ldb + n]
// Conv mask (per operand, conv_T > 0): the operand is a (frames x taps*C) im2col view
// of an NTC activation X (B, T, C) with frame stride ld: element (f, q) =
// X[(f + tap0)*ld + q] when 0 <= f%T + q/C + tap0 < T, else 0 (for taps > 1 the
// activation must be contiguous, ld == C, so q = tap*C + c walks into the next frames).
// f is the row index for RK operands and the K index for CK operands; q is the
// contiguous index.  This serves
//   forward   y   = conv(x)          : A = im2col(x)  (RK, tap0 = -2), B = W'[co][k*C+ci]
//   backward  dx  = conv^T(dy)       : A = im2col(dy) (RK, tap0 = -2), B = W''[k*Co+co][ci]
//   backward  dW' = dy^T im2col(x)   : A = dy (CK),   B = im2col(x) (CK, tap0 = -2)
//   LSTM      dW_hh = dG^T h_{t-1}   : B = h shifted one frame (CK, C = H, tap0 = -1)
// (Conv1d semantics: model_vc_mel.py:20-38,49-59,92-102,132-161.)
//
// Tiling (templated, picked per shape): block tile BM x BN, k-stage BK, 4 waves each
// owning (WM/32) x (WN/32) MFMA 32x32 tiles.  RK operands sit in LDS as [row][BK+4]
// (row stride keeps the ds_read_b128 fragment reads conflict-free), CK operands as
// [BK][rows+4] (staged by coalesced float4 rows, read with ds_read_b32).  Within a stage
// lane half h takes k = h*BK/2 + p for MFMA p (the k order inside a stage is a
// permutation applied to A and B alike, so the sum is unchanged).  Register-staged double
// buffer, one barrier per stage; XCD-aware tile order.  Split-K writes fp32 slabs
// reduced in k order by a second kernel (deterministic; no float atomics).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

struct Opnd {
  const float* p;
  int64_t ld;
  int conv_T, conv_C, tap0;  // conv_T == 0: plain matrix
  // BatchNorm + activation on load (bf16 kernel, BN instantiations only; conv operands):
  // element = act(coef[c] x + coef[C + c]) for a frame inside its sequence, else 0
  const float* coef;
  int act;
};

// the fused Conv-BN stacks' transform of a stored pre-BN value (bn.hip apply_kernel's fmaf).
// ACT is a template argument: with a runtime activation the compiler evaluated every branch
// (two transcendentals per element) for every layer — 2.4x the GEMM time.
// tanh: common.h's v_exp_f32 + v_rcp_f32 form (~1e-7 absolute); the value is rounded to
// bf16 right away, and the stack's backward recomputes it the same way
template <int ACT>
__device__ __forceinline__ float bn_act(float x, float a, float s) {
  const float p = fmaf(x, a, s);
  return ACT == 1 ? fmaxf(p, 0.f) : (ACT == 2 ? avc_tanh_fast(p) : p);
}

// (alpha, shift) of a BN-on-load operand's channels, staged in LDS once per workgroup
constexpr int kBnMaxC = 1024;

// Batched launch (c != 0): blockIdx.z is the batch index, the operands and C of batch z
// start z * (a, b, c) floats further (no split-K then).
struct Batch {
  int64_t a, b, c;
};

// One operand tile (ROWS x BK) of a stage: staging map, LDS image and fragment reads.
//   RK: LDS [ROWS][BK+4], staged as float4 along k, fragments read with ds_read_b128.
//   CK: LDS [BK][ROWS+4], staged as float4 along rows (coalesced), fragments ds_read_b32.
// Loads are buffer loads (32-bit byte offsets from the operand base, descriptor range
// 2 GiB): every masked element (row past the operand, k past K, conv tap outside its
// sequence) gets an out-of-range offset and reads as zero in hardware, so the k loop has
// no branches and a handful of VALU per float4.  The staging map gives every slot of a
// thread the same k (RK) or the same row (CK), so the k/tap bookkeeping of RK operands
// and the row/tap state of CK operands are per thread, not per slot.
constexpr uint32_t kOOB = 0x80000000u;   // >= the descriptor's num_records: reads return 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)kOOB, 0x00020000);
}

// EB: bytes per element of the operand in memory — 4 (fp32) or 2 (bf16, the bf16 kernel's
// "bf16 source" operands: copies written by their producers, staged into the bf16 LDS image
// as they are).  A slot is always 16 bytes: VE = 4 fp32 or 8 bf16 elements.
template <bool RK, int ROWS, int BK, int NT, int EB = 4>
struct OpTile {
  static constexpr int VE = 16 / EB;                 // elements per 16-byte slot
  static constexpr int LD = RK ? BK + 4 : ROWS + 4;
  static constexpr int FLOATS = RK ? ROWS * LD : BK * LD;
  static constexpr int F4 = ROWS * BK / VE;          // slots per stage
  static constexpr int PER = F4 / NT;
  static_assert(PER * NT == F4, "staging map");
  static_assert(RK ? NT % (BK / VE) == 0 : NT % (ROWS / VE) == 0, "slots of a thread share k (RK) / row (CK)");
  f32x4 v[PER];             // 16 raw bytes per slot (4 fp32 or 8 bf16)
  f32x4 v2[PER];            // second staging set (bf16 kernel: two stages in flight)
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t off[PER];        // byte offset of the slot's next 16 bytes (valid when unmasked)
  bool rok[PER];            // RK: row inside the operand
  int tpos[PER];            // conv: frame position in its sequence (RK: fixed; CK: advancing)
  int kpos[PER];            // CK: frame index of the slot
  int kk;                   // RK: k of the thread's slots
  int tap, kmod;            // conv: RK: k / C, k % C (advancing); CK: q / C (fixed)
  int step_q, step_r;       // conv: RK: BK / C, BK % C; CK: -, BK % T (uniform)
  bool rowok;               // CK: the thread's row inside the operand
  int kch[2];               // BN on load: the staged set's first channel (RK: per stage; CK: fixed)
  uint32_t okm[2];          // BN on load: slots of the staged set inside their sequence
  // slot i of this thread -> (row r, k)
  __device__ __forceinline__ static void coords(int i, int& r, int& k) {
    const int e = threadIdx.x + i * NT;
    if (RK) { r = e / (BK / VE); k = VE * (e % (BK / VE)); }
    else    { k = e / (ROWS / VE); r = VE * (e % (ROWS / VE)); }
  }
  __device__ __forceinline__ void init(const Opnd& o, int64_t r0, int64_t kbeg, int64_t R) {
    rsrc = make_rsrc(o.p);
    const int shift = o.conv_T > 0 ? o.tap0 : 0;   // tap0 only means something for a conv view
    if (o.conv_T > 0) {
      step_q = RK ? BK / o.conv_C : 0;
      step_r = RK ? BK % o.conv_C : BK % o.conv_T;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int rr, kq;
      coords(i, rr, kq);
      const int64_t r = r0 + rr, k = kbeg + kq;
      if (RK) {
        rok[i] = r < R;
        off[i] = (uint32_t)((((r + shift) * o.ld) + k) * EB);
        if (o.conv_T > 0) tpos[i] = (int)(r % o.conv_T);
        if (i == 0) {
          kk = (int)k;
          if (o.conv_T > 0) { tap = (int)(k / o.conv_C); kmod = (int)(k % o.conv_C); }
        }
      } else {
        kpos[i] = (int)k;
        off[i] = (uint32_t)((((k + shift) * o.ld) + r) * EB);
        if (o.conv_T > 0) tpos[i] = (int)(k % o.conv_T);
        if (i == 0) {
          rowok = r < R;
          if (o.conv_T > 0) tap = (int)(r / o.conv_C);
          if (o.conv_T > 0) kch[0] = kch[1] = rowok ? (int)(r % o.conv_C) : 0;   // rows = channels c .. c+3
        }
      }
    }
  }
  __device__ __forceinline__ void load(const Opnd& o, int64_t K) { load_to(o, K, v); }
  // load into set SET; BN: also record which slots are inside their sequence and (RK) the
  // stage's channel coefficients, for the transform applied when the set is stored
  template <bool BN, int SET>
  __device__ __forceinline__ void load_s(const Opnd& o, int64_t K) {
    if constexpr (BN) {
      uint32_t m = 0;
      if (RK) {
        const bool kin = kk < K;
        const int tt0 = tap + o.tap0;
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (rok[i] && kin && (unsigned)(tpos[i] + tt0) < (unsigned)o.conv_T) m |= 1u << i;
        kch[SET] = kmod;
      } else {
        const int tt0 = tap + o.tap0;
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (rowok && kpos[i] < K && (unsigned)(tpos[i] + tt0) < (unsigned)o.conv_T) m |= 1u << i;
      }
      okm[SET] = m;
    }
    load_to(o, K, SET ? v2 : v);
  }
  // the next stage's loads into `dst` (v or v2); the address state advances by one stage
  __device__ __forceinline__ void load_to(const Opnd& o, int64_t K, f32x4 (&dst)[PER]) {
    if (RK) {
      const bool kin = kk < K;
      const int tt0 = tap + o.tap0;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        bool ok = rok[i] && kin;
        if (o.conv_T > 0) ok = ok && (unsigned)(tpos[i] + tt0) < (unsigned)o.conv_T;
        dst[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? off[i] : kOOB, 0, 0));
        off[i] += BK * EB;
      }
      kk += BK;
      if (o.conv_T > 0) {   // k += BK as (tap, kmod) with the uniform BK / C, BK % C
        tap += step_q;
        kmod += step_r;
        if (kmod >= o.conv_C) { kmod -= o.conv_C; ++tap; }
      }
    } else {
      const int tt0 = tap + o.tap0;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        bool ok = rowok && kpos[i] < K;
        if (o.conv_T > 0) ok = ok && (unsigned)(tpos[i] + tt0) < (unsigned)o.conv_T;
        dst[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? off[i] : kOOB, 0, 0));
        off[i] += (uint32_t)(BK * o.ld * EB);
        kpos[i] += BK;
        if (o.conv_T > 0) {   // (frame + BK) % T with the uniform BK % T
          tpos[i] += step_r;
          if (tpos[i] >= o.conv_T) tpos[i] -= o.conv_T;
        }
      }
    }
  }
  template <int SET = 0>
  __device__ __forceinline__ void store(float* lds) const {
    const f32x4 (&src)[PER] = SET ? v2 : v;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int r, k;
      coords(i, r, k);
      *reinterpret_cast<f32x4*>(lds + (RK ? r * LD + k : k * LD + r)) = src[i];
    }
  }
  // bf16 image [row][LDB] (k contiguous) of an RK operand: each slot as one 8-byte write
  // BN: slot values become bn_act(value) (inside the sequence) or 0 before the rounding
  // cl: the (alpha | shift) table in LDS (kBnMaxC floats each), al / sh: this set's channels
  template <int ACT, int SET>
  __device__ __forceinline__ f32x4 staged(int i, const f32x4& al, const f32x4& sh) const {
    const f32x4 x = SET ? v2[i] : v[i];
    if constexpr (ACT < 0) return x;
    else {
      if (!((okm[SET] >> i) & 1u)) return f32x4{0.f, 0.f, 0.f, 0.f};
      return f32x4{bn_act<ACT>(x[0], al[0], sh[0]), bn_act<ACT>(x[1], al[1], sh[1]),
                   bn_act<ACT>(x[2], al[2], sh[2]), bn_act<ACT>(x[3], al[3], sh[3])};
    }
  }
  template <bool BN, int SET>
  __device__ __forceinline__ void coefs(const float* cl, f32x4& al, f32x4& sh) const {
    if constexpr (BN) {
      al = *reinterpret_cast<const f32x4*>(cl + kch[SET]);
      sh = *reinterpret_cast<const f32x4*>(cl + kBnMaxC + kch[SET]);
    }
  }
  // ACT < 0: no BatchNorm on load; else the activation of the BN operand (uniform branch in
  // the callers below, so each path is straight-line code)
  template <int LDB, int SET, int ACT>
  __device__ __forceinline__ void store_bf16_act(__bf16* lds, const float* cl) const {
    static_assert(RK, "CK operands use store_bf16_kr");
    if constexpr (EB == 2) {   // already bf16: one 16-byte write per slot
      static_assert(ACT < 0, "BatchNorm on load needs an fp32 operand");
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        int r, k;
        coords(i, r, k);
        *reinterpret_cast<f32x4*>(lds + r * LDB + k) = SET ? v2[i] : v[i];
      }
      return;
    }
    f32x4 al, sh;
    coefs<(ACT >= 0), SET>(cl, al, sh);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int r, k;
      coords(i, r, k);
      const f32x4 x = staged<ACT, SET>(i, al, sh);
      const bf16x4 b = {(__bf16)x[0], (__bf16)x[1], (__bf16)x[2], (__bf16)x[3]};
      *reinterpret_cast<bf16x4*>(lds + r * LDB + k) = b;
    }
  }
  template <int LDB, int SET = 0, bool BN = false>
  __device__ __forceinline__ void store_bf16(__bf16* lds, int act = 0, const float* cl = nullptr) const {
    if constexpr (!BN) store_bf16_act<LDB, SET, -1>(lds, cl);
    else if (act == 1) store_bf16_act<LDB, SET, 1>(lds, cl);
    else if (act == 2) store_bf16_act<LDB, SET, 2>(lds, cl);
    else store_bf16_act<LDB, SET, 0>(lds, cl);
  }
  // bf16 image [k][ROWS + 32] (rows contiguous) of a CK operand: each slot's 4 rows as one
  // 8-byte write (a wave writes whole k rows: conflict-free); read back transposed with
  // ds_read_b64_tr_b16 (frag_tr below).  The 32-element pad makes the k-row stride 16 dwords
  // mod 64, so the 4 k rows one 32-lane half reads sit on disjoint banks.
  static constexpr int LDK = ROWS + 32;
  template <int SET, int ACT>
  __device__ __forceinline__ void store_bf16_kr_act(__bf16* lds, const float* cl) const {
    if constexpr (EB == 2) {   // 8 rows of one k, already bf16: one 16-byte write per slot
      static_assert(ACT < 0, "BatchNorm on load needs an fp32 operand");
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        int r, k;
        coords(i, r, k);
        *reinterpret_cast<f32x4*>(lds + k * LDK + r) = SET ? v2[i] : v[i];
      }
      return;
    }
    f32x4 al, sh;
    coefs<(ACT >= 0), SET>(cl, al, sh);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int r, k;
      coords(i, r, k);
      const f32x4 x = staged<ACT, SET>(i, al, sh);
      const bf16x4 b = {(__bf16)x[0], (__bf16)x[1], (__bf16)x[2], (__bf16)x[3]};
      *reinterpret_cast<bf16x4*>(lds + k * LDK + r) = b;
    }
  }
  template <int SET = 0, bool BN = false>
  __device__ __forceinline__ void store_bf16_kr(__bf16* lds, int act = 0, const float* cl = nullptr) const {
    if constexpr (!BN) store_bf16_kr_act<SET, -1>(lds, cl);
    else if (act == 1) store_bf16_kr_act<SET, 1>(lds, cl);
    else if (act == 2) store_bf16_kr_act<SET, 2>(lds, cl);
    else store_bf16_kr_act<SET, 0>(lds, cl);
  }
  // fp32 as three bf16 planes (X6 mode of gemm_bf16_kernel): hi = RNE(x), mid = RNE(x - hi),
  // lo = RNE(x - hi - mid).  Both differences are exact in fp32, and x - hi - mid has at most
  // 8 significant bits, so hi + mid + lo == x exactly (normal numbers).  Images `pe` elements
  // apart; RK: [row][LDB], CK: [k][LDK].
  template <int LDB, int SET = 0>
  __device__ __forceinline__ void store_x3(__bf16* lds, int pe) const {
    static_assert(EB == 4, "the split needs fp32 operands");
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int r, k;
      coords(i, r, k);
      const f32x4 x = SET ? v2[i] : v[i];
      bf16x4 hi, mid, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (__bf16)x[e];
        const float r1 = x[e] - (float)hi[e];
        mid[e] = (__bf16)r1;
        lo[e] = (__bf16)(r1 - (float)mid[e]);
      }
      __bf16* d = lds + (RK ? r * LDB + k : k * (ROWS + 32) + r);
      *reinterpret_cast<bf16x4*>(d) = hi;
      *reinterpret_cast<bf16x4*>(d + pe) = mid;
      *reinterpret_cast<bf16x4*>(d + 2 * pe) = lo;
    }
  }
  // fragment values of MFMAs p = 4g .. 4g+3 (k = h*BK/2 + p) for tile row `row`
  __device__ __forceinline__ f32x4 frag4(const float* lds, int row, int h, int g) const {
    if (RK) return *reinterpret_cast<const f32x4*>(lds + row * LD + h * (BK / 2) + 4 * g);
    f32x4 v;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) v[jj] = lds[(h * (BK / 2) + 4 * g + jj) * LD + row];
    return v;
  }
  // fragment values of MFMA p (0..BK/2-1) for tile row `row`, lane half h: k = h*BK/2 + p
  __device__ __forceinline__ void frag(const float* lds, int row, int h, float (&out)[BK / 2]) const {
    if (RK) {
#pragma unroll
      for (int c = 0; c < BK / 8; ++c) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(lds + row * LD + h * (BK / 2) + 4 * c);
        out[4 * c] = x[0]; out[4 * c + 1] = x[1]; out[4 * c + 2] = x[2]; out[4 * c + 3] = x[3];
      }
    } else {
#pragma unroll
      for (int p = 0; p < BK / 2; ++p) out[p] = lds[(h * (BK / 2) + p) * LD + row];
    }
  }
};

// Block tile BM x BN, k-stage BK, waves of WM x WN (each (WM/32) x (WN/32) MFMA 32x32x2).
// DEEP: two k-stages of global loads in flight (register sets v / v2 alternate), so a
// stage's load latency hides behind two stages of MFMAs instead of one.
template <int BM, int BN, int BK, int WM, int WN, bool A_RK, bool B_RK, bool PIPE = false, bool DEEP = false>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void gemm_kernel(
    int M, int N, int K, Opnd A, Opnd B, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias1, const float* __restrict__ bias2, int accumulate,
    int k_per_split, float* __restrict__ slab, Batch bat) {
  constexpr int NWN = BN / WN;
  constexpr int NT = 64 * (BM / WM) * NWN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  using TA = OpTile<A_RK, BM, BK, NT>;
  using TBt = OpTile<B_RK, BN, BK, NT>;
  __shared__ __attribute__((aligned(16))) float smem[2][TA::FLOATS + TBt::FLOATS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / NWN, wc = wave % NWN;
  // XCD-aware tile order (speed only): blocks b, b+8, ... share an XCD under round-robin
  // dispatch; give each such group a contiguous run of tiles (x fastest) so tiles that
  // share A rows sit on one L2.  Bijective for any grid size.
  const int nx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int L = blockIdx.x + nx * blockIdx.y;
  const int xcd = L % 8, slot = L / 8, qq = nwg / 8, rr = nwg % 8;
  const int logical = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  const int64_t m0 = (int64_t)(logical / nx) * BM, n0 = (int64_t)(logical % nx) * BN;
  if (bat.c) {
    A.p += (int64_t)blockIdx.z * bat.a;
    B.p += (int64_t)blockIdx.z * bat.b;
    C += (int64_t)blockIdx.z * bat.c;
  }
  const int64_t kbeg = bat.c ? 0 : (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = bat.c ? (int64_t)K : min((int64_t)K, kbeg + k_per_split);
  const int nk = (int)((kend - kbeg + BK - 1) / BK);

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TA sa;
  TBt sb;
  sa.init(A, m0, kbeg, M);
  sb.init(B, n0, kbeg, N);
  if (nk > 0) {
    sa.load(A, kend);
    sb.load(B, kend);
    sa.store(smem[0]);
    sb.store(smem[0] + TA::FLOATS);
    if (DEEP && nk > 1) {
      sa.load_to(A, kend, sa.v2);
      sb.load_to(B, kend, sb.v2);
    }
  }
  __syncthreads();

  const int h = lane >> 5, li = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (DEEP) {
      // stage kt + 2 into the register set stage kt used (already in LDS)
      if (kt + 2 < nk) {
        if (kt & 1) { sa.load_to(A, kend, sa.v2); sb.load_to(B, kend, sb.v2); }
        else        { sa.load_to(A, kend, sa.v);  sb.load_to(B, kend, sb.v); }
      }
    } else if (kt + 1 < nk) {
      sa.load(A, kend);
      sb.load(B, kend);
    }
    const float* As = smem[buf];
    const float* Bs = smem[buf] + TA::FLOATS;
    if (PIPE) {
      // fragments in groups of 4 k-steps, the next group's LDS reads issued ahead of the
      // current group's MFMAs (one wave per SIMD at 1 block/CU: the reads must hide
      // behind this wave's own matrix work)
      constexpr int G = BK / 8;
      f32x4 fa[2][TI], fb[2][TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) fa[0][i] = sa.frag4(As, wr * WM + i * 32 + li, h, 0);
#pragma unroll
      for (int j = 0; j < TJ; ++j) fb[0][j] = sb.frag4(Bs, wc * WN + j * 32 + li, h, 0);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (g + 1 < G) {
#pragma unroll
          for (int i = 0; i < TI; ++i) fa[(g + 1) & 1][i] = sa.frag4(As, wr * WM + i * 32 + li, h, g + 1);
#pragma unroll
          for (int j = 0; j < TJ; ++j) fb[(g + 1) & 1][j] = sb.frag4(Bs, wc * WN + j * 32 + li, h, g + 1);
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[g & 1][i][jj], fb[g & 1][j][jj], acc[i][j], 0, 0, 0);
      }
    } else {
      float af[TI][BK / 2], bf[TJ][BK / 2];
#pragma unroll
      for (int i = 0; i < TI; ++i) sa.frag(As, wr * WM + i * 32 + li, h, af[i]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) sb.frag(Bs, wc * WN + j * 32 + li, h, bf[j]);
#pragma unroll
      for (int p = 0; p < BK / 2; ++p)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][p], bf[j][p], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      if (DEEP && ((kt + 1) & 1)) {
        sa.template store<1>(smem[buf ^ 1]);
        sb.template store<1>(smem[buf ^ 1] + TA::FLOATS);
      } else {
        sa.store(smem[buf ^ 1]);
        sb.store(smem[buf ^ 1] + TA::FLOATS);
      }
    }
    __syncthreads();
  }

  // epilogue: C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* out = slab ? slab + (int64_t)blockIdx.z * M * N : C;
  const int64_t ld = slab ? N : ldc;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int64_t n = n0 + wc * WN + j * 32 + li;
    if (n >= N) continue;
    float bsum = 0.f;
    if (!slab) {
      if (bias1) bsum += bias1[n];
      if (bias2) bsum += bias2[n];
    }
    if (!slab && accumulate) {   // every prior value in flight before the first store
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < M) acc[i][j][r] = (acc[i][j][r] + bsum) + out[m * ld + n];
        }
      bsum = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) out[m * ld + n] = acc[i][j][r] + bsum;
      }
    }
  }
}

// bf16-MFMA GEMM ("bf16 compute, fp32 master": BASELINE config 3).  Same operand modes,
// masking, split-K and epilogue as gemm_kernel; the fp32 operands are rounded to bf16
// (RNE, v_cvt_pk_bf16_f32) when a stage is written to LDS as [row][BK + 8] bf16, and
// v_mfma_f32_32x32x16_bf16 accumulates in fp32 (lane (r = l & 31, h = l >> 5) reads the 8
// contiguous k = 16 ks + 8h .. +8 of its row with one ds_read_b128, the operand map of
// the instruction, for A and B alike).
// BNOP (fused Conv-BN stacks): 1 = A, 2 = B is a conv operand with BatchNorm + activation
// applied on load (Opnd::coef / act).
// SRC: bit 0 = A, bit 1 = B is held in memory as bf16 (ld in bf16 elements; conv channel
// counts multiples of 8).
// X6 (precision "fp32", the fp32 GEMMs on bf16 MFMA): each fp32 operand is staged as its three
// bf16 planes (OpTile::store_x3) and the product a*b = (ah + am + al)(bh + bm + bl) is taken
// as ah*bh into one accumulator and ah*bm + am*bh + ah*bl + al*bh + am*bm into a second; the
// three dropped terms (am*bl, al*bm, al*bl) are below 2^-24 |a b|, and bf16 x bf16 products
// are exact in fp32.  The small terms sum at their own magnitude, so adding the two
// accumulators once at the end leaves the rounding of a plain fp32 accumulation
// (tests/test_gemm_x6_gpu.py: error against fp64 within that of gemm_kernel).  Six
// 32x32x16 bf16 MFMAs do the work of 8 fp32 32x32x2 MFMAs at 16x their rate.
template <int BM, int BN, int BK, int WM, int WN, bool A_RK, bool B_RK, bool DEEP = false, int BNOP = 0, int SRC = 0,
          bool X6 = false>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void gemm_bf16_kernel(
    int M, int N, int K, Opnd A, Opnd B, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias1, const float* __restrict__ bias2, int accumulate,
    int k_per_split, float* __restrict__ slab, Batch bat) {
  constexpr bool ABN = BNOP == 1, BBN = BNOP == 2;
  __shared__ __attribute__((aligned(16))) float cl[BNOP ? 2 * kBnMaxC : 4];
  if constexpr (BNOP != 0) {   // the BN operand's (alpha | shift), staged once
    const Opnd& o = ABN ? A : B;
    for (int c = threadIdx.x; c < o.conv_C; c += blockDim.x) {
      cl[c] = o.coef[c];
      cl[kBnMaxC + c] = o.coef[o.conv_C + c];
    }
    __syncthreads();
  }
  constexpr int NWN = BN / WN;
  constexpr int NT = 64 * (BM / WM) * NWN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int LDB = BK + 8;
  using TA = OpTile<A_RK, BM, BK, NT, (SRC & 1) ? 2 : 4>;
  using TBt = OpTile<B_RK, BN, BK, NT, (SRC & 2) ? 2 : 4>;
  // RK operands: [row][BK + 8] images read with ds_read_b128; CK operands: [k][rows + 32]
  // images read with ds_read_b64_tr_b16
  constexpr int A_EL1 = A_RK ? BM * LDB : BK * TA::LDK;
  constexpr int B_EL1 = B_RK ? BN * LDB : BK * TBt::LDK;
  constexpr int NPL = X6 ? 3 : 1;                  // planes per operand image
  constexpr int A_EL = NPL * A_EL1, B_EL = NPL * B_EL1;
  static_assert(!X6 || (BNOP == 0 && SRC == 0), "X6: fp32 operands");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][A_EL + B_EL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / NWN, wc = wave % NWN;
  const int nx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int L = blockIdx.x + nx * blockIdx.y;
  const int xcd = L % 8, slot = L / 8, qq = nwg / 8, rr = nwg % 8;
  const int logical = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  const int64_t m0 = (int64_t)(logical / nx) * BM, n0 = (int64_t)(logical % nx) * BN;
  if (bat.c) {
    A.p += (int64_t)blockIdx.z * bat.a;
    B.p += (int64_t)blockIdx.z * bat.b;
    C += (int64_t)blockIdx.z * bat.c;
  }
  const int64_t kbeg = bat.c ? 0 : (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = bat.c ? (int64_t)K : min((int64_t)K, kbeg + k_per_split);
  const int nk = (int)((kend - kbeg + BK - 1) / BK);

  f32x16 acc[TI][TJ];
  f32x16 acs[X6 ? TI : 1][X6 ? TJ : 1];            // X6: the small terms
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if constexpr (X6)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acs[i][j][r] = 0.f;

  TA sa;
  TBt sb;
  sa.init(A, m0, kbeg, M);
  sb.init(B, n0, kbeg, N);
  auto stage = [&](__bf16* img) {
    if constexpr (X6) {
      sa.template store_x3<LDB>(img, A_EL1);
      sb.template store_x3<LDB>(img + A_EL, B_EL1);
      return;
    }
    if constexpr (A_RK) sa.template store_bf16<LDB, 0, ABN>(img, A.act, cl);
    else sa.template store_bf16_kr<0, ABN>(img, A.act, cl);
    if constexpr (B_RK) sb.template store_bf16<LDB, 0, BBN>(img + A_EL, B.act, cl);
    else sb.template store_bf16_kr<0, BBN>(img + A_EL, B.act, cl);
  };
  auto stage2 = [&](__bf16* img) {   // from the second staging set
    if constexpr (X6) {
      sa.template store_x3<LDB, 1>(img, A_EL1);
      sb.template store_x3<LDB, 1>(img + A_EL, B_EL1);
      return;
    }
    if constexpr (A_RK) sa.template store_bf16<LDB, 1, ABN>(img, A.act, cl);
    else sa.template store_bf16_kr<1, ABN>(img, A.act, cl);
    if constexpr (B_RK) sb.template store_bf16<LDB, 1, BBN>(img + A_EL, B.act, cl);
    else sb.template store_bf16_kr<1, BBN>(img + A_EL, B.act, cl);
  };
  auto load1 = [&]() { sa.template load_s<ABN, 0>(A, kend); sb.template load_s<BBN, 0>(B, kend); };
  auto load2 = [&]() { sa.template load_s<ABN, 1>(A, kend); sb.template load_s<BBN, 1>(B, kend); };
  if (nk > 0) {
    load1();
    stage(smem[0]);
  }
  if (DEEP) {                        // stages 1 and 2 in flight before the first barrier
    if (nk > 1) load1();
    if (nk > 2) load2();
  }
  __syncthreads();

  const int h = lane >> 5, li = lane & 31;
  // transposed-read lane map (T10): lane 16g + 4q + p supplies k row 8h + q (+4) and rows
  // 16 (g & 1) + 4p .. +3 of the 32-row block; it receives row (lane & 31)'s 8 k values
  const int tr_off = ((lane >> 2) & 3) + 8 * h;               // k row within the 16-k step
  const int tr_row = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  auto frag_tr = [&](const __bf16* img, int LDK, int row0, int ks) {
    const __bf16* p0 = img + (ks * 16 + tr_off) * LDK + row0 + tr_row;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(p0 + 4 * LDK));
    const s16x4 w[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, w);
  };
  auto compute = [&](const __bf16* As) {
    const __bf16* Bs = As + A_EL;
    if constexpr (X6) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 fa[3][TI], fb[3][TJ];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
#pragma unroll
          for (int i = 0; i < TI; ++i)
            fa[q][i] = A_RK ? *reinterpret_cast<const bf16x8*>(As + q * A_EL1 + (wr * WM + i * 32 + li) * LDB +
                                                                ks * 16 + 8 * h)
                            : frag_tr(As + q * A_EL1, TA::LDK, wr * WM + i * 32, ks);
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            fb[q][j] = B_RK ? *reinterpret_cast<const bf16x8*>(Bs + q * B_EL1 + (wc * WN + j * 32 + li) * LDB +
                                                                ks * 16 + 8 * h)
                            : frag_tr(Bs + q * B_EL1, TBt::LDK, wc * WN + j * 32, ks);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
            acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acs[i][j], 0, 0, 0);
            acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acs[i][j], 0, 0, 0);
            acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acs[i][j], 0, 0, 0);
            acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acs[i][j], 0, 0, 0);
            acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acs[i][j], 0, 0, 0);
          }
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[TI], fb[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[i] = A_RK ? *reinterpret_cast<const bf16x8*>(As + (wr * WM + i * 32 + li) * LDB + ks * 16 + 8 * h)
                     : frag_tr(As, TA::LDK, wr * WM + i * 32, ks);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        fb[j] = B_RK ? *reinterpret_cast<const bf16x8*>(Bs + (wc * WN + j * 32 + li) * LDB + ks * 16 + 8 * h)
                     : frag_tr(Bs, TBt::LDK, wc * WN + j * 32, ks);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };
#ifndef AVC_X6_SCHED
#define AVC_X6_SCHED 6
#endif
  if constexpr (X6 && DEEP) {
    // as the DEEP loop below, with the refills unconditional (past-K loads read zeros; a
    // stage written past the last k is never computed), so that each half is one straight
    // block: the next stage's split conversions and LDS writes are interleaved between the
    // MFMAs (AVC_X6_SCHED vector instructions per MFMA) instead of following them.  Isolated
    // (profiles/r06/gemm_x6_sched.txt): 6 per MFMA 374 vs 390 us for 0 on the LSTM dW
    // 4096x1024x8192, others within 2 %; the unconditional refills alone took the step from
    // 13.05 to 12.85-12.89 ms (ab_fp32_x6_v3.txt)
    constexpr int NMF = TI * TJ * 6 * (BK / 16);
    auto interleave = [&]() {
      if constexpr (AVC_X6_SCHED > 0) {
#pragma unroll
        for (int q = 0; q < NMF; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, AVC_X6_SCHED, 0);
        }
      }
    };
    for (int kt = 0; kt < nk; kt += 2) {
      compute(smem[0]);
      stage(smem[1]);
      load1();
      interleave();
      __syncthreads();
      if (kt + 1 < nk) {
        compute(smem[1]);
        stage2(smem[0]);
        load2();
        interleave();
        __syncthreads();
      }
    }
  } else if (DEEP) {
    // two register stages in flight: at the top of an iteration LDS buffer 0 holds stage kt,
    // set 1 (v) stage kt + 1 and set 2 (v2) stage kt + 2; each half computes one buffer and
    // refills the other from the set whose loads are oldest, then reloads that set
    for (int kt = 0; kt < nk; kt += 2) {
      compute(smem[0]);
      if (kt + 1 < nk) {
        stage(smem[1]);
        if (kt + 3 < nk) load1();
      }
      __syncthreads();
      if (kt + 1 < nk) {
        compute(smem[1]);
        if (kt + 2 < nk) {
          stage2(smem[0]);
          if (kt + 4 < nk) load2();
        }
        __syncthreads();
      }
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load1();
      compute(smem[buf]);
      if (kt + 1 < nk) stage(smem[buf ^ 1]);
      __syncthreads();
    }
  }

  if constexpr (X6)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += acs[i][j];
  float* out = slab ? slab + (int64_t)blockIdx.z * M * N : C;
  const int64_t ld = slab ? N : ldc;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int64_t n = n0 + wc * WN + j * 32 + li;
    if (n >= N) continue;
    float bsum = 0.f;
    if (!slab) {
      if (bias1) bsum += bias1[n];
      if (bias2) bsum += bias2[n];
    }
    if (!slab && accumulate) {   // every prior value in flight before the first store
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < M) acc[i][j][r] = (acc[i][j][r] + bsum) + out[m * ld + n];
        }
      bsum = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) out[m * ld + n] = acc[i][j][r] + bsum;
      }
    }
  }
}

// 2-D: blockIdx.x * 256 + thread = column, blockIdx.y strides rows (no 64-bit divide);
// slabs summed in split order (deterministic)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(int64_t M, int64_t N, int splits,
                                                           const float* __restrict__ slab, float* __restrict__ C,
                                                           int64_t ldc, const float* __restrict__ bias1,
                                                           const float* __restrict__ bias2, int accumulate) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int64_t total = M * N;
  float bsum = 0.f;
  if (bias1) bsum += bias1[n];
  if (bias2) bsum += bias2[n];
  for (int64_t m = blockIdx.y; m < M; m += gridDim.y) {
    const int64_t i = m * N + n;
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += slab[s * total + i];
    v += bsum;
    float* dst = C + m * ldc + n;
    if (accumulate) v += *dst;
    *dst = v;
  }
}

// The fused Conv-BN stacks' split-K reduce (bf16 conv GEMMs always end in one): C = the
// split sum (+ bias), and per row block blockIdx.y (a contiguous range of M / gridDim.y
// rows) and column n the fp64 partials part[y][n][2] of
//   MODE 1: (sum v, sum v^2) — the BatchNorm statistics of the conv output v (bn.hip
//           stats_finalize_raw_kernel sums them);
//   MODE 2: (sum g, sum g (yp - mean)), g = act'(pre) v, pre = alpha yp + shift — the
//           BatchNorm backward sums of the layer whose pre-BN output yp (M x N) this input
//           gradient v belongs to (bn.hip bwd_partial_kernel's sums; relu' from pre > 0,
//           tanh' = 1 - avc_tanh_fast(pre)^2 recomputed as the forward computed it).
// Block = 64 columns x 4 waves; wave w takes rows r0 + w, r0 + w + 4, ... of the block's
// range (the loads of 4 rows in flight per thread), the 4 waves' sums are added in wave
// order through LDS (deterministic).
template <int MODE, int ACTP>
__global__ __launch_bounds__(256) void splitk_stats_kernel(int64_t M, int64_t N, int splits,
                                                          const float* __restrict__ slab, float* __restrict__ C,
                                                          int64_t ldc, const float* __restrict__ bias,
                                                          const float* __restrict__ yp, const float* __restrict__ coefp,
                                                          double* __restrict__ part) {
  __shared__ double red[4][64][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + lane;
  const int64_t total = M * N;
  const int64_t r0 = M * blockIdx.y / gridDim.y, r1 = M * (blockIdx.y + 1) / gridDim.y;
  double s1 = 0.0, s2 = 0.0;
  if (n < N) {
    const float bsum = bias ? bias[n] : 0.f;
    float a = 0.f, sh = 0.f, mu = 0.f;
    if (MODE == 2) { a = coefp[n]; sh = coefp[N + n]; mu = coefp[2 * N + n]; }
#pragma unroll 4
    for (int64_t m = r0 + w; m < r1; m += 4) {
      const int64_t i = m * N + n;
      float v = 0.f;
      for (int s = 0; s < splits; ++s) v += slab[s * total + i];
      v += bsum;
      C[m * ldc + n] = v;
      if (MODE == 1) {
        s1 += (double)v;
        s2 += (double)v * (double)v;
      } else {
        const float y = yp[i];
        const float pre = fmaf(y, a, sh);
        float g = v;
        if (ACTP == 1) g = pre > 0.f ? v : 0.f;
        else if (ACTP == 2) { const float z = avc_tanh_fast(pre); g = v * (1.f - z * z); }
        s1 += (double)g;
        s2 += (double)g * (double)(y - mu);
      }
    }
  }
  red[w][lane][0] = s1;
  red[w][lane][1] = s2;
  __syncthreads();
  if (w == 0 && n < N) {
    const double a = ((red[0][lane][0] + red[1][lane][0]) + red[2][lane][0]) + red[3][lane][0];
    const double b = ((red[0][lane][1] + red[1][lane][1]) + red[2][lane][1]) + red[3][lane][1];
    part[((int64_t)blockIdx.y * N + n) * 2 + 0] = a;
    part[((int64_t)blockIdx.y * N + n) * 2 + 1] = b;
  }
}

bool aligned_ld(int64_t ld) { return (ld & 3) == 0; }

// Tile configurations (id -> BM, BN, BK; waves of 64x64 unless noted)
struct GemmShape { int id, bm, bn, bk; };
constexpr GemmShape kCfg[] = {
    {0, 128, 128, 16},   // 4 waves of 64x64
    {1, 128, 64, 16},    // 4 waves of 64x32: twice the blocks for small grids
    {2, 128, 128, 32},   // 4 waves of 64x64, half the barriers
    {3, 64, 64, 16},     // 4 waves of 32x32: small outputs
    {4, 128, 128, 32},   // cfg 2 with the fragment reads pipelined behind the MFMAs
    {5, 64, 64, 16},     // cfg 3 pipelined
    {6, 128, 64, 32},    // 4 waves of 64x32, BK 32, pipelined
    {7, 128, 128, 64},   // BK 64, pipelined (139 KB LDS, 1 block/CU)
    {8, 64, 64, 32},     // BK 32, pipelined
    {9, 128, 128, 32},   // 8 waves of 64x32, pipelined (sweep candidate)
    {10, 64, 64, 64},    // BK 64, pipelined (sweep candidate)
    {11, 128, 64, 32},   // 8 waves of 32x32, pipelined (sweep candidate)
    {12, 128, 128, 32},  // cfg 2 with two k-stages of loads in flight
    {13, 64, 64, 32},    // cfg 8 with two k-stages of loads in flight
    {14, 128, 128, 32},  // cfg 9 with two k-stages of loads in flight
};

int g_force_cfg = -1;  // tools/gemm_bench.hip overrides this
// LDS (bytes per CU) that GEMM launches leave free for a latency-bound kernel on another
// stream (autovc_gemm_set_lds_reserve): each workgroup is padded with unused dynamic LDS
// so that the largest count that still fits in 160 KiB - reserve is also the most that fit.
unsigned g_lds_reserve = 0;
Batch g_batch = {0, 0, 0};   // set by gemm_impl for every launch
constexpr unsigned kLdsPerCU = 160 * 1024;

unsigned dyn_lds_for(unsigned static_bytes) {
  if (g_lds_reserve == 0 || static_bytes == 0 || static_bytes + g_lds_reserve > kLdsPerCU) return 0;
  // n workgroups of kLdsPerCU / (n + 1) + 256 bytes leave kLdsPerCU / (n + 1) - 256 free:
  // n <= kLdsPerCU / reserve - 1, and n of the real size must fit beside the reserve
  unsigned n = std::min((kLdsPerCU - g_lds_reserve) / static_bytes, kLdsPerCU / (g_lds_reserve + 256) - 1);
  if (n > 8) n = 8;
  if (n == 0) return 0;
  const unsigned per = kLdsPerCU / (n + 1) + 256;   // n + 1 no longer fit
  return per > static_bytes ? per - static_bytes : 0;
}

template <int BM, int BN, int BK, bool AR, bool BR>
constexpr unsigned f32_lds_bytes() {
  return 2u * 4u * ((AR ? BM * (BK + 4) : BK * (BM + 4)) + (BR ? BN * (BK + 4) : BK * (BN + 4)));
}

GemmShape pick_config(int M, int N, int K, int splits) {
  if (g_force_cfg >= 0) return kCfg[g_force_cfg];
  // tools/gemm_bench.hip sweep (round 1, buffer-load staging, random operands):
  // 128x128/BK32 once the 128-tile grid fills the chip >= 2x over (115-124 TF at
  // 8192x1024..4096); narrower unsplit outputs on 64x64/BK32 with pipelined fragment
  // reads (conv fwd/dX 105-109 TF); split-K weight gradients on 64x64/BK16 (92-99 TF).
  // (8-wave tiles, cfg 9/11, won 5-7 % in the isolated sweep but nothing inside the step:
  // 21.62 vs 21.52 ms, same box, alternating)
  constexpr int NCFG = (int)(sizeof(kCfg) / sizeof(kCfg[0]));
  // round 3 (whole step, alternating): cfg 9 for the big grids too, 14.80-14.83 vs
  // 14.86-14.89 ms/step with identical losses (profiles/r03/ab_gemm_bigk.txt)
  static_assert(NCFG > 9, "tile configurations");
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128) * splits;
  if (t128 >= 512) return kCfg[9];
  // deep-K outputs that fill the chip once with 128-tiles (the LSTM weight gradients,
  // 4096 x 1024 over K = B*T = 8192, on the gradient side stream): 128x128/BK32 measured
  // 17.86 vs 17.98 ms/step against 64x64 (round 2, tools/ab_gemm_bigk.sh); its 8-wave form
  // (cfg 9: 64x32 per wave, pipelined fragment reads) 14.82-14.89 vs 14.95-14.98 ms/step in
  // round 3, where these GEMMs run at the end of the replayed step with the chip to themselves
  // (profiles/r03/ab_gemm_bigk.txt)
  if (t128 >= 256 && K >= 4096) return kCfg[9];
  // (cfg 13 — BK 32, two k-stages in flight — for these measured slower in the step, with the
  // BLSTM weight gradients split 32 / 16 / 8 ways: profiles/r05/ab_blstm_side2.txt)
  if (splits > 1) return kCfg[3];
  return kCfg[8];
}

template <int BM, int BN, int BK, int WM, int WN, bool PIPE = false, bool DEEP = false>
void launch_layouts(int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob,
                    float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps, float* slab) {
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
#define AVC_L(AR, BR) hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, AR, BR, PIPE, DEEP>), grid, dim3(NT), \
                                         dyn_lds_for(f32_lds_bytes<BM, BN, BK, AR, BR>()), st, M, N, K, \
                                         oa, ob, C, ldc, b1, b2, acc, kps, slab, g_batch)
  if (!a_trans && !b_trans) AVC_L(true, true);
  else if (!a_trans && b_trans) AVC_L(true, false);
  else if (a_trans && !b_trans) AVC_L(false, true);
  else AVC_L(false, false);
#undef AVC_L
}

void launch_gemm(int id, int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob,
                 float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps, float* slab) {
  switch (id) {
    case 0: launch_layouts<128, 128, 16, 64, 64>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 1: launch_layouts<128, 64, 16, 64, 32>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 2: launch_layouts<128, 128, 32, 64, 64>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 4: launch_layouts<128, 128, 32, 64, 64, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 5: launch_layouts<64, 64, 16, 32, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 6: launch_layouts<128, 64, 32, 64, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 7: launch_layouts<128, 128, 64, 64, 64, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 8: launch_layouts<64, 64, 32, 32, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 9: launch_layouts<128, 128, 32, 64, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 10: launch_layouts<64, 64, 64, 32, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 11: launch_layouts<128, 64, 32, 32, 32, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 12: launch_layouts<128, 128, 32, 64, 64, false, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 13: launch_layouts<64, 64, 32, 32, 32, true, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 14: launch_layouts<128, 128, 32, 64, 32, true, true>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    default: launch_layouts<64, 64, 16, 32, 32>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
  }
}

// bf16 tiles: 128x128 (4 waves of 64x64) once that grid fills the chip, else 64x64; BK 64:
// with the MFMA work per stage 16x smaller than fp32's, the kernel waits on its operand
// loads, so a stage keeps twice the bytes in flight (BK 32: conv fwd 67 us, LSTM dW 438 us)
constexpr GemmShape kCfgBf16[] = {
    {0, 128, 128, 64},   // 4 waves of 64x64
    {1, 64, 64, 64},     // 4 waves of 32x32
    {2, 256, 128, 64},   // 8 waves of 64x64 (one workgroup per CU)
    {3, 256, 256, 64},   // 8 waves of 128x64 (one workgroup per CU)
    {4, 256, 256, 32},   // 8 waves of 128x64, BK 32
};
int g_force_cfg_bf16 = -1;   // tools/gemm_bf16_bench.hip overrides these
int g_force_splits_bf16 = 0;

GemmShape pick_config_bf16(int M, int N, int splits) {
  if (g_force_cfg_bf16 >= 0) return kCfgBf16[g_force_cfg_bf16];
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128) * splits;
  return t128 >= 256 ? kCfgBf16[0] : kCfgBf16[1];
}

// Large bf16 GEMMs: one workgroup per CU on 256-row tiles, split-K chosen here so that about
// one wave of 256 workgroups runs (tools/gemm_bf16_bench.hip, round 2, bf16-exact operands
// = the fp32 result): 256x256/BK32 when the tile grid times a split of <= 4 fills the chip with
// >= 1024 k per split (LSTM dW 4096x1024x8192: 4 splits, 128 us vs 221 for 128x128 unsplit;
// LSTM dX 8192x1024x4096: 2 splits, 127 vs 132), else 256x128 with <= 4 splits of >= 512 k
// (conv fwd/dX 8192x512x2560: 2 splits, 57 vs 68 us; conv dW 512x2560x8192: 4 splits, 79 vs
// 87 for 128x128 at 4), and 256x128 unsplit for grids of >= 256 such tiles (LSTM input
// projections 8192x4096x1024: 151 us).  Smaller outputs keep the caller's split and the
// 128x128 / 64x64 tiles.
struct PlanBf16 { int cfg, splits; };
PlanBf16 plan_bf16(int M, int N, int K, int requested) {
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  const int64_t t2 = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
  if (t2 >= 256) return {2, 1};
  for (int s = 1; s <= 4; ++s)
    if (t256 * s >= 224 && t256 * s <= 288 && K / s >= 1024) return {4, s};
  if (t2 >= 16) {
    int s = (int)std::max<int64_t>(1, std::min<int64_t>(4, (256 + t2 / 2) / t2));
    while (s > 1 && K / s < 512) --s;
    // shallow K (<= 1024) cannot split its way to a full chip: one 256-row tile per CU on
    // 32-128 CUs left the encoder BLSTM projections (8192 x 128 x 512) at 25 us; the caller's
    // split on 128 / 64 tiles fills the chip (step 8.415-8.419 vs 8.425-8.483 ms,
    // profiles/r05/ab_bf16_shallow.txt)
    if (!(K <= 1024 && t2 * s < 256)) return {2, s};
  }
  return {-1, requested};
}

template <int BM, int BN, int BK, bool AR, bool BR>
constexpr unsigned bf16_lds_bytes() {
  return 2u * 2u * ((AR ? BM * (BK + 8) : BK * (BM + 32)) + (BR ? BN * (BK + 8) : BK * (BN + 32)));
}

// the fused Conv-BN stacks' bf16 GEMMs (slabs only: the reduce writes C and the statistics):
// forward (A = im2col of the previous layer's output, RK; B = Wf, RK), input gradient (A =
// im2col(dy), RK; B = Wd, CK), weight gradient (A = dy, CK; B = im2col(x), CK).  BNOP 1 / 2:
// BatchNorm + activation applied on load to A / B (fp32 operand); SRC: bf16-source operands.
template <int BM, int BN, int BK, int WM, int WN, bool AR, bool BR, int BNOP, int SRC>
void launch_bn_bf16(dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob, int kps, float* slab) {
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  constexpr bool DEEP = BM == 256 && !(BN == 256 && !AR && !BR);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, BK, WM, WN, AR, BR, DEEP, BNOP, SRC>), grid, dim3(NT),
                     dyn_lds_for(bf16_lds_bytes<BM, BN, BK, AR, BR>()), st, M, N, K, oa, ob, (float*)nullptr,
                     (int64_t)N, (const float*)nullptr, (const float*)nullptr, 0, kps, slab, Batch{0, 0, 0});
}

template <bool AR, bool BR, int BNOP, int SRC>
void launch_gemm_bn_bf16(int id, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob, int kps,
                         float* slab) {
  switch (id) {
    case 0: launch_bn_bf16<128, 128, 64, 64, 64, AR, BR, BNOP, SRC>(grid, st, M, N, K, oa, ob, kps, slab); break;
    case 2: launch_bn_bf16<256, 128, 64, 64, 64, AR, BR, BNOP, SRC>(grid, st, M, N, K, oa, ob, kps, slab); break;
    case 3: launch_bn_bf16<256, 256, 64, 128, 64, AR, BR, BNOP, SRC>(grid, st, M, N, K, oa, ob, kps, slab); break;
    case 4: launch_bn_bf16<256, 256, 32, 128, 64, AR, BR, BNOP, SRC>(grid, st, M, N, K, oa, ob, kps, slab); break;
    default: launch_bn_bf16<64, 64, 64, 32, 32, AR, BR, BNOP, SRC>(grid, st, M, N, K, oa, ob, kps, slab); break;
  }
}

template <int BM, int BN, int BK, int WM, int WN, int SRC = 0>
void launch_layouts_bf16(int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob,
                         float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps, float* slab) {
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  // two stages in flight only on the 256-row tiles, and not for 256x256 with both operands
  // K-strided (spills): tools/gemm_bf16_bench.hip, profiles/r02/gemm_bf16_deep.txt
#define AVC_DEEP(AR, BR) (BM == 256 && !(BN == 256 && !(AR) && !(BR)))
#define AVC_L(AR, BR) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, BK, WM, WN, AR, BR, AVC_DEEP(AR, BR), 0, SRC>), grid, dim3(NT), \
                                         dyn_lds_for(bf16_lds_bytes<BM, BN, BK, AR, BR>()), st, M, N, \
                                         K, oa, ob, C, ldc, b1, b2, acc, kps, slab, g_batch)
  if (!a_trans && !b_trans) AVC_L(true, true);
  else if (!a_trans && b_trans) AVC_L(true, false);
  else if (a_trans && !b_trans) AVC_L(false, true);
  else AVC_L(false, false);
#undef AVC_L
#undef AVC_DEEP
}

template <int SRC>
void launch_gemm_bf16_src(int id, int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa,
                          Opnd ob, float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps,
                          float* slab) {
  switch (id) {
    case 0: launch_layouts_bf16<128, 128, 64, 64, 64, SRC>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 2: launch_layouts_bf16<256, 128, 64, 64, 64, SRC>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 3: launch_layouts_bf16<256, 256, 64, 128, 64, SRC>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 4: launch_layouts_bf16<256, 256, 32, 128, 64, SRC>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    default: launch_layouts_bf16<64, 64, 64, 32, 32, SRC>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
  }
}

// src: bit 0 = A, bit 1 = B held as bf16 (autovc_gemm_bf16src_f32); 0 = fp32 operands
void launch_gemm_bf16(int id, int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa,
                      Opnd ob, float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps,
                      float* slab, int src = 0) {
  switch (src) {
    case 1: launch_gemm_bf16_src<1>(id, a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 2: launch_gemm_bf16_src<2>(id, a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 3: launch_gemm_bf16_src<3>(id, a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    default: launch_gemm_bf16_src<0>(id, a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
  }
}

// precision "fp32" GEMMs on bf16 MFMA (gemm_bf16_kernel X6), the default: 256x128/BK16 (8 waves
// of 64x64, two stages in flight), 128x128/BK32 (4 waves of 64x64), 64x64/BK32 for small
// outputs.  Three bf16 planes per operand image: 86-110 KB of LDS for the 256-row tile.  Step
// A/B (alternating, one box): 13.05-13.06 vs 14.00-14.08 ms/step with the fp32 MFMA kernel
// (profiles/r06/ab_fp32_x6_v2.txt; isolated 1.3-1.6x on the step's shapes,
// gemm_x6_time_v2.txt).  AVC_FP32_X6=0 (or autovc_gemm_set_fp32_x6(0)) selects gemm_kernel.
int g_fp32_x6 = [] { const char* e = getenv("AVC_FP32_X6"); return e ? atoi(e) : 1; }();
constexpr GemmShape kCfgX6[] = {
    {0, 256, 128, 16},
    {1, 128, 128, 32},
    {2, 64, 64, 32},
};
// (cfg, splits) that put >= 192 workgroups on the chip with >= 1024 k per split, largest tile
// first; otherwise the 64x64 tile with the caller's split.  z: batch (no split) or 0.
PlanBf16 plan_x6(int M, int N, int K, int requested, int z) {
  const int64_t t0 = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
  const int64_t t1 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (z > 0) return {t0 * z >= 192 ? 0 : t1 * z >= 192 ? 1 : 2, 1};
  for (int s = 1; s <= 4; ++s)
    if (t0 * s >= 192 && (s == 1 || K / s >= 1024)) return {0, s};
  for (int s = 1; s <= 4; ++s)
    if (t1 * s >= 192 && (s == 1 || K / s >= 1024)) return {1, s};
  return {2, requested};
}
template <int BM, int BN, int BK, bool AR, bool BR>
constexpr unsigned x6_lds_bytes() {
  return 3u * bf16_lds_bytes<BM, BN, BK, AR, BR>();
}
template <int BM, int BN, int BK, int WM, int WN>
void launch_layouts_x6(int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob,
                       float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps, float* slab) {
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
#define AVC_L(AR, BR) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, BK, WM, WN, AR, BR, BM == 256, 0, 0, true>), grid, \
                                         dim3(NT), dyn_lds_for(x6_lds_bytes<BM, BN, BK, AR, BR>()), st, M, N, K, oa, \
                                         ob, C, ldc, b1, b2, acc, kps, slab, g_batch)
  if (!a_trans && !b_trans) AVC_L(true, true);
  else if (!a_trans && b_trans) AVC_L(true, false);
  else if (a_trans && !b_trans) AVC_L(false, true);
  else AVC_L(false, false);
#undef AVC_L
}
void launch_gemm_x6(int id, int a_trans, int b_trans, dim3 grid, hipStream_t st, int M, int N, int K, Opnd oa, Opnd ob,
                    float* C, int64_t ldc, const float* b1, const float* b2, int acc, int kps, float* slab) {
  switch (id) {
    case 0: launch_layouts_x6<256, 128, 16, 64, 64>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    case 1: launch_layouts_x6<128, 128, 32, 64, 64>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
    default: launch_layouts_x6<64, 64, 32, 32, 32>(a_trans, b_trans, grid, st, M, N, K, oa, ob, C, ldc, b1, b2, acc, kps, slab); break;
  }
}

}  // namespace

// precision "fp32" GEMMs through the bf16-plane kernel (1) or the fp32 MFMA kernel (0);
// returns the previous mode
extern "C" int autovc_gemm_set_fp32_x6(int on) {
  const int prev = g_fp32_x6;
  g_fp32_x6 = on ? 1 : 0;
  return prev;
}

// the split-K factor autovc_gemm_f32 will use for a request (size its workspace with it)
extern "C" int autovc_gemm_f32_splits(int M, int N, int K, int requested) {
  if (requested < 1) requested = 1;
  if (!g_fp32_x6 || M <= 0 || N <= 0 || K <= 0) return requested;
  return plan_x6(M, N, K, requested, 0).splits;
}

extern "C" int autovc_gemm_fp32_x6(void) { return g_fp32_x6; }

// split-K workspace: the partial slabs (tiles rounded up to 256 x 256), summed in split order
// by splitk_reduce_kernel
extern "C" int64_t autovc_gemm_workspace_floats(int M, int N, int splits) {
  return splits > 1 ? (int64_t)splits * ((M + 255) / 256 * 256) * ((N + 255) / 256 * 256) : 0;
}

static int gemm_impl(bool bf16, int batch, int64_t a_bs, int64_t b_bs, int64_t c_bs, int M, int N, int K,
                               const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                               const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                               float* C, int64_t ldc, const float* bias1, const float* bias2,
                               int accumulate, int splits, float* workspace, hipStream_t stream, int src = 0) {
  AVC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "autovc_gemm: negative dims");
  if (M == 0 || N == 0) return avc::kOk;
  AVC_CHECK_ARG(A && B && C, "autovc_gemm: null operand");
  AVC_CHECK_ARG(AVC_ALIGNED16(A) && AVC_ALIGNED16(B), "autovc_gemm: A/B must be 16-byte aligned");
  AVC_CHECK_ARG(aligned_ld(lda) && aligned_ld(ldb), "autovc_gemm: lda/ldb must be multiples of 4");
  AVC_CHECK_ARG(src >= 0 && src <= 3 && (src == 0 || (bf16 && batch == 1)),
                "autovc_gemm_bf16src_f32: bad src %d", src);
  AVC_CHECK_ARG(!(src & 1) || (!a_conv_T && lda % 8 == 0 && (a_trans ? M % 8 == 0 : K % 8 == 0)),
                "autovc_gemm_bf16src_f32: a bf16 A must be plain with lda and its contiguous dim multiples of 8");
  AVC_CHECK_ARG(!(src & 2) || (!b_conv_T && ldb % 8 == 0 && (b_trans ? N % 8 == 0 : K % 8 == 0)),
                "autovc_gemm_bf16src_f32: a bf16 B must be plain with ldb and its contiguous dim multiples of 8");
  // the contiguous extent of each operand must be a multiple of 4 (float4 staging)
  AVC_CHECK_ARG(a_trans ? (M % 4 == 0) : (K % 4 == 0), "autovc_gemm: A contiguous dim %% 4 != 0");
  AVC_CHECK_ARG(b_trans ? (N % 4 == 0) : (K % 4 == 0), "autovc_gemm: B contiguous dim %% 4 != 0");
  AVC_CHECK_ARG(!a_conv_T || (a_conv_C % 4 == 0 && a_conv_C > 0),
                "autovc_gemm: A conv channels must be a positive multiple of 4");
  AVC_CHECK_ARG(!b_conv_T || (b_conv_C % 4 == 0 && b_conv_C > 0),
                "autovc_gemm: B conv channels must be a positive multiple of 4");
  // buffer-load byte offsets are 32-bit (descriptor range 2 GiB)
  const int64_t a_ext = a_trans ? (int64_t)K * lda : (int64_t)M * lda;
  const int64_t b_ext = b_trans ? (int64_t)K * ldb : (int64_t)N * ldb;
  AVC_CHECK_ARG(4 * (a_ext + 2 * lda) < (int64_t)kOOB && 4 * (b_ext + 2 * ldb) < (int64_t)kOOB,
                "autovc_gemm: operand extents must stay below 2 GiB");
  if (splits < 1) splits = 1;
  if (bf16 && g_force_splits_bf16 > 0 && batch == 1) splits = g_force_splits_bf16;
  AVC_CHECK_ARG(batch >= 1 && (batch == 1 || splits == 1), "autovc_gemm: batched calls cannot split K");
  if (bf16 && batch == 1 && g_force_cfg_bf16 < 0) {
    const PlanBf16 pl = plan_bf16(M, N, K, splits);
    if (pl.cfg >= 0) {
      AVC_CHECK_ARG(pl.splits <= splits || workspace,
                    "autovc_gemm_bf16_f32: split-K plan needs the workspace of autovc_gemm_bf16_splits");
      splits = pl.splits;
      // the weight gradients (both operands K-strided) at most 3 splits: they run on the gradient
      // side stream beside the recurrences, where half the chip for twice as long costs the
      // step less than 4-way slabs and their reduce (training step 8.53-8.55 vs 8.99-9.05 ms;
      // 3 splits 8.67-8.68, 1 split 8.75-8.79; profiles/r05/ab_bf16_dw_splits.txt)
      // (round 6, with the XCD-local lstm1 backward and the bf16 routing: 3 splits 7.56-7.65 vs
      // 7.61-7.66 ms/step for 2 over six alternating pairs, uncapped 7.69;
      // profiles/r06/ab_bf16_dw_splits_r06.txt)
      if (a_trans && b_trans) splits = std::min(splits, 3);
    }
  }
  GemmShape cfg = bf16 ? pick_config_bf16(M, N, batch > 1 ? batch : splits) : pick_config(M, N, K, splits);
  if (bf16 && batch == 1 && g_force_cfg_bf16 < 0) {
    const PlanBf16 pl = plan_bf16(M, N, K, splits);
    if (pl.cfg >= 0) cfg = kCfgBf16[pl.cfg];
  }
  const bool x6 = !bf16 && g_fp32_x6 && g_force_cfg < 0;
  if (x6) {
    // the planned split, never above the caller's (its workspace): callers size it with
    // autovc_gemm_f32_splits
    const PlanBf16 pl = plan_x6(M, N, K, splits, batch > 1 ? batch : 0);
    cfg = kCfgX6[pl.cfg];
    if (batch == 1) splits = std::min(splits, pl.splits);
  }
  if (batch > 1 && !bf16 && !x6) {   // batched: tile count x batch decides between 128x128 and 64x64
    const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128) * batch;
    // the 128-tile batched case (the Winograd GEMMs): 8 waves of 64x32 with pipelined fragment
    // reads (cfg 9) — isolated 78.6 vs 88.2 us on 8 x 2048x512x512 (tools/gemm_bench.hip wino,
    // profiles/r02/gemm_wino_sweep.txt), in the step 16.465-16.485 vs 16.491-16.542 ms
    // alternating
    cfg = g_force_cfg >= 0 ? kCfg[g_force_cfg] : t128 >= 512 ? kCfg[9] : kCfg[8];
  }
  const int BKc = cfg.bk;
  int64_t kps = ((int64_t)K + splits - 1) / splits;
  kps = ((kps + BKc - 1) / BKc) * BKc;
  splits = (int)((K + kps - 1) / kps);
  if (splits < 1) splits = 1;
  AVC_CHECK_ARG(splits == 1 || workspace, "autovc_gemm_f32: split-K needs a workspace");
  Opnd oa{A, lda, a_conv_T, a_conv_C, a_tap0, nullptr, 0};
  Opnd ob{B, ldb, b_conv_T, b_conv_C, b_tap0, nullptr, 0};
  const dim3 grid((N + cfg.bn - 1) / cfg.bn, (M + cfg.bm - 1) / cfg.bm, batch > 1 ? batch : splits);
  float* slab = splits > 1 ? workspace : nullptr;
  g_batch = batch > 1 ? Batch{a_bs, b_bs, c_bs} : Batch{0, 0, 0};
  if (bf16)
    launch_gemm_bf16(cfg.id, a_trans, b_trans, grid, stream, M, N, K, oa, ob, C, ldc, bias1, bias2, accumulate,
                     (int)kps, slab, src);
  else if (x6)
    launch_gemm_x6(cfg.id, a_trans, b_trans, grid, stream, M, N, K, oa, ob, C, ldc, bias1, bias2, accumulate, (int)kps,
                   slab);
  else
    launch_gemm(cfg.id, a_trans, b_trans, grid, stream, M, N, K, oa, ob, C, ldc, bias1, bias2, accumulate, (int)kps,
                slab);
  AVC_CHECK_LAUNCH("autovc_gemm");
  if (splits > 1) {
    const int gx = (N + 255) / 256;
    const int gy = (int)std::max<int64_t>(1, std::min<int64_t>(M, 4096 / gx + 1));
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gx, gy), dim3(256), 0, stream, (int64_t)M, (int64_t)N,
                       splits, slab, C, ldc, bias1, bias2, accumulate);
    AVC_CHECK_LAUNCH("autovc_gemm/splitk_reduce");
  }
  return avc::kOk;
}

extern "C" int autovc_gemm_f32(int M, int N, int K,
                               const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                               const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                               float* C, int64_t ldc, const float* bias1, const float* bias2,
                               int accumulate, int splits, float* workspace, hipStream_t stream) {
  return gemm_impl(false, 1, 0, 0, 0, M, N, K, A, lda, a_trans, a_conv_T, a_conv_C, a_tap0, B, ldb, b_trans, b_conv_T,
                   b_conv_C, b_tap0, C, ldc, bias1, bias2, accumulate, splits, workspace, stream);
}

extern "C" int autovc_gemm_bf16_f32(int M, int N, int K,
                                    const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                                    const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                                    float* C, int64_t ldc, const float* bias1, const float* bias2,
                                    int accumulate, int splits, float* workspace, hipStream_t stream) {
  return gemm_impl(true, 1, 0, 0, 0, M, N, K, A, lda, a_trans, a_conv_T, a_conv_C, a_tap0, B, ldb, b_trans, b_conv_T,
                   b_conv_C, b_tap0, C, ldc, bias1, bias2, accumulate, splits, workspace, stream);
}


// autovc_gemm_bf16_f32 with A (src bit 0) and / or B (bit 1) read from bf16 copies the
// producers already wrote (ld in bf16 elements): half of those operands' bytes.  The recurrences' backward writes the
// gate gradients twice (dG fp32, dGb = RNE(dG)), so the weight and input gradients that
// read dGb equal autovc_gemm_bf16_f32 on dG bit for bit.
extern "C" int autovc_gemm_bf16src_f32(int M, int N, int K,
                                       const void* A, int64_t lda, int a_trans,
                                       const void* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                                       float* C, int64_t ldc, const float* bias1, const float* bias2,
                                       int accumulate, int splits, float* workspace, int src, hipStream_t stream) {
  return gemm_impl(true, 1, 0, 0, 0, M, N, K, reinterpret_cast<const float*>(A), lda, a_trans, 0, 0, 0,
                   reinterpret_cast<const float*>(B), ldb, b_trans, b_conv_T, b_conv_C, b_tap0, C, ldc, bias1, bias2, accumulate, splits, workspace, stream,
                   src);
}

extern "C" int autovc_gemm_bf16_splits(int M, int N, int K, int requested) {
  if (M <= 0 || N <= 0 || K <= 0) return requested < 1 ? 1 : requested;
  const PlanBf16 pl = plan_bf16(M, N, K, requested < 1 ? 1 : requested);
  return pl.splits;
}

// ------------------------------------------------------------------ fused Conv-BN stacks (bf16)
// (autovc_amd.functional.ConvBNChainBf16Fn; model_vc_mel.py:49-59,92-102,132-169 under
// BASELINE config 3's bf16 matmuls).  The conv GEMMs of a stack read the previous layer's
// PRE-BN output and apply its BatchNorm + activation while staging (Opnd::coef), and their
// split-K reduce emits the BatchNorm partials, so no BatchNorm pass reads or writes an
// activation of its own.
namespace {
struct BnPlan { GemmShape cfg; int splits; int kps; };
// split-K of the small outputs plan_bf16 leaves to the caller (functional._splits_for's rule:
// >= 1024 64x64 tile-splits while each keeps >= 1024 k, deep splits for < 64 tiles)
int small_splits(int M, int N, int K) {
  const int64_t tiles = (int64_t)((M + 63) / 64) * ((N + 63) / 64);
  int s = 1;
  while (tiles * s < 1024 && K / (s + 1) >= 1024 && s < 8) ++s;
  if (tiles < 64) s = std::max<int>(s, (int)std::min<int64_t>({64, K / 256, std::max<int64_t>(1, 1024 / tiles)}));
  return std::max(1, s);
}

BnPlan plan_bn(int M, int N, int K, bool dw) {
  const PlanBf16 pl = plan_bf16(M, N, K, small_splits(M, N, K));
  int splits = pl.splits;
  // (the stacks' weight gradients keep the plan's split: capping it at 2 or 1 measured
  // slower, 8.70-8.73 / 9.27-9.29 vs 8.53-8.55 ms/step, profiles/r05/ab_bf16_dw_splits.txt)
  (void)dw;
  const GemmShape cfg = pl.cfg >= 0 ? kCfgBf16[pl.cfg] : pick_config_bf16(M, N, splits);
  int64_t kps = ((int64_t)K + splits - 1) / splits;
  kps = (kps + cfg.bk - 1) / cfg.bk * cfg.bk;
  splits = (int)std::max<int64_t>(1, ((int64_t)K + kps - 1) / kps);
  return {cfg, splits, (int)kps};
}
constexpr int kStatsRows = 256;

// bnop 0 plain / 1 forward (A with BN) / 2 weight gradient (B with BN); mode 0: plain reduce
// (+ bias), 1 / 2: splitk_stats_kernel<mode> into part
int bn_gemm(int bnop, int src, int a_trans, int b_trans, int M, int N, int K, Opnd oa, Opnd ob, float* C,
            const float* bias, int mode, const float* yp, const float* coefp, int actp, double* part, float* ws,
            hipStream_t st) {
  const BnPlan pl = plan_bn(M, N, K, a_trans && b_trans);
  const dim3 grid((N + pl.cfg.bn - 1) / pl.cfg.bn, (M + pl.cfg.bm - 1) / pl.cfg.bm, pl.splits);
  g_batch = Batch{0, 0, 0};
  const int id = pl.cfg.id;
  // (layout, BNOP, SRC) combinations of the stacks; anything else is the plain fp32-source GEMM
  if (!a_trans && !b_trans && bnop == 1 && src == 0) launch_gemm_bn_bf16<true, true, 1, 0>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (!a_trans && !b_trans && bnop == 0 && src == 2) launch_gemm_bn_bf16<true, true, 0, 2>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (!a_trans && !b_trans && bnop == 0 && src == 3) launch_gemm_bn_bf16<true, true, 0, 3>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (!a_trans && b_trans && bnop == 0 && src == 3) launch_gemm_bn_bf16<true, false, 0, 3>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (a_trans && b_trans && bnop == 2 && src == 0) launch_gemm_bn_bf16<false, false, 2, 0>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (a_trans && b_trans && bnop == 0 && src == 1) launch_gemm_bn_bf16<false, false, 0, 1>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (a_trans && b_trans && bnop == 0 && src == 3) launch_gemm_bn_bf16<false, false, 0, 3>(id, grid, st, M, N, K, oa, ob, pl.kps, ws);
  else if (bnop == 0 && src == 0)
    launch_gemm_bf16(id, a_trans, b_trans, grid, st, M, N, K, oa, ob, C, N, nullptr, nullptr, 0, pl.kps, ws);
  else {
    avc::set_error("autovc_bnconv: unsupported operand combination (bnop %d, src %d)", bnop, src);
    return avc::kErrArg;
  }
  AVC_CHECK_LAUNCH("autovc_bnconv (gemm)");
  if (mode == 0) {
    const int gx = (N + 255) / 256;
    const int gy = (int)std::max<int64_t>(1, std::min<int64_t>(M, 4096 / gx + 1));
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gx, gy), dim3(256), 0, st, (int64_t)M, (int64_t)N, pl.splits, ws, C,
                       (int64_t)N, bias, nullptr, 0);
  } else {
    const dim3 g2((N + 63) / 64, (unsigned)std::min<int64_t>(kStatsRows, M));
#define AVC_STATS(MODE, ACT) hipLaunchKernelGGL((splitk_stats_kernel<MODE, ACT>), g2, dim3(256), 0, st, (int64_t)M, \
                                               (int64_t)N, pl.splits, ws, C, (int64_t)N, bias, yp, coefp, part)
    if (mode == 1) AVC_STATS(1, 0);
    else if (actp == 1) AVC_STATS(2, 1);
    else if (actp == 2) AVC_STATS(2, 2);
    else AVC_STATS(2, 0);
#undef AVC_STATS
  }
  AVC_CHECK_LAUNCH("autovc_bnconv (reduce)");
  return avc::kOk;
}

bool bn_dims_ok(int B, int T, int Ci, int Co) {
  return B > 0 && T > 0 && Ci > 0 && Co > 0 && Ci % 4 == 0 && Co % 4 == 0 &&
         4 * ((int64_t)B * T * std::max(Ci, Co) * 5 + 4 * (int64_t)std::max(Ci, Co)) < (int64_t)kOOB;
}
}  // namespace

extern "C" int autovc_bnconv_stats_rows(int64_t M) { return (int)std::max<int64_t>(1, std::min<int64_t>(kStatsRows, M)); }

extern "C" int64_t autovc_bnconv_workspace_floats(int B, int T, int Ci, int Co) {
  if (B <= 0 || T <= 0 || Ci <= 0 || Co <= 0) return 0;
  const int M = B * T;
  const BnPlan f = plan_bn(M, Co, 5 * Ci, false), x = plan_bn(M, Ci, 5 * Co, false), w = plan_bn(Co, 5 * Ci, M, true);
  return std::max({(int64_t)f.splits * M * Co, (int64_t)x.splits * M * Ci, (int64_t)w.splits * Co * 5 * Ci});
}

// src: bit 0 = the activation operand (x / dy), bit 1 = the other (W / x) is bf16 in memory
// (2-byte elements, same strides in elements); a BN-on-load operand (x_coef) must be fp32
bool bn_src_ok(int src, int Ci, int Co) { return src >= 0 && src <= 3 && (src == 0 || (Ci % 8 == 0 && Co % 8 == 0)); }

extern "C" int autovc_bnconv_fwd_bf16_f32(int B, int T, int Ci, int Co, const void* x, const float* x_coef, int x_act,
                                          const void* Wf, const float* bias, float* y, double* part, int src,
                                          float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(bn_dims_ok(B, T, Ci, Co) && x && Wf && y && part && workspace, "autovc_bnconv_fwd_bf16_f32: bad args");
  AVC_CHECK_ARG(x_act >= 0 && x_act <= 2 && AVC_ALIGNED16(x) && AVC_ALIGNED16(Wf) && (!x_coef || AVC_ALIGNED16(x_coef)),
                "autovc_bnconv_fwd_bf16_f32: activation / alignment");
  AVC_CHECK_ARG(bn_src_ok(src, Ci, Co) && !(x_coef && (src & 1)), "autovc_bnconv_fwd_bf16_f32: bad src %d", src);
  AVC_CHECK_ARG(!x_coef || Ci <= kBnMaxC, "autovc_bnconv_fwd_bf16_f32: BatchNorm input channels > %d", kBnMaxC);
  const int M = B * T;
  const Opnd oa{(const float*)x, Ci, T, Ci, -2, x_coef, x_act};
  const Opnd ob{(const float*)Wf, 5 * Ci, 0, 0, 0, nullptr, 0};
  return bn_gemm(x_coef ? 1 : 0, src, 0, 0, M, Co, 5 * Ci, oa, ob, y, bias, 1, nullptr, nullptr, 0, part, workspace,
                 stream);
}

extern "C" int autovc_bnconv_dx_bf16_f32(int B, int T, int Co, int Ci, const void* dy, const void* Wd, float* dz,
                                         const float* y_prev, const float* coef_prev, int act_prev, double* part,
                                         int src, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(bn_dims_ok(B, T, Ci, Co) && dy && Wd && dz && workspace, "autovc_bnconv_dx_bf16_f32: bad args");
  AVC_CHECK_ARG(!y_prev || (coef_prev && part && act_prev >= 0 && act_prev <= 2),
                "autovc_bnconv_dx_bf16_f32: the BatchNorm sums need y_prev, coef_prev, part");
  AVC_CHECK_ARG(AVC_ALIGNED16(dy) && AVC_ALIGNED16(Wd), "autovc_bnconv_dx_bf16_f32: alignment");
  AVC_CHECK_ARG(bn_src_ok(src, Ci, Co) && (src == 0 || src == 3), "autovc_bnconv_dx_bf16_f32: bad src %d", src);
  const int M = B * T;
  const Opnd oa{(const float*)dy, Co, T, Co, -2, nullptr, 0};
  const Opnd ob{(const float*)Wd, Ci, 0, 0, 0, nullptr, 0};
  return bn_gemm(0, src, 0, 1, M, Ci, 5 * Co, oa, ob, dz, nullptr, y_prev ? 2 : 0, y_prev, coef_prev, act_prev, part,
                 workspace, stream);
}

extern "C" int autovc_bnconv_dw_bf16_f32(int B, int T, int Co, int Ci, const void* dy, const void* x,
                                         const float* x_coef, int x_act, float* dWf, int src, float* workspace,
                                         hipStream_t stream) {
  AVC_CHECK_ARG(bn_dims_ok(B, T, Ci, Co) && dy && x && dWf && workspace, "autovc_bnconv_dw_bf16_f32: bad args");
  AVC_CHECK_ARG(x_act >= 0 && x_act <= 2 && AVC_ALIGNED16(dy) && AVC_ALIGNED16(x) && (!x_coef || AVC_ALIGNED16(x_coef)),
                "autovc_bnconv_dw_bf16_f32: activation / alignment");
  AVC_CHECK_ARG(bn_src_ok(src, Ci, Co) && !(x_coef && (src & 2)), "autovc_bnconv_dw_bf16_f32: bad src %d", src);
  AVC_CHECK_ARG(!x_coef || Ci <= kBnMaxC, "autovc_bnconv_dw_bf16_f32: BatchNorm input channels > %d", kBnMaxC);
  const int M = B * T;
  const Opnd oa{(const float*)dy, Co, 0, 0, 0, nullptr, 0};
  const Opnd ob{(const float*)x, Ci, T, Ci, -2, x_coef, x_act};
  return bn_gemm(x_coef ? 2 : 0, src, 1, 1, Co, 5 * Ci, M, oa, ob, dWf, nullptr, 0, nullptr, nullptr, 0, nullptr,
                 workspace, stream);
}

extern "C" int autovc_gemm_set_lds_reserve(int bytes) {
  AVC_CHECK_ARG(bytes >= 0 && bytes <= 96 * 1024, "autovc_gemm_set_lds_reserve: 0 <= bytes <= 96 KiB");
  g_lds_reserve = (unsigned)bytes;
  return avc::kOk;
}

// batch independent GEMMs C_z = A_z B_z (z < batch) in one launch; operand / output z starts
// z * (a_bstride, b_bstride, c_bstride) floats after the first (Winograd conv: 8 GEMMs)
extern "C" int autovc_gemm_batched_f32(int batch, int M, int N, int K, const float* A, int64_t lda,
                                       int64_t a_bstride, int a_trans, const float* B, int64_t ldb,
                                       int64_t b_bstride, int b_trans, float* C, int64_t ldc, int64_t c_bstride,
                                       int bf16, hipStream_t stream) {
  AVC_CHECK_ARG(batch >= 1 && batch <= 65535 && (batch == 1 || c_bstride > 0),
                "autovc_gemm_batched_f32: bad batch / strides");
  AVC_CHECK_ARG(a_bstride % 4 == 0 && b_bstride % 4 == 0 && c_bstride >= 0,
                "autovc_gemm_batched_f32: operand batch strides must be multiples of 4");
  AVC_CHECK_ARG(4 * ((int64_t)batch * std::max(a_bstride, b_bstride)) < (int64_t)kOOB,
                "autovc_gemm_batched_f32: batched operands must stay below 2 GiB");
  return gemm_impl(bf16 != 0, batch, a_bstride, b_bstride, c_bstride, M, N, K, A, lda, a_trans, 0, 0, 0, B, ldb,
                   b_trans, 0, 0, 0, C, ldc, nullptr, nullptr, 0, 1, nullptr, stream);
}
