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
// Tiling: 128x128 block tile, BK = 16, 256 threads = 4 waves in 2x2, each wave 64x64 =
// 2x2 MFMA 32x32 tiles (64 accumulators / lane).  LDS holds [row][BK+4] images of both
// operands (row stride 80 B: conflict-free ds_read_b128 fragment reads); within a BK
// stage lane half h takes k = 8h..8h+7 for its 8 MFMAs (the k order inside a stage is
// a permutation applied to A and B alike, so the sum is unchanged).  Register-staged
// double buffer, one barrier per stage.  Split-K writes fp32 slabs reduced in k order
// by a second kernel (deterministic; no float atomics).
#include <algorithm>

#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 16, LDK = BK + 4;
constexpr int kThreads = 256;

struct Opnd {
  const float* p;
  int64_t ld;
  int conv_T, conv_C, tap0;  // conv_T == 0: plain matrix
};

// load 4 consecutive contiguous-index elements of an operand at (r..., k...) -> float4
// RK: row r, k..k+3 contiguous.   CK: k-row kk, r..r+3 contiguous.
template <bool RK>
__device__ __forceinline__ f32x4 load4(const Opnd& o, int64_t r, int64_t k, int64_t R, int64_t K) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  const int64_t f = RK ? r : k;        // frame / row index of storage
  const int64_t q = RK ? k : r;        // contiguous index
  const bool in = RK ? (r < R && k < K) : (k < K && r < R);
  if (!in) return v;
  int64_t off = f * o.ld + q;
  if (o.conv_T > 0) {
    const int tap = (int)(q / o.conv_C);
    const int64_t tt = f % o.conv_T + tap + o.tap0;
    if (tt < 0 || tt >= o.conv_T) return v;
    off += (int64_t)o.tap0 * o.ld;
  }
  return *reinterpret_cast<const f32x4*>(o.p + off);
}

// Each thread stages 2 float4 per operand tile (128 rows x 16 k = 512 float4).
template <bool RK>
struct Stager {
  f32x4 v[2];
  __device__ __forceinline__ void load(const Opnd& o, int64_t r0, int64_t k0, int64_t R, int64_t K, int tid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (RK) {
        const int row = (tid >> 2) + 64 * s, kq = tid & 3;
        v[s] = load4<true>(o, r0 + row, k0 + 4 * kq, R, K);
      } else {
        const int kr = tid & 15, rq = (tid >> 4) + 16 * s;
        v[s] = load4<false>(o, r0 + 4 * rq, k0 + kr, R, K);
      }
    }
  }
  __device__ __forceinline__ void store(float* lds, int tid) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (RK) {
        const int row = (tid >> 2) + 64 * s, kq = tid & 3;
        *reinterpret_cast<f32x4*>(lds + row * LDK + 4 * kq) = v[s];
      } else {
        const int kr = tid & 15, rq = (tid >> 4) + 16 * s;
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[(4 * rq + j) * LDK + kr] = v[s][j];
      }
    }
  }
};

template <bool A_RK, bool B_RK>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(
    int M, int N, int K, Opnd A, Opnd B, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias1, const float* __restrict__ bias2, int accumulate,
    int k_per_split, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float smem[2][2][BM * LDK];  // [buf][A/B]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = min((int64_t)K, kbeg + k_per_split);
  const int nk = (int)((kend - kbeg + BK - 1) / BK);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stager<A_RK> sa;
  Stager<B_RK> sb;
  if (nk > 0) {
    sa.load(A, m0, kbeg, M, kend, tid);
    sb.load(B, n0, kbeg, N, kend, tid);
    sa.store(smem[0][0], tid);
    sb.store(smem[0][1], tid);
  }
  __syncthreads();

  const int h = lane >> 5, li = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      sa.load(A, m0, kbeg + (int64_t)(kt + 1) * BK, M, kend, tid);
      sb.load(B, n0, kbeg + (int64_t)(kt + 1) * BK, N, kend, tid);
    }
    const float* As = smem[buf][0];
    const float* Bs = smem[buf][1];
    f32x4 af[2][2], bf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float* pa = As + (wr * 64 + t * 32 + li) * LDK + 8 * h;
      const float* pb = Bs + (wc * 64 + t * 32 + li) * LDK + 8 * h;
      af[t][0] = *reinterpret_cast<const f32x4*>(pa);
      af[t][1] = *reinterpret_cast<const f32x4*>(pa + 4);
      bf[t][0] = *reinterpret_cast<const f32x4*>(pb);
      bf[t][1] = *reinterpret_cast<const f32x4*>(pb + 4);
    }
#pragma unroll
    for (int p = 0; p < 8; ++p) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][p >> 2][p & 3], bf[j][p >> 2][p & 3],
                                                            acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      sa.store(smem[buf ^ 1][0], tid);
      sb.store(smem[buf ^ 1][1], tid);
    }
    __syncthreads();
  }

  // epilogue: C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* out = slab ? slab + (int64_t)blockIdx.z * M * N : C;
  const int64_t ld = slab ? N : ldc;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wc * 64 + j * 32 + li;
    if (n >= N) continue;
    float bsum = 0.f;
    if (!slab) {
      if (bias1) bsum += bias1[n];
      if (bias2) bsum += bias2[n];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float v = acc[i][j][r] + bsum;
          float* dst = out + m * ld + n;
          if (!slab && accumulate) v += *dst;
          *dst = v;
        }
      }
    }
  }
}

__global__ void splitk_reduce_kernel(int64_t M, int64_t N, int splits, const float* __restrict__ slab,
                                     float* __restrict__ C, int64_t ldc, const float* __restrict__ bias1,
                                     const float* __restrict__ bias2, int accumulate) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, n = i % N;
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += slab[s * total + i];
    if (bias1) v += bias1[n];
    if (bias2) v += bias2[n];
    float* dst = C + m * ldc + n;
    if (accumulate) v += *dst;
    *dst = v;
  }
}

bool aligned_ld(int64_t ld) { return (ld & 3) == 0; }

}  // namespace

extern "C" int64_t autovc_gemm_workspace_floats(int M, int N, int splits) {
  return splits > 1 ? (int64_t)splits * M * N : 0;
}

extern "C" int autovc_gemm_f32(int M, int N, int K,
                               const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                               const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                               float* C, int64_t ldc, const float* bias1, const float* bias2,
                               int accumulate, int splits, float* workspace, hipStream_t stream) {
  AVC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "autovc_gemm_f32: negative dims");
  if (M == 0 || N == 0) return avc::kOk;
  AVC_CHECK_ARG(A && B && C, "autovc_gemm_f32: null operand");
  AVC_CHECK_ARG(AVC_ALIGNED16(A) && AVC_ALIGNED16(B), "autovc_gemm_f32: A/B must be 16-byte aligned");
  AVC_CHECK_ARG(aligned_ld(lda) && aligned_ld(ldb), "autovc_gemm_f32: lda/ldb must be multiples of 4");
  // the contiguous extent of each operand must be a multiple of 4 (float4 staging)
  AVC_CHECK_ARG(a_trans ? (M % 4 == 0) : (K % 4 == 0), "autovc_gemm_f32: A contiguous dim %% 4 != 0");
  AVC_CHECK_ARG(b_trans ? (N % 4 == 0) : (K % 4 == 0), "autovc_gemm_f32: B contiguous dim %% 4 != 0");
  AVC_CHECK_ARG(!a_conv_T || (a_conv_C % 4 == 0 && a_conv_C > 0),
                "autovc_gemm_f32: A conv channels must be a positive multiple of 4");
  AVC_CHECK_ARG(!b_conv_T || (b_conv_C % 4 == 0 && b_conv_C > 0),
                "autovc_gemm_f32: B conv channels must be a positive multiple of 4");
  if (splits < 1) splits = 1;
  int64_t kps = ((int64_t)K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  splits = (int)((K + kps - 1) / kps);
  if (splits < 1) splits = 1;
  AVC_CHECK_ARG(splits == 1 || workspace, "autovc_gemm_f32: split-K needs a workspace");
  Opnd oa{A, lda, a_conv_T, a_conv_C, a_tap0};
  Opnd ob{B, ldb, b_conv_T, b_conv_C, b_tap0};
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  float* slab = splits > 1 ? workspace : nullptr;
#define AVC_GEMM_LAUNCH(AR, BR)                                                                   \
  hipLaunchKernelGGL((gemm_kernel<AR, BR>), grid, dim3(kThreads), 0, stream, M, N, K, oa, ob, C, \
                     ldc, bias1, bias2, accumulate, (int)kps, slab)
  if (!a_trans && !b_trans) AVC_GEMM_LAUNCH(true, true);
  else if (!a_trans && b_trans) AVC_GEMM_LAUNCH(true, false);
  else if (a_trans && !b_trans) AVC_GEMM_LAUNCH(false, true);
  else AVC_GEMM_LAUNCH(false, false);
#undef AVC_GEMM_LAUNCH
  AVC_CHECK_LAUNCH("autovc_gemm_f32");
  if (splits > 1) {
    const int64_t total = (int64_t)M * N;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, stream, (int64_t)M, (int64_t)N,
                       splits, slab, C, ldc, bias1, bias2, accumulate);
    AVC_CHECK_LAUNCH("autovc_gemm_f32/splitk_reduce");
  }
  return avc::kOk;
}
