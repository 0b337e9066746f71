// WaveNet vocoder inference (r9y9 wavenet_vocoder 0.1.1 incremental_forward, driven by
// synthesis.py:44-73) for gfx950.
//
// Per output sample the network is a chain of 24 residual layers; every layer needs the
// whole previous layer's output, so one sample step is a sequence of grid-wide
// dependencies, each paid as a kernel boundary (the cheapest grid-wide sync on MI355X,
// MI355X_MICROARCH.md price list).  The step is ONE kernel per layer + a skip tail + head:
//
//   layer(l) : g_l = tanh(z[:256]) * sigmoid(z[256:]),  z = the dilated conv of layer l:
//                z = W_0 x_l(t-2d) + W_1 x_l(t-d) + W_2 x_l(t) + pre(l, t)
//              with the current tap folded back one layer (exact in real arithmetic):
//                x_l(t) = sqrt(.5) (W_out(l-1) g_(l-1) + b_out(l-1) + x_(l-1)(t))
//                W_2 x_l(t) = [sqrt(.5) W_2 W_out(l-1)] g_(l-1) + [sqrt(.5) W_2] x_(l-1)(t)
//                             + sqrt(.5) W_2 b_out(l-1)  (the last term folded into pre)
//              so the layer's GEMV on the chain reads only [g_(l-1); x_(l-1)(t)] (768
//              inputs): the past taps W_0 x_l(t-2d) + W_1 x_l(t-d) were multiplied by the
//              previous step's tail and head launches (past_taps) and arrive with pre.
//              The same kernel does layer l-1's residual work: its slice of x_l(t)
//              (written to ring l for the later taps) and of the skip accumulation.
//              layer(0) first samples the previous output (the MoL head from the head
//              kernel's partial sums + Philox draw) and builds x_0 = first_conv(input).
//   tail     : the last layer's skip rows (+ past taps of half the layers for step t+1)
//   head     : h1 = relu(W1 relu(skips) + b1) and its MoL partials (+ the other half)
// 26 launches per sample step instead of 49 for the two-kernel-per-layer form.
//
// pre(l, t) = W_cond(l) c_up(t) + b_cond(l) + b_conv(l) for every layer and sample comes
// from ONE MFMA GEMM per conditioning chunk (autovc_gemm_f32) — the conditioning 1x1 convs
// are sample-independent, so they leave the sequential chain.
//
// Layer inputs (x_0 included) live in per-layer rings of RING (power of two >= 2*d_max + 1)
// frames: the dilated taps read ring slots (t - j*d) & (RING-1); slots before
// t = 0 are zero, as the reference's zero-initialised conv input buffers.
//
// The ring slot and the conditioning row of a step are kernel arguments (static in a
// captured hipGraph: one graph per (slot, row) of its first step), so no step kernel waits
// for a dependent counter read; only layer 0 (sampling draw, recorded outputs) reads the
// step counter, which the head advances.
#include "common.h"
#include "../../include/autovc_hip.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace {

constexpr float kSqrtHalf = 0.70710677f;  // float(math.sqrt(0.5))
constexpr int kBT = 8;                    // utterances per batch tile
constexpr int kMaxNO = 32;                // MoL head width limit (3 x up to 10 mixtures)
constexpr int kCtrSlots = 128;

struct WnArgs {
  int B, T, R, G, S, NO, K, RING, n_layers, lps, Tch, legacy;
  const float* packed;
  const float* pre;
  float* ring;
  float* yin;
  float* skip;
  float* h1;
  float* gbuf;
  float* ptap;       // past-tap products of the next step: (2, n_layers, B, G), by step parity
  float* molp;       // MoL head partials of the head kernel's row blocks: (S / kHR, B, kMaxNO)
  // all-CU generation (wn_grid_kernel): tagged 16-byte hand-off granules
  float* gring;      // (n_layers, RING, B, 256) x {g_l[o], x_l[2o], x_l[2o+1], step + 1}
  float* gsk;        // (B, 256) x {skip sum, -, -, step + 1}
  float* gh1;        // (B, 256) x {h1, -, -, step + 1}
  float* gpt;        // (2 parities, n_layers, B, 512) x {past-tap sum, step + 1} (8 bytes)
  // layer-pipelined generation (wn_pipe_kernel): each layer's skip rows, handed to the tail
  float* gsl;        // (n_layers, B, 256) x {skip row of layer l, step + 1} (8 bytes)
  int* ctr;
  const float* teacher;
  int teacher_len;
  float* y_out;
  float* mol_out;
  uint32_t seed_lo, seed_hi;
  int utt_base;
  float log_scale_min;
};

// ---- packed weight layout (floats): see autovc_wavenet_packed_floats
// per layer: gate block G x KX, KX = K*R + H: [W_0 .. W_(K-2) (tap-major) | sqrt(.5) W_(K-1) W_out(l-1)
// (H) | sqrt(.5) W_(K-1) (R)] (layer 0: [W_0 .. W_(K-2) | 0 | W_(K-1)]); then the layer's
// [W_out (R x H); W_skip (S x H)] and their biases (R + S).
__host__ __device__ inline int gate_width(const WnArgs& a) { return a.K * a.R + a.G / 2; }
__host__ __device__ inline int64_t layer_floats(const WnArgs& a) {
  const int H = a.G / 2;
  return (int64_t)a.G * gate_width(a) + (int64_t)(a.R + a.S) * H + (a.R + a.S);
}
__host__ __device__ inline float* gbuf_of(const WnArgs& a, int l) {
  return a.gbuf + (int64_t)(l & 1) * a.B * (a.G / 2);
}
__host__ __device__ inline const float* layer_base(const WnArgs& a, int l) {
  return a.packed + 2 * (int64_t)a.R + l * layer_floats(a);
}
__host__ __device__ inline const float* head_base(const WnArgs& a) { return layer_base(a, a.n_layers); }

// ---- Philox4x32-10 uniforms (oracle/wavenet.py philox_uniforms)
__device__ inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ inline float uniform_from_word(uint32_t w) {
#pragma clang fp contract(off)
  const double v = ((double)(w >> 9) + 0.5) * 1.1920928955078125e-07;  // 2^-23
  return (float)(1e-5 + (1.0 - 2e-5) * v);
}

// sample_from_discretized_mix_logistic (wavenet_vocoder/mixture.py) with Philox uniforms.
__device__ float mol_sample(const float* y, int nr, int64_t t, int utt, const WnArgs& a) {
  float u[12];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    uint32_t c[4] = {(uint32_t)t, (uint32_t)utt, (uint32_t)j, 0u};
    philox(c, a.seed_lo, a.seed_hi);
    u[4 * j] = uniform_from_word(c[0]);
    u[4 * j + 1] = uniform_from_word(c[1]);
    u[4 * j + 2] = uniform_from_word(c[2]);
    u[4 * j + 3] = uniform_from_word(c[3]);
  }
  int best = 0;
  float bv = -INFINITY;
  for (int j = 0; j < nr; ++j) {
    const float uj = j < 10 ? u[j] : 0.5f;  // nr <= 10 is checked on the host
    const float v = y[j] - logf(-logf(uj));
    if (v > bv) { bv = v; best = j; }
  }
  const float mean = y[nr + best];
  const float ls = fmaxf(y[2 * nr + best], a.log_scale_min);
  const float ul = u[10];
  const float x = mean + expf(ls) * (logf(ul) - logf(1.0f - ul));
  return fminf(fmaxf(x, -1.0f), 1.0f);
}

// The step-dependent, parameter-independent part of mol_sample for one (utterance, index j)
// lane: j < nr -> logf(-logf(u_j)) (the Gumbel term), j == 10 -> logf(u) - logf(1 - u) of the
// logistic draw.  Computed while the MoL parameters are still in flight; mol_finish finishes
// with the same float operations as mol_sample.
__device__ inline float mol_noise(int j, int64_t t, int utt, const WnArgs& a) {
  uint32_t c[4] = {(uint32_t)t, (uint32_t)utt, (uint32_t)(j >> 2), 0u};
  philox(c, a.seed_lo, a.seed_hi);
  const int w = j & 3;
  const float u = uniform_from_word(w == 0 ? c[0] : w == 1 ? c[1] : w == 2 ? c[2] : c[3]);
  if (j == 10) return logf(u) - logf(1.0f - u);
  return logf(-logf(u));
}

// Butterfly reduction of NV per-lane partial sums over the 64 lanes of a wave (NV-1
// exchanges for the halving rounds instead of 6*NV; every array index a compile-time
// constant, so nothing is demoted to LDS) on gfx950's cross-lane hardware instead of
// ds_bpermute (an LDS round trip per shuffle, 4-5 % slower per WaveNet sample step,
// profiles/r04/wn_grid_ab.txt): level 0 pairs lanes l, l ^ 32 with v_permlane32_swap, level 1 l,
// l ^ 16 with v_permlane16_swap (one swap moves two values: the kept half of one lane group
// and the sent half of the other), level 2 l, l ^ 15 (DPP row_mirror), level 3 l, l ^ 7
// (row_half_mirror), levels 4 / 5 l ^ 2, l ^ 1 (quad_perm).  The pairings generate every
// lane, so lane L with (L & (64/NV - 1)) == 0 ends with the full sum of value L / (64/NV), as
// wave_reduce_multi; the pairing tree is fixed, so every NV rounds each value alike.
template <int LVL>
__device__ __forceinline__ float dpp_partner(float v) {
  constexpr int ctrl = LVL == 2 ? 0x140 : LVL == 3 ? 0x141 : LVL == 4 ? 0x4E : 0xB1;
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, false));
}
template <int N, int LVL>
__device__ __forceinline__ void butterfly_hw(float* cur, int lane) {
  if constexpr (LVL < 6) {
    constexpr int bit = LVL == 0 ? 32 : LVL == 1 ? 16 : LVL == 2 ? 8 : LVL == 3 ? 4 : LVL == 4 ? 2 : 1;
    if constexpr (LVL < 2) {
      if constexpr (N > 1) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
          const auto r = LVL == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(cur[j]), __float_as_uint(cur[j + N / 2]), false, false)
                                  : __builtin_amdgcn_permlane16_swap(__float_as_uint(cur[j]), __float_as_uint(cur[j + N / 2]), false, false);
          cur[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
        }
        butterfly_hw<N / 2, LVL + 1>(cur, lane);
      } else {
        const auto r = LVL == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(cur[0]), __float_as_uint(cur[0]), false, false)
                                : __builtin_amdgcn_permlane16_swap(__float_as_uint(cur[0]), __float_as_uint(cur[0]), false, false);
        cur[0] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
        butterfly_hw<1, LVL + 1>(cur, lane);
      }
    } else {
      if constexpr (N > 1) {
        const bool up = (lane & bit) != 0;
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
          const float keep = up ? cur[j + N / 2] : cur[j];
          const float send = up ? cur[j] : cur[j + N / 2];
          cur[j] = keep + dpp_partner<LVL>(send);
        }
        butterfly_hw<N / 2, LVL + 1>(cur, lane);
      } else {
        cur[0] += dpp_partner<LVL>(cur[0]);
        butterfly_hw<1, LVL + 1>(cur, lane);
      }
    }
  }
}

template <int NV>
__device__ inline float wave_reduce_hw(float (&v)[NV], int lane) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "power-of-two value count");
  float cur[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) cur[j] = v[j];
  butterfly_hw<NV, 0>(cur, lane);
  return cur[0];
}

template <int NV>
__device__ inline float wave_reduce_multi(float (&v)[NV], int lane) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "power-of-two value count");
  float cur[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) cur[j] = v[j];
  butterfly_hw<NV, 0>(cur, lane);
  return cur[0];
}

__device__ inline float dot4(f32x4 w, f32x4 x, float acc) {
  acc += w[0] * x[0];
  acc += w[1] * x[1];
  acc += w[2] * x[2];
  acc += w[3] * x[3];
  return acc;
}

__device__ inline f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// The absolute sample step: a kernel argument for direct launches (targ >= 0), else (graph
// replay) the counter the previous step's head kernel advanced.  Only layer 0 (sampling draw,
// recorded outputs, teacher inputs) and the head read it: every load of the step kernels is
// addressed by the ring slot and the conditioning row, which are kernel arguments in both
// modes (a captured graph covers one RING-aligned conditioning chunk), so no load waits for
// a dependent counter read (it cost 0.86 us per launch on the critical path).
__device__ inline int abs_step(const WnArgs& a, int targ) { return targ >= 0 ? targ : a.ctr[0]; }

// ring row of layer input l (l = 0: x_0 = first_conv(input)) at slot s: (B, R)
__device__ inline float* ring_row(const WnArgs& a, int l, int s) {
  return a.ring + ((int64_t)l * a.RING + s) * a.B * a.R;
}

// A workgroup barrier that waits for LDS traffic only: __syncthreads' release fence would
// also drain the wave's outstanding global loads.
__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MoL parameters of step tp = tp1 - 1 (from h1) for the batch tile, then the input of
// step tp1.  Runs on the whole workgroup (NW waves).  Writes s_in[b].
template <int NW, int UB>
__device__ void sample_stage(const WnArgs& a, int tp1, int b0, int nb, float* s_mol, float* s_in) {
  constexpr int MAXR = (kMaxNO + NW - 1) / NW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* hb = head_base(a);
  const float* W2 = hb + (int64_t)a.S * a.S + a.S;
  const float* b2 = W2 + (int64_t)a.NO * a.S;
  const int tp = tp1 - 1;
  if (tp >= 0) {
    float acc[MAXR][UB];
#pragma unroll
    for (int q = 0; q < MAXR; ++q)
#pragma unroll
      for (int b = 0; b < UB; ++b) acc[q][b] = 0.f;
    for (int k = lane * 4; k < a.S; k += 256) {
      f32x4 h[UB];
#pragma unroll
      for (int b = 0; b < UB; ++b) h[b] = ld4(a.h1 + (int64_t)(b0 + (b < nb ? b : 0)) * a.S + k);
      f32x4 w[MAXR];
#pragma unroll
      for (int q = 0; q < MAXR; ++q) {
        const int r = wave + q * NW;
        w[q] = ld4(W2 + (int64_t)(r < a.NO ? r : 0) * a.S + k);
      }
#pragma unroll
      for (int q = 0; q < MAXR; ++q)
#pragma unroll
        for (int b = 0; b < UB; ++b) acc[q][b] = dot4(w[q], h[b], acc[q][b]);
    }
#pragma unroll
    for (int q = 0; q < MAXR; ++q) {
      const int r = wave + q * NW;
      if (r < a.NO) {  // wave-uniform
        const float v = wave_reduce_multi<UB>(acc[q], lane);
        if ((lane & (64 / UB - 1)) == 0) s_mol[(lane / (64 / UB)) * kMaxNO + r] = v + b2[r];
      }
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nb) {
    const int b = threadIdx.x;
    const int gb = b0 + b;
    float in_v = 0.f;
    float smp = 0.f;
    if (tp >= 0) smp = mol_sample(s_mol + b * kMaxNO, a.NO / 3, tp, a.utt_base + gb, a);
    if (a.teacher != nullptr && tp1 < a.teacher_len) in_v = a.teacher[(int64_t)gb * a.teacher_len + tp1];
    else if (tp >= 0) in_v = smp;
    if (s_in) s_in[b] = in_v;
    if (blockIdx.x == 0) {
      if (tp1 < a.T) a.yin[(int64_t)gb * a.T + tp1] = in_v;
      if (tp >= 0) {
        a.y_out[(int64_t)gb * a.T + tp] = smp;
        if (a.mol_out)
          for (int j = 0; j < a.NO; ++j) a.mol_out[((int64_t)gb * a.T + tp) * a.NO + j] = s_mol[b * kMaxNO + j];
      }
    }
  }
  __syncthreads();
}

// layer(l): one workgroup per kRP gate pairs (o, o + G/2) and kUB utterances: 2*kRP gate rows
// x kUB utterances per workgroup (4 x 4 reads fewer operand bytes per CU than 2 rows x 8
// utterances: (rows + utterances) x K floats; the per-CU operand fill bounds the launch).
// Waves 0..kGW-1 split the GEMV's KX inputs in 256-float chunks (no chunk straddles a
// segment: R, H % 256 == 0); for l >= 1 waves kGW..kGW+kRW-1 do layer l-1's residual rows
// (R/H rows of x_l(t) and S/H skip rows per gate pair) with every operand they need, the
// skip accumulator and the residual input included, loaded at kernel start.  Loads that
// do not depend on the step (weights, biases, the skip accumulator) are issued before the
// step counter is read.
constexpr int kRP = 2;                    // gate pairs per workgroup
constexpr int kUB = 4;                    // utterances per workgroup
constexpr int kGC = 3;                    // chunks of the critical GEMV [g_(l-1) | x_(l-1)(t)]:
                                          // H + R = 768 = 3 x 256 for r9y9
constexpr int kGS = 2;            // gate-row groups: 1 = a wave takes all 4 rows of its
                                          // chunk, 2 = two waves per chunk, 2 rows each
constexpr int kGW = kGC * kGS;            // gate waves
constexpr int kWR = 2 * kRP / kGS;        // gate rows per gate wave
constexpr int kRW = 2;                // residual waves
constexpr int kResRows = 8 / kRW;         // residual rows per residual wave (>= kRP*(R+S)/H / kRW)
constexpr int kLayerThreads = 64 * (kGW + kRW);
constexpr int kTailWaves = 4;         // tail / head: one wave per output row
constexpr int kPR = 32;                // past-tap workgroups: gate rows per workgroup (16, 32 or 64)
constexpr int kPRT = kPR / 16;            // 16-row MFMA tiles per workgroup

// MoL head output of the previous step: the head kernel's row-block workgroups (kHR rows
// of h1 each) also multiply their rows into W2 and leave (S / kHR) partial sums per (utterance,
// output); layer 0 adds them in fixed order — 16 loads per output issued at kernel start
// instead of W2 (30 KB) and h1 per workgroup and a GEMV on the chain.
constexpr int kHR = 16;                   // head rows per head workgroup (4 waves x 4 rows)

// s_mol <- MoL parameters of step tp1 - 1; then s_in <- the input of step tp1 (sampled, or
// the teacher value); block 0 of the tile records the sample and the input.
__device__ void mol_finish(const WnArgs& a, int tp1, int wave, int lane, int b0, int nb, float mol_v, float* s_mol,
                           const float* s_gum, float* s_in) {
  const int tp = tp1 - 1;
  if (tp >= 0 && (int)threadIdx.x < kUB * kMaxNO) s_mol[threadIdx.x] = mol_v;   // [b][j], b = tid / kMaxNO
  lds_barrier();
  if (wave == 0) {
    // the mixture pick on 16 lanes per utterance (lane 16 b + j): the argmax of
    // y_j - logf(-logf(u_j)) over j < nr in four shuffle rounds, ties to the lowest j (the
    // serial loop's strict '>'; NaN never wins), then lane j = 0 finishes as mol_sample does
    const int b = lane >> 4, j = lane & 15, nr = a.NO / 3;
    float v = -INFINITY;
    if (tp >= 0 && b < nb && j < nr) {
      v = s_mol[b * kMaxNO + j] - s_gum[b * 16 + j];
      if (!(v == v)) v = -INFINITY;
    }
    int bi = j;
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) {
      const float ov = __shfl_xor(v, m);
      const int oi = __shfl_xor(bi, m);
      if (ov > v || (ov == v && oi < bi)) { v = ov; bi = oi; }
    }
    if (j == 0 && b < nb) {
      const int gb = b0 + b;
      float in_v = 0.f;
      float smp = 0.f;
      if (tp >= 0) {
        const float mean = s_mol[b * kMaxNO + nr + bi];
        const float ls = fmaxf(s_mol[b * kMaxNO + 2 * nr + bi], a.log_scale_min);
        const float x = mean + expf(ls) * s_gum[b * 16 + 10];
        smp = fminf(fmaxf(x, -1.0f), 1.0f);
      }
      if (a.teacher != nullptr && tp1 < a.teacher_len) in_v = a.teacher[(int64_t)gb * a.teacher_len + tp1];
      else if (tp >= 0) in_v = smp;
      s_in[b] = in_v;
      if (blockIdx.x == 0 && tp >= 0) {
        a.y_out[(int64_t)gb * a.T + tp] = smp;
        if (a.mol_out)
          for (int q = 0; q < a.NO; ++q) a.mol_out[((int64_t)gb * a.T + tp) * a.NO + q] = s_mol[b * kMaxNO + q];
      }
    }
  }
  lds_barrier();
}

template <bool L0>
__global__ __launch_bounds__(kLayerThreads) void wn_layer_kernel(WnArgs a, int layer, int slot, int prow, int targ) {
  // slot: ring slot of this sample step (t & (RING-1)); prow: its row in the conditioning
  // chunk (t % Tch); targ: t for direct launches, -1 under graph replay (layer 0 then reads
  // the step counter)
  __shared__ float s_mol[L0 ? kUB * kMaxNO : 1];
  __shared__ float s_gum[L0 ? kUB * 16 : 1];
  __shared__ float s_in[kUB];
  __shared__ float s_red[kGW][kWR * kUB];
  __shared__ int s_arrived;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b0 = blockIdx.y * kUB;
  const int nb = min(kUB, a.B - b0);
  const int H = a.G / 2;
  const int o0 = blockIdx.x * kRP;          // first gate pair of the workgroup
  const int KX = gate_width(a);
  const int KT = (a.K - 1) * a.R;           // end of the ring taps
  const float* base = layer_base(a, layer);
  const float* gprev = L0 ? nullptr : gbuf_of(a, layer - 1);
  auto urow = [&](int b) { return (int64_t)(b0 + (b < nb ? b : 0)); };
  auto wrow = [&](int r) { return o0 + (r >> 1) + (r & 1) * H; };   // gate row r of the workgroup

  // inputs of GEMV chunk kc (k = kc + lane*4, kc >= KT: the ring taps 0..K-2 were
  // multiplied by the previous step's tail/head launches into ptap) for the kUB utterances;
  // false = the chunk contributes nothing (layer 0's g_(l-1) block has zero weights; its
  // current tap is the sampled input, built after the draw)
  auto load_x = [&](int kc, f32x4 (&x)[kUB]) -> bool {
    const int k = kc + lane * 4;
    if (L0) return false;
    if (kc < KT + H) {                      // g_(l-1)
#pragma unroll
      for (int b = 0; b < kUB; ++b) x[b] = ld4(gprev + urow(b) * H + (k - KT));
    } else {                                // current tap x_(l-1)(t)
      const float* xr = ring_row(a, layer - 1, slot) + (k - KT - H);
#pragma unroll
      for (int b = 0; b < kUB; ++b) x[b] = ld4(xr + urow(b) * a.R);
    }
    return true;
  };

  // ---------------- prologue: every load of the launch, none waits for another
  const int c0 = wave % kGC, grp = wave / kGC;  // chunk and row group of a gate wave
  const bool gate = wave < kGW && KT + c0 * 256 < KX;
  const int kc0 = KT + c0 * 256;
  const bool cur0 = L0 && kc0 >= KT + H;    // layer 0's current-tap chunk: x_0(t) from the draw
  f32x4 w0[kWR], x0[kUB], fw0 = {}, fb0 = {};
  bool live0 = false;
  if (gate) {
#pragma unroll
    for (int r = 0; r < kWR; ++r) w0[r] = ld4(base + (int64_t)wrow(grp * kWR + r) * KX + kc0 + lane * 4);
    live0 = load_x(kc0, x0);
    if (L0) {                               // (unconditional in the wave: no register shuffle
      const int i = (cur0 ? kc0 - KT - H : 0) + lane * 4;   //  that would drain the loads)
      fw0 = ld4(a.packed + i);
      fb0 = ld4(a.packed + a.R + i);
      live0 = live0 || cur0;
    }
  }
  // conditioning pre-activations of the epilogue lanes (gate rows 2fp, 2fp+1 x utterance fb)
  const int fp = (lane / kUB) % kRP, fb = lane % kUB;
  float pre_a = 0.f, pre_b = 0.f;
  if (wave < kGW && lane < kRP * kUB) {
    const float* pr = a.pre + ((int64_t)prow * a.B + urow(fb)) * ((int64_t)a.n_layers * a.G) + (int64_t)layer * a.G;
    const float* pt = a.ptap + (((int64_t)(slot & 1) * a.n_layers + layer) * a.B + urow(fb)) * a.G;
    pre_a = pr[wrow(2 * fp)] + pt[wrow(2 * fp)];
    pre_b = pr[wrow(2 * fp + 1)] + pt[wrow(2 * fp + 1)];
  }
  // residual waves (layer l-1's x_l(t) and skip rows): weights, biases, g, skip, residual input
  const int rx = a.R / H, nrp = rx + a.S / H;            // residual rows per gate pair
  const int lp = layer - 1;
  const float* pbase = L0 ? nullptr : layer_base(a, lp) + (int64_t)a.G * KX;
  const float* pbias = L0 ? nullptr : pbase + (int64_t)(a.R + a.S) * H;
  const int rwave = wave - kGW;
  const bool resid = !L0 && rwave >= 0;
  // after the butterfly, lane L (L % kRStep == 0) holds sum index L/kRStep = q*kUB + b
  constexpr int kRStep = 64 / (kResRows * kUB);        // lanes per reduced residual value
  const int my_q = (lane / kRStep) / kUB, my_b = (lane / kRStep) % kUB;
  const int my_gb = b0 + (my_b < nb ? my_b : 0);
  f32x4 rw[kResRows], rg[kUB];
  int myrow = 0;
  float rbias = 0.f, rskip = 0.f, rres = 0.f;
  if (resid) {
#pragma unroll
    for (int q = 0; q < kResRows; ++q) {
      int j = rwave + q * kRW;                            // residual row index in the workgroup
      if (j >= kRP * nrp) j = 0;                          // padding rows: computed and dropped
      const int p = j / nrp, jj = j - p * nrp;
      const int row = jj < rx ? (o0 + p) * rx + jj : a.R + (o0 + p) * (nrp - rx) + (jj - rx);
      rw[q] = ld4(pbase + (int64_t)row * H + lane * 4);   // H == 256: one chunk per lane
      if (q == my_q) myrow = row;
    }
#pragma unroll
    for (int b = 0; b < kUB; ++b) rg[b] = ld4(gbuf_of(a, lp) + urow(b) * H + lane * 4);
    rbias = pbias[myrow];
    // both loads issued unconditionally (a branch here made the compiler drain the loads
    // in flight before the barrier below)
    const bool xrow = myrow < a.R;
    rskip = a.skip[(int64_t)my_gb * a.S + (xrow ? 0 : myrow - a.R)];
    rres = ring_row(a, lp, slot)[(int64_t)my_gb * a.R + (xrow ? myrow : 0)];
  }
  // layer 0: the MoL head of the previous step, from the head kernel's partial sums
  // (thread b * kMaxNO + j: utterance b, output j), and the sampling noise
  float mol_v = 0.f;
  if (L0) {
    if ((int)threadIdx.x < kUB * kMaxNO) {
      const int b = threadIdx.x / kMaxNO, j = threadIdx.x % kMaxNO;
      const int jj = j < a.NO ? j : 0;
      const float* mp = a.molp + urow(b) * kMaxNO + jj;
      float part[256 / kHR];
#pragma unroll
      for (int w = 0; w < 256 / kHR; ++w) part[w] = mp[(int64_t)w * a.B * kMaxNO];
      mol_v = head_base(a)[(int64_t)a.S * a.S + a.S + (int64_t)a.NO * a.S + jj];   // b2
#pragma unroll
      for (int w = 0; w < 256 / kHR; ++w) mol_v += part[w];
    }
    if (wave == kGW + kRW - 1) {
      // the last wave has no residual rows in layer 0: it draws the noise (lane 16 b + j)
      const int t_abs = abs_step(a, targ);
      static_assert(kUB * 16 <= 64, "one noise lane per (utterance, index)");
      const int b = lane >> 4, j = lane & 15;
      if (t_abs >= 1 && b < nb && (j < a.NO / 3 || j == 10)) s_gum[lane] = mol_noise(j, t_abs - 1, a.utt_base + b0 + b, a);
    }
  }
  if (threadIdx.x == 0) s_arrived = 0;
  lds_barrier();                            // (layer >= 1: the loads above stay in flight)

  // ---------------- layer 0: sample the previous step's output; x_0(t) is its current tap
  if (L0) {
    const int t = abs_step(a, targ);
    mol_finish(a, t, wave, lane, b0, nb, mol_v, s_mol, s_gum, s_in);
    if (gate && cur0) {
#pragma unroll
      for (int b = 0; b < kUB; ++b) {
        const float in_v = s_in[b < nb ? b : 0];
        x0[b] = f32x4{in_v * fw0[0] + fb0[0], in_v * fw0[1] + fb0[1], in_v * fw0[2] + fb0[2], in_v * fw0[3] + fb0[3]};
      }
      if (blockIdx.x == 0) {                // x_0(t) into ring 0: the later taps, layer 1's inputs
        float* xr = ring_row(a, 0, slot) + (kc0 - KT - H) + lane * 4;
        for (int b = 0; b < nb; ++b) *reinterpret_cast<f32x4*>(xr + (int64_t)(b0 + b) * a.R) = x0[b];
      }
    }
  }

  // ---------------- gate GEMV (first chunk from the prologue; further chunks only when KX - KT > kGW*256)
  if (wave < kGW) {
    float acc[kWR * kUB];
#pragma unroll
    for (int j = 0; j < kWR * kUB; ++j) acc[j] = 0.f;
    if (live0) {
#pragma unroll
      for (int r = 0; r < kWR; ++r)
#pragma unroll
        for (int b = 0; b < kUB; ++b) acc[r * kUB + b] = dot4(w0[r], x0[b], acc[r * kUB + b]);
    }
    for (int c = c0 + kGC; KT + c * 256 < KX; c += kGC) {
      const int kc = KT + c * 256;
      f32x4 x[kUB];
      if (L0 && kc >= KT + H) {
        const int i = kc - KT - H + lane * 4;
        const f32x4 fw = ld4(a.packed + i), fb4 = ld4(a.packed + a.R + i);
#pragma unroll
        for (int b = 0; b < kUB; ++b) {
          const float in_v = s_in[b < nb ? b : 0];
          x[b] = f32x4{in_v * fw[0] + fb4[0], in_v * fw[1] + fb4[1], in_v * fw[2] + fb4[2], in_v * fw[3] + fb4[3]};
        }
        if (blockIdx.x == 0) {
          float* xr = ring_row(a, 0, slot) + i;
          for (int b = 0; b < nb; ++b) *reinterpret_cast<f32x4*>(xr + (int64_t)(b0 + b) * a.R) = x[b];
        }
      } else if (!load_x(kc, x)) {
        continue;
      }
#pragma unroll
      for (int r = 0; r < kWR; ++r) {
        const f32x4 w = ld4(base + (int64_t)wrow(grp * kWR + r) * KX + kc + lane * 4);
#pragma unroll
        for (int b = 0; b < kUB; ++b) acc[r * kUB + b] = dot4(w, x[b], acc[r * kUB + b]);
      }
    }
    const float s = wave_reduce_multi<kWR * kUB>(acc, lane);
    if ((lane & (64 / (kWR * kUB) - 1)) == 0) s_red[wave][lane / (64 / (kWR * kUB))] = s;
    // the last gate wave to arrive finishes the gate (no barrier with the residual waves)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int prev = 0;
    if (lane == 0) prev = atomicAdd(&s_arrived, 1);
    prev = __shfl(prev, 0);
    if (prev == kGW - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (lane < kRP * kUB && fb < nb) {
        float za = pre_a, zb = pre_b;
        // gate row r = 2 fp (+1) lives in row group r / kWR at position r % kWR
        const int ga = 2 * fp, gbr = 2 * fp + 1;
#pragma unroll
        for (int c = 0; c < kGC; ++c) {
          za += s_red[(ga / kWR) * kGC + c][(ga % kWR) * kUB + fb];
          zb += s_red[(gbr / kWR) * kGC + c][(gbr % kWR) * kUB + fb];
        }
        gbuf_of(a, layer)[(int64_t)(b0 + fb) * H + o0 + fp] = tanhf(za) * avc_sigmoid(zb);
      }
    }
  } else if (resid) {
    // layer l-1's residual rows: x_l(t) -> ring l, skip rows -> the skip accumulator
    float acc[kResRows * kUB];
#pragma unroll
    for (int q = 0; q < kResRows; ++q)
#pragma unroll
      for (int b = 0; b < kUB; ++b) acc[q * kUB + b] = dot4(rw[q], rg[b], 0.f);
    const float v0 = wave_reduce_multi<kResRows * kUB>(acc, lane);
    const int j = rwave + my_q * kRW;
    if (lane % kRStep == 0 && j < kRP * nrp && my_b < nb) {
      const int gb = b0 + my_b;
      const float v = v0 + rbias;
      if (myrow < a.R) {
        ring_row(a, layer, slot)[(int64_t)gb * a.R + myrow] = (v + rres) * kSqrtHalf;
      } else {
        float* sp = a.skip + (int64_t)gb * a.S + (myrow - a.R);
        if (lp == 0) *sp = v;
        else *sp = a.legacy ? (rskip + v) * kSqrtHalf : (rskip + v);
      }
    }
  }
}

// Past taps of the NEXT sample step: P_l(t+1) = sum_{j < K-1} W_j x_l(t+1 - (K-1-j) d_l), for
// kPR gate rows of one layer and the kBT-utterance tile.  Every input is known once the
// last layer of step t has run (x_l(t) is the newest), so the tail and head launches of
// step t carry this work in extra workgroups (layers [0, L/2) and [L/2, L)), and the 24
// chain launches of step t+1 fetch only the current-tap blocks: their per-CU operand fill
// (the launch's bound) drops from 73 to 41 KB, while these workgroups stream
// 32 rows x 4 KB of weights in large, latency-tolerant batches.  Each wave takes 128-deep
// chunks of the (K-1)*R taps on MFMA tiles (a 64-value butterfly per 8 rows took 2.5 us per
// group); the workgroup sums the waves' partials in LDS.
template <int NW>
__device__ void past_taps(const WnArgs& a, int l_lo, int idx, int slot) {
  // v_mfma_f32_16x16x4_f32 tiles: A = 16 weight rows x 4 k (lane l: row l % 16, k group
  // l / 16), B = 4 k x 16 utterance columns (8 real, 8 clamped and dropped).  Each lane
  // loads 4 consecutive k of its row / utterance; element j of those feeds MFMA j, so the
  // four MFMAs of an iteration cover 16 k (the same k order for A and B).
  static_assert(kBT == 8 && (kPR == 16 || kPR == 32 || kPR == 64), "past-tap tiling: 1-4 x 16 rows, 8 utterances");
  __shared__ float s_part[NW][kPR][kBT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rblocks = a.G / kPR;
  const int layer = l_lo + idx / rblocks;
  const int row0 = (idx % rblocks) * kPR;
  const int b0 = blockIdx.y * kBT;
  const int nb = min(kBT, a.B - b0);
  const int KT = (a.K - 1) * a.R, KX = gate_width(a);
  const int d = 1 << (layer % a.lps);
  const int sn = (slot + 1) & (a.RING - 1);           // ring slot of step t+1
  const float* base = layer_base(a, layer);
  const int m = lane & 15, q = lane >> 4;
  const int ub = b0 + ((m & 7) < nb ? (m & 7) : 0);   // utterance of B column m (8..15: dropped)
  f32x4 acc[kPRT];
#pragma unroll
  for (int r = 0; r < kPRT; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int KC = 128;                // k per wave-chunk (8 MFMA iterations of 16 k)
  for (int c = wave; c * KC < KT; c += NW) {
    const int kc = c * KC, tap = kc / a.R;
    const float* xr = ring_row(a, layer, (sn - (a.K - 1 - tap) * d) & (a.RING - 1)) + (int64_t)ub * a.R +
                      (kc - tap * a.R) + 4 * q;
    const float* w0 = base + (int64_t)(row0 + m) * KX + kc + 4 * q;
    // every load of the chunk in flight before the first MFMA: the workgroup is bound by
    // how many bytes its CU has requested, not by the MFMAs
    f32x4 xv[KC / 16], wv[kPRT][KC / 16];
#pragma unroll
    for (int it = 0; it < KC / 16; ++it) {
      xv[it] = ld4(xr + it * 16);
#pragma unroll
      for (int r = 0; r < kPRT; ++r) wv[r][it] = ld4(w0 + (int64_t)(16 * r) * KX + it * 16);
    }
    __builtin_amdgcn_sched_barrier(0);      // keep the scheduler from sinking loads to their uses
#pragma unroll
    for (int it = 0; it < KC / 16; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < kPRT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[r][it][j], xv[it][j], acc[r], 0, 0, 0);
    }
  }
  // C layout: lane l holds rows 4 (l / 16) + v (v = 0..3) of column l % 16
  if (m < kBT) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int r = 0; r < kPRT; ++r) s_part[wave][16 * r + 4 * q + v][m] = acc[r][v];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < kPR * kBT; j += 64 * NW) {
    const int r = j >> 3, b = j & 7;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += s_part[w][r][b];
    if (b < nb) a.ptap[(((int64_t)(sn & 1) * a.n_layers + layer) * a.B + b0 + b) * a.G + row0 + r] = v;
  }
}

__host__ __device__ inline int past_tap_blocks(const WnArgs& a, int n_layers_part) { return n_layers_part * (a.G / kPR); }

// tail: the last layer's skip rows, one wave per row (workgroups x < ceil(S/NW)); the
// workgroups above carry past_taps for layers [0, L/2).
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, 1))) void wn_tail_kernel(WnArgs a, int slot) {
  const int own = (a.S + NW - 1) / NW;
  if ((int)blockIdx.x >= own) {
    past_taps<NW>(a, 0, blockIdx.x - own, slot);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b0 = blockIdx.y * kBT;
  const int nb = min(kBT, a.B - b0);
  const int H = a.G / 2;
  const int lp = a.n_layers - 1;
  const int srow = min(blockIdx.x * NW + wave, a.S - 1);
  const int row = a.R + srow;
  const float* pbase = layer_base(a, lp) + (int64_t)a.G * gate_width(a);
  const float* bias = pbase + (int64_t)(a.R + a.S) * H;
  const float* gprev = gbuf_of(a, lp);
  const int bl = (lane >> 3) < nb ? (lane >> 3) : 0;
  const float bv = bias[row];
  const float sk = a.skip[(int64_t)(b0 + bl) * a.S + srow];
  float acc[kBT];
#pragma unroll
  for (int b = 0; b < kBT; ++b) acc[b] = 0.f;
  for (int k = lane * 4; k < H; k += 256) {
    const f32x4 wv = ld4(pbase + (int64_t)row * H + k);
    f32x4 g[kBT];
#pragma unroll
    for (int b = 0; b < kBT; ++b) g[b] = ld4(gprev + (int64_t)(b0 + (b < nb ? b : 0)) * H + k);
#pragma unroll
    for (int b = 0; b < kBT; ++b) acc[b] = dot4(wv, g[b], acc[b]);
  }
  const float s = wave_reduce_multi<kBT>(acc, lane);
  (void)slot;
  if ((lane & 7) != 0 || blockIdx.x * NW + wave >= a.S) return;
  const int b = lane >> 3;
  if (b >= nb) return;
  float* sp = a.skip + (int64_t)(b0 + b) * a.S + srow;
  const float v = s + bv;
  if (lp == 0) *sp = v;
  else *sp = a.legacy ? (sk + v) * kSqrtHalf : (sk + v);
}

// head: h1 = relu(W1 relu(skips) + b1), kHR rows per workgroup (kHR / NW per wave), and the
// MoL partials of those rows (layer 0 of the next step adds the S / kHR partials);
// advances the step counter; the workgroups above S / kHR carry past_taps for layers
// [L/2, L).
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, 1))) void wn_head_kernel(WnArgs a, int slot, int targ) {
  static_assert(kHR % NW == 0, "head rows per wave");
  constexpr int RPW = kHR / NW;
  __shared__ float s_h1[kHR][kBT];
  const int own = a.S / kHR;
  if ((int)blockIdx.x >= own) {
    past_taps<NW>(a, a.n_layers / 2, blockIdx.x - own, slot);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b0 = blockIdx.y * kBT;
  const int nb = min(kBT, a.B - b0);
  const int row0 = blockIdx.x * kHR;
  const float* W1 = head_base(a);
  const float* b1 = W1 + (int64_t)a.S * a.S;
  const float* W2 = b1 + a.S;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) a.ctr[0] = abs_step(a, targ) + 1;
  // relu(skip) of the utterance tile, one 4-float chunk per lane (S == 256)
  f32x4 x[kBT];
#pragma unroll
  for (int b = 0; b < kBT; ++b) {
    x[b] = ld4(a.skip + (int64_t)(b0 + (b < nb ? b : 0)) * a.S + lane * 4);
    x[b][0] = fmaxf(x[b][0], 0.f); x[b][1] = fmaxf(x[b][1], 0.f);
    x[b][2] = fmaxf(x[b][2], 0.f); x[b][3] = fmaxf(x[b][3], 0.f);
  }
  f32x4 wv[RPW];
  float bv[RPW];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row0 + wave * RPW + q;
    wv[q] = ld4(W1 + (int64_t)row * a.S + lane * 4);
    bv[q] = b1[row];
  }
  // the MoL partial operands: thread t < NO * kBT takes output j = t / kBT, utterance t % kBT
  const int mj = min((int)threadIdx.x / kBT, a.NO - 1), mb = threadIdx.x % kBT;
  float w2[kHR];
#pragma unroll
  for (int r = 0; r < kHR; ++r) w2[r] = W2[(int64_t)mj * a.S + row0 + r];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    float acc[kBT];
#pragma unroll
    for (int b = 0; b < kBT; ++b) acc[b] = dot4(wv[q], x[b], 0.f);
    const float s = wave_reduce_multi<kBT>(acc, lane);
    if ((lane & 7) == 0) {
      const int b = lane >> 3;
      const float h = fmaxf(s + bv[q], 0.f);
      s_h1[wave * RPW + q][b] = h;
      if (b < nb) a.h1[(int64_t)(b0 + b) * a.S + row0 + wave * RPW + q] = h;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < a.NO * kBT && mb < nb) {
    float p = 0.f;
#pragma unroll
    for (int r = 0; r < kHR; ++r) p += w2[r] * s_h1[r][mb];
    a.molp[((int64_t)blockIdx.x * a.B + b0 + mb) * kMaxNO + mj] = p;
  }
  (void)slot;
}

// Sample the last output (step T-1) after the final head.
__global__ __launch_bounds__(256) void wn_final_sample_kernel(WnArgs a, int tp1) {
  __shared__ float s_mol[kBT * kMaxNO];
  const int b0 = blockIdx.y * kBT;
  sample_stage<4, kBT>(a, tp1, b0, min(kBT, a.B - b0), s_mol, nullptr);
}

__global__ void wn_set_ctr_kernel(int* ctr, int t) { ctr[0] = t; }

// ---- upsample network: 4 x [ConvTranspose2d(1,1,(3,s),stride (1,s),pad (1,0)) + ReLU]
// One workgroup per (utterance, conditioning frame): time never mixes across frames
// (kernel == stride), so every stage of a frame stays in LDS; the last stage writes the
// time-major (T, B, C) conditioning the GEMM consumes.
constexpr int kUpMaxStages = 8;
struct UpArgs {
  int B, Tc, C, n, P;
  int s[kUpMaxStages];
  int woff[kUpMaxStages];
};

__global__ __launch_bounds__(256) void wn_upsample_kernel(UpArgs u, const float* __restrict__ c,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out) {
  extern __shared__ float lds[];
  const int frame = blockIdx.x, b = blockIdx.y;
  const int prev_max = u.P / u.s[u.n - 1];
  float* buf0 = lds;
  float* buf1 = lds + u.C * prev_max;
  for (int f = threadIdx.x; f < u.C; f += blockDim.x) buf0[f] = c[((int64_t)b * u.C + f) * u.Tc + frame];
  __syncthreads();
  int n_in = 1;
  float* in = buf0;
  float* nxt = buf1;
  for (int st = 0; st < u.n; ++st) {
    const int s = u.s[st];
    const float* ws = w + u.woff[st];  // [3][s]
    const float bs = bias[st];
    const int n_out = n_in * s;
    const bool last = st == u.n - 1;
    for (int e = threadIdx.x; e < u.C * n_out; e += blockDim.x) {
      const int f = e % u.C, q = e / u.C;   // q: position within the frame
      const int p = q / s, j = q - p * s;
      float acc = bs;
      // out[f] = sum_k w[k][j] in[f + 1 - k]
      if (f + 1 < u.C) acc += ws[j] * in[p * u.C + f + 1];
      acc += ws[s + j] * in[p * u.C + f];
      if (f >= 1) acc += ws[2 * s + j] * in[p * u.C + f - 1];
      acc = fmaxf(acc, 0.f);
      if (last) out[(((int64_t)frame * u.P + q) * u.B + b) * u.C + f] = acc;
      else nxt[q * u.C + f] = acc;
    }
    __syncthreads();
    float* tmp = in; in = nxt; nxt = tmp;
    n_in = n_out;
  }
}

// ================================================================ persistent generation helpers
__device__ int g_wn_fault = 0;         // sticky: a persistent generation timed out (autovc_wavenet_fault)

// A wave-uniform base pointer forced into SGPRs: a buffer descriptor built from a value the
// compiler keeps in VGPRs (e.g. live across divergent code) otherwise becomes a waterfall loop
// around every load.  A no-op for a base already in SGPRs.
__device__ __forceinline__ float* wave_uniform(const float* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ f32x4 ld4_l2(const float* base, int off) {
  // an L1-bypassing (sc1) 16-byte load of data another workgroup of this XCD wrote: `base` is
  // wave-uniform (the descriptor lives in SGPRs; a per-lane base would make the compiler
  // loop over the lanes), `off` the lane's float offset
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(base), (short)0, 0x7fffffff,
                                                                     0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)off * 4u, 0, 16));
}

__device__ __forceinline__ f32x4 ld4_ro(const float* base, int off) {
  // a 16-byte load of read-only weights through a wave-uniform buffer descriptor
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(base), (short)0, 0x7fffffff,
                                                                     0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)off * 4u, 0, 0));
}

// ================================================================ all-CU weight-resident generation
// (B <= 8, the r9y9 shapes R = 512, G = 512, S = 256, 3 taps, 8..24 layers).  ONE persistent
// launch per autovc_wavenet_generate_f32 call; its 256 workgroups (one per CU) run the 26
// phases of every sample step (layers 0..L-1, the last layer's skip rows, h1) as a DATAFLOW:
// no grid barrier, every hand-off is a tagged 16-byte granule.  Workgroup o owns gate pair
// (o, o + H), residual rows 2o, 2o + 1 (x_(l+1)) and skip row o of every layer, and head row
// o, and publishes per phase and utterance exactly ONE granule {g_l[o], x_l[2o], x_l[2o+1],
// tag} (x_l = layer l's input, computed in phase l from layer l-1's output) with one sc1
// (write-through) store; the tag is the step + 1, so a consumer knows a granule is this step's
// by reading it (16-byte sc1 stores are observed untorn on gfx950 / ROCm 7.2, MI355X_MICROARCH
// "Valid forms").  The next phase's inputs [g_l | x_l] are exactly the 256 granules of the
// previous phase (4 KB per utterance): chain lane o (waves 0-3) polls granule o of every
// utterance with sc1 loads until all tags match — the store and its observation replace the
// barrier's vmcnt drain, two atomic round trips and the release broadcast.
//   weights: the gate rows of every layer resident in LDS ([l][o][6]: the 3 weights of gate
//   rows o_s and o_s + H that meet granule o, 147 KB at 24 layers); the 3 residual weights a
//   lane needs for the next phase (W_out rows 2o_s, 2o_s + 1 and W_skip row o_s at column o)
//   and W2 are loaded into registers before the lane starts polling, so their fetch hides
//   under the wait for the producers.
// Lane o multiplies its granule into 5 partial sums per utterance (2 gate rows, 3 residual
// rows); a wave butterfly and an LDS counter handshake among the 4 chain waves leave the sums
// to wave 0, whose lanes b < B run the cell update and publish.  The past taps of the next step
// (W_0 x_l(t+1-2d) + W_1 x_l(t+1-d): 48 MB of weights per step, too many to hold) are computed
// by waves 4..7 of workgroup o (up to 4 16-row blocks of layer o % L) on MFMA as soon as their
// inputs are published, into 8-byte {value, tag} granules the chain lane polls; they never
// synchronise with the chain waves.  The sample of step t-1 is drawn by every workgroup itself
// at the start of step t (the same Philox stream, the same value everywhere).  A wait that times
// out (the 256 workgroups were not all resident) sets an error word every other wait checks,
// and the call's samples are poisoned with NaN and bit 2 of autovc_wavenet_fault is set.
constexpr int kGrW = 8;                       // waves per workgroup: 4 chain + 4 past-tap
constexpr int kGMaxL = 24;
constexpr int kGMaxB = 8;
constexpr int kGFault = 2;
constexpr int kGErrInts = 32;                 // the error word's line (ints)

struct GLds {                                 // float offsets into the dynamic LDS block
  int gw, h1, molp, mol, gum, in, part, xres, cnt, total;
};
__host__ __device__ inline GLds g_lds(int L, int NO) {
  (void)NO;
  GLds o;
  int p = 0;
  o.gw = p;    p += L * 256 * 6;              // gate weights [l][o][6]
  o.h1 = p;    p += kGMaxB * 256;             // h1 of the previous step [b][o] (the MoL GEMV's input)
  o.molp = p;  p += 4 * 32 * kGMaxB;          // per-wave MoL partials [wave][j][b]
  o.mol = p;   p += kGMaxB * 32;              // MoL parameters [b][j]
  o.gum = p;   p += kGMaxB * 16;              // sampling noise [b][j]
  o.in = p;    p += kGMaxB;                   // this step's input sample per utterance
  // per-wave partial sums of a phase [parity][wave][value] and x_(l-1)[2o_s], [2o_s + 1] per
  // utterance [parity][b][2]: double-buffered by phase, since a chain wave may enter the next
  // phase (its inputs come from other workgroups) while wave 0 still reads this one's
  o.part = p;  p += 2 * 4 * 64;
  o.xres = p;  p += 2 * kGMaxB * 2;
  o.cnt = p;   p += 4;                        // the chain waves' LDS handshake counter
  o.total = p;
  return o;
}

__host__ __device__ inline int64_t g_ring_f4(const WnArgs& a) {   // granules of the tagged ring
  return (int64_t)a.n_layers * a.RING * a.B * 256;
}

// NOTE: __float_as_int, not __builtin_bit_cast: this clang lowers a bit_cast of an ext-vector
// ELEMENT (g[3]) as a read of element 0 (the vector's address), which made every poll compare
// the granule's first word against the tag
__device__ __forceinline__ int tag_of(f32x4 g) { return __float_as_int(g[3]); }

// one 16-byte write-through (sc1) store {v0, v1, v2, tag} at base + off floats; `base` is
// wave-uniform (the descriptor lives in SGPRs)
__device__ __forceinline__ void st4_sc1(float* base, int off, float v0, float v1, float v2, int tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(base), (short)0, 0x7fffffff, 0x00020000);
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 w = {__float_as_int(v0), __float_as_int(v1), __float_as_int(v2), tag};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (uint32_t)off * 4u, 0, 16);
}
// 8-byte {value, tag} granule, write-through
__device__ __forceinline__ void st2t_sc1(float* base, int off, float v, int tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(base), (short)0, 0x7fffffff, 0x00020000);
  typedef int i32x2 __attribute__((ext_vector_type(2)));
  const i32x2 w = {__float_as_int(v), tag};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (uint32_t)off * 4u, 0, 16);
}
__device__ __forceinline__ float2 ld2_l2(const float* base, int off) {   // sc1 8-byte load
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(base), (short)0, 0x7fffffff,
                                                                     0x00020000);
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)off * 4u, 0, 16));
  return make_float2(v[0], v[1]);
}

// Which wait of wn_grid_kernel timed out first: {wait kind, step, phase or job, workgroup}
// (autovc_wavenet_grid_diag reads and clears it).  Kinds: 1 layer inputs, 2 past-tap sums,
// 3 the chain waves' LDS handshake, 4 past-tap inputs, 5 past-tap consumers, 6 skip sums, 7 h1.
__device__ int g_wn_grid_diag[5] = {};

// bounded spin state of one wave: the deadline, the device-wide error word, what it waits for
struct Spin {
  uint64_t t0;
  int* err;
  int ticks;
  int kind, step, ph;
  int seen = -1;                              // the tag last observed (diagnostics)
  bool slow = false;                          // off the critical path: long sleeps, every check
  int n = 0;
  int chk = 3;                                // the error word and the clock every (chk + 1)th retry
  __device__ bool tick() {                    // false: give up (timed out, or another wave did)
    if (!slow && (++n & chk) != 0) {
      __builtin_amdgcn_s_sleep(1);
      return true;
    }
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)ticks) {
      int z = 0;
      if (__hip_atomic_compare_exchange_strong(err, &z, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(&g_wn_grid_diag[1], step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&g_wn_grid_diag[2], ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&g_wn_grid_diag[3], (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&g_wn_grid_diag[4], seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&g_wn_grid_diag[0], kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return false;
    }
    if (slow) __builtin_amdgcn_s_sleep(32);   // ~2k clocks: a waiting past-tap wave costs the fabric little
    else __builtin_amdgcn_s_sleep(1);
    return true;
  }
};

// LDS handshake of the 4 chain waves: each wave's LDS writes are complete before its lane 0
// adds to the counter; every wave then waits for the k-th round (4 k arrivals).  Bounded: a
// wave that gave up elsewhere never arrives, and the device error word then ends the wait.
__device__ __forceinline__ bool chain_sync(int* cnt, int& k, int lane, int* err, int ticks, int step, int ph) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int want = 4 * ++k;
  Spin sp{__builtin_amdgcn_s_memrealtime(), err, ticks, 3, step, ph};
  int n = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
    if ((++n & 255) == 0 && !sp.tick()) return false;
  asm volatile("" ::: "memory");
  return true;
}

// Poll the NB granules of lane o (utterance slots b: base + ((b < B ? b : 0) * 256 + o) * 4
// floats) until every lane of the wave holds this step's tag.  false: the wait gave up.
template <int NB>
__device__ __forceinline__ bool poll_granules(const float* base, int o, int B, int tag, f32x4 (&g)[NB], int* err,
                                              int ticks, int kind, int ph) {
  Spin sp{__builtin_amdgcn_s_memrealtime(), err, ticks, kind, tag - 1, ph};
  if constexpr (NB > 1) {
    // poll utterance 0's granule alone: the producer lane group publishes every utterance's
    // granule with one store instruction, so the rest are out (almost always) once it is, and
    // the waiting costs the fabric one 16-byte load per lane per retry instead of NB
    while (true) {
      asm volatile("" ::: "memory");
      g[0] = ld4_l2(base, o * 4);
      if (__builtin_amdgcn_ballot_w64(tag_of(g[0]) != tag) == 0) break;
      sp.seen = __builtin_amdgcn_readfirstlane(tag_of(g[0]));
      if (!sp.tick()) return false;
    }
  }
  while (true) {
    // every retry re-issues every load (the clobber keeps the compiler from reusing a value
    // loaded in an earlier pass), and all of them are in flight before the first compare; a
    // retry of only the late granules costs phi copies of all NB granules (spills at NB = 8)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int b = 0; b < NB; ++b) g[b] = ld4_l2(base, ((b < B ? b : 0) * 256 + o) * 4);
    int bad = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b) bad |= tag_of(g[b]) ^ tag;
    if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) return true;
    sp.seen = __builtin_amdgcn_readfirstlane(tag_of(g[0]));
    if (!sp.tick()) return false;
  }
}

// One 128-deep chunk kc (tap kc / 4, k0 = 128 (kc % 4)) of the past taps of step `job` for the
// 16 gate rows of block blk of layer lp on v_mfma_f32_16x16x4_f32 tiles (past_taps' operand
// map: lane l feeds weight row l % 16 / utterance column l % 16 with 4 consecutive k of group
// l / 16).  The x inputs come from the tagged ring: x_lp(s)[k] is component 1 + (k & 1) of
// granule k / 2; steps s < 0 are zero.  false: a wait gave up.
__device__ __forceinline__ bool wn_grid_past_tap_chunk(const WnArgs& a, int lp, int blk, int d, int job, int kc,
                                                       int lane, f32x4& pacc, int* err, int ticks) {
  constexpr int R = 512, KX = 3 * 512 + 256;
  const int m = lane & 15, q = lane >> 4;
  const int tap = kc >> 2, k0 = (kc & 3) * 128;
  const int s = job - (2 - tap) * d;
  const int ub = (m & 7) < a.B ? (m & 7) : 0;
  const float* w0 = layer_base(a, lp) + (int64_t)(blk * 16 + m) * KX + tap * R + k0 + 4 * q;
  f32x4 acc = pacc;
  if (s >= 0) {
    const float* xr = a.gring + ((int64_t)lp * a.RING + (s & (a.RING - 1))) * a.B * 256 * 4;   // wave-uniform
#pragma unroll
    for (int h = 0; h < 8; h += 4) {          // four 16-deep steps in flight
      f32x4 wv[4], xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = ld4(w0 + (h + i) * 16);
      Spin sp{__builtin_amdgcn_s_memrealtime(), err, ticks, 4, job, kc};
      while (true) {
        asm volatile("" ::: "memory");       // re-issue every load on a retry (see poll_granules)
        f32x4 ga[4], gb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o2 = (k0 + (h + i) * 16 + 4 * q) / 2;        // granules o2, o2 + 1
          ga[i] = ld4_l2(xr, (ub * 256 + o2) * 4);
          gb[i] = ld4_l2(xr, (ub * 256 + o2) * 4 + 4);
        }
        int bad = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bad |= (tag_of(ga[i]) ^ (s + 1)) | (tag_of(gb[i]) ^ (s + 1));
          xv[i] = f32x4{ga[i][1], ga[i][2], gb[i][1], gb[i][2]};
        }
        if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) break;
        sp.seen = __builtin_amdgcn_readfirstlane(tag_of(ga[0]));
        if (!sp.tick()) return false;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[i][j], xv[i][j], acc, 0, 0, 0);
    }
  }
  pacc = acc;
  return true;
}


// NB: utterance slots of the launch (1, 2, 4 or 8 >= B; slots >= B compute on utterance 0
// and are dropped), so every per-utterance loop is straight-line code
template <int NB>
__global__ __launch_bounds__(64 * kGrW, 1) void wn_grid_kernel(WnArgs a, int t0, int t1, int* errw, int ticks) {
  // no mul-add contraction: the NB instantiations (1, 2, 4, 8 utterance slots) must round every
  // utterance's arithmetic the same way (batch invariance: an utterance's samples do not depend
  // on the batch it was generated in)
#pragma clang fp contract(off)
  constexpr int R = 512, H = 256, S = 256, KX = 3 * 512 + 256, KT = 2 * 512;
  constexpr int NV = 5 * NB <= 8 ? 8 : 5 * NB <= 16 ? 16 : 5 * NB <= 32 ? 32 : 64;   // partials, padded
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int L = a.n_layers, B = a.B, T = a.T, RING = a.RING, NO = a.NO;
  const GLds lo = g_lds(L, NO);
  float* s_gw = lds + lo.gw;
  float* s_h1 = lds + lo.h1;
  float* s_molp = lds + lo.molp;
  float* s_mol = lds + lo.mol;
  float* s_gum = lds + lo.gum;
  float* s_in = lds + lo.in;
  float* s_part = lds + lo.part;
  float* s_xres = lds + lo.xres;
  int* s_cnt = reinterpret_cast<int*>(lds + lo.cnt);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int os = blockIdx.x;                  // this workgroup's gate pair / residual pair / skip and head row
  const float* W1 = head_base(a);
  const float* b1 = W1 + (int64_t)S * S;
  const float* W2 = b1 + S;
  const float* b2 = W2 + (int64_t)NO * S;
  const int64_t RB4 = (int64_t)B * 256 * 4;   // floats of one ring slot (all utterances)

  // ---- resident gate weights: s_gw[l][o][r * 3 + {g, x0, x1}] = W(o_s + r H)[KT + o], [KT + H + 2o], [.. + 1]
  for (int e = tid; e < L * 256; e += 64 * kGrW) {
    const int l = e / 256, o = e % 256;
    const float* base = layer_base(a, l) + KT;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float* w = base + (int64_t)(os + r * H) * KX;
      s_gw[e * 6 + 3 * r] = w[o];
      s_gw[e * 6 + 3 * r + 1] = w[H + 2 * o];
      s_gw[e * 6 + 3 * r + 2] = w[H + 2 * o + 1];
    }
  }
  if (tid == 0) *s_cnt = 0;
  // The polls are sc1 loads: drop any line of the hand-off region an earlier kernel's plain
  // access left in this XCD's L2 (system-scope acquire = buffer_inv sc0 sc1) before the first.
  if (tid < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();

  if (wave >= 4) {
    // =========================== past-tap waves: blocks of layer lp = os % L
    const int lp = os % L, pk = os / L, pn = (int)((gridDim.x - lp + L - 1) / L);
    constexpr int kPTB = 512 / 16;            // 16-row blocks per layer (G = 512)
    const int pnb = pk < kPTB ? (kPTB - pk + pn - 1) / pn : 0;
    const int pw = wave - 4;
    if (pw >= pnb) return;
    const int blk = pk + pn * pw, d = 1 << (lp % a.lps);
    const int m = lane & 15, q = lane >> 4;
    for (int job = t0 + 1; job <= t1; ++job) {
      if (job >= T) break;                    // P(T) feeds no step
      // wait (slowly: P(job) is needed a whole step later) until the owners of these rows
      // (rows r and r - H -> workgroup r mod H) have published layer lp of step job - 1: they
      // are past P(job - 2), whose parity this job overwrites, and x_lp(job - 1) — the d = 1
      // layers' newest input — is out
      if (job - 1 >= 0) {
        const int owner = (blk * 16 + (lane & 15)) & (H - 1);
        const float* xr = a.gring + ((int64_t)lp * RING + ((job - 1) & (RING - 1))) * RB4;
        Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 5, job, lp};
        sp.slow = true;
        while (true) {
          asm volatile("" ::: "memory");
          const int tg = tag_of(ld4_l2(xr, 4 * owner));
          if (__builtin_amdgcn_ballot_w64(tg != job) == 0) break;
          sp.seen = __builtin_amdgcn_readfirstlane(tg);
          if (!sp.tick()) return;
        }
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int kc = 0; kc < 8; ++kc)
        if (!wn_grid_past_tap_chunk(a, lp, blk, d, job, kc, lane, acc, errw, ticks)) return;
      if (m < B) {
        float* pt = a.gpt + ((int64_t)(job & 1) * L + lp) * B * 512 * 2;      // wave-uniform
#pragma unroll
        for (int v = 0; v < 4; ++v) st2t_sc1(pt, m * 1024 + 2 * (blk * 16 + 4 * q + v), acc[v], job + 1);
      }
    }
    return;
  }

  // =========================== chain waves 0-3: lane o = granule o
  const int o = wave * 64 + lane;
  int kx = 0;                                 // chain_sync rounds
  int cur_t = t0, cur_p = 0;                  // (diagnostics of a timed-out wait)
  bool ok = true;
  // first_conv weights of channels 2o, 2o + 1 (layer 0's x inputs) and of 2 os, 2 os + 1
  const float fw0 = a.packed[2 * o], fw1 = a.packed[2 * o + 1], fb0 = a.packed[R + 2 * o], fb1 = a.packed[R + 2 * o + 1];
  const float fwo0 = a.packed[2 * os], fwo1 = a.packed[2 * os + 1], fbo0 = a.packed[R + 2 * os],
              fbo1 = a.packed[R + 2 * os + 1];
  const float w1o = W1[(int64_t)os * S + o], b1o = b1[os];
  // the last layer's skip bias of row os (the tail's epilogue: loaded once, off the chain)
  const float bsk_last = (layer_base(a, L - 1) + (int64_t)a.G * KX + (int64_t)(R + S) * H)[R + os];
  // residual weights of layer lr at column o: W_out rows 2 os, 2 os + 1, W_skip row os
  float rw0 = 0.f, rw1 = 0.f, rw2 = 0.f;
  auto fetch_res = [&](int lr) {
    const float* pb = layer_base(a, lr) + (int64_t)a.G * KX;
    rw0 = pb[(int64_t)(2 * os) * H + o];
    rw1 = pb[(int64_t)(2 * os + 1) * H + o];
    rw2 = pb[(int64_t)(R + os) * H + o];
  };
  // W2 for the MoL GEMV: lane (j = lane % 32, 32-deep k slice 2 wave + lane / 32)
  const int mj = lane & 31, mks = 2 * wave + (lane >> 5);
  f32x4 w2r[8];
  auto fetch_w2 = [&]() {
    const int jj = mj < NO ? mj : 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w2r[i] = ld4(W2 + (int64_t)jj * S + 32 * mks + 4 * i);
  };
  auto noise = [&](int tp) {                  // wave 3: lane 16 (b % 4) + j, utterances 0..3 then 4..7
    if (wave != 3 || tp < 0) return;
    for (int half = 0; half < 2; ++half) {
      const int b = 4 * half + (lane >> 4), j = lane & 15;
      if (b < B && (j < NO / 3 || j == 10)) s_gum[b * 16 + j] = mol_noise(j, tp, a.utt_base + b, a);
    }
  };
  // butterfly the partial sums of this wave, park them in s_part[wave][j], then hand them to
  // wave 0 (every chain wave joins the handshake)
  int par = 0;                                // phase parity: s_part / s_xres buffer
  auto reduce_park = [&](float (&acc)[NV]) {
    if constexpr (NV == 64) {
      // 8 utterances: the 5 partial groups one butterfly of 8 each (50 shuffles, 8 live
      // copies instead of 64); the same pairing tree per value as the single butterfly
#pragma unroll
      for (int g = 0; g < 5; ++g) {
        float cur[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = acc[g * 8 + j];
        butterfly_hw<8, 0>(cur, lane);
        if ((lane & 7) == 0) s_part[par * 256 + wave * 64 + g * 8 + (lane >> 3)] = cur[0];
      }
    } else {
      const float v = wave_reduce_hw<NV>(acc, lane);
      if ((lane & (64 / NV - 1)) == 0) s_part[par * 256 + wave * 64 + lane / (64 / NV)] = v;
    }
    return chain_sync(s_cnt, kx, lane, errw, ticks, cur_t, cur_p);
  };
  auto psum = [&](int j) {
    const float* sp = s_part + par * 256;
    return ((sp[j] + sp[64 + j]) + sp[128 + j]) + sp[192 + j];
  };

  noise(t0 - 1);
  float skip_acc = 0.f;                       // epilogue lane b: the skip sum of utterance b
  for (int t = t0; t < t1 && ok; ++t) {
    const int ts = t & (RING - 1), prow = t % a.Tch;
    for (int p = 0; p < L + 2 && ok; ++p, par ^= 1) {
      cur_t = t;
      cur_p = p;
      float acc[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) acc[j] = 0.f;
      if (p < L) {
        const int l = p;
        // epilogue operands of lane b (wave 0): conditioning + past taps of the gate pair, the
        // residual biases of layer l-1
        float pre_a = 0.f, pre_b = 0.f, bias0 = 0.f, bias1 = 0.f, bias2 = 0.f;
        if (wave == 0 && lane < B) {
          const float* pr = a.pre + ((int64_t)prow * B + lane) * ((int64_t)L * a.G) + (int64_t)l * a.G;
          pre_a = pr[os];
          pre_b = pr[os + H];
          if (l >= 1) {
            const float* pbias = layer_base(a, l - 1) + (int64_t)a.G * KX + (int64_t)(R + S) * H;
            bias0 = pbias[2 * os]; bias1 = pbias[2 * os + 1]; bias2 = pbias[R + os];
          }
        }
        // this phase's past-tap sums (rows o_s, o_s + H), computed a step ahead by the past-tap
        // waves: their loads go out now, so the round trip hides under the input wait
        const float* ptl = a.gpt + ((int64_t)(t & 1) * L + l) * B * 512 * 2;   // wave-uniform
        float2 pva = make_float2(0.f, 0.f), pvb = make_float2(0.f, 0.f);
        if (wave == 0 && lane < B && t > 0) {
          pva = ld2_l2(ptl, lane * 1024 + 2 * os);
          pvb = ld2_l2(ptl, lane * 1024 + 2 * (os + H));
        }
        const float* wgl = s_gw + ((int64_t)l * 256 + o) * 6;
        if (l == 0) {
          // ---- the MoL parameters of step t-1 from its h1, then the draw (every workgroup)
          const int tp = t - 1;
          if (tp >= 0) {
            fetch_w2();                       // in flight during the h1 wait; live in this phase only
            f32x4 gh[NB];
            if (!poll_granules<NB>(a.gh1, o, B, tp + 1, gh, errw, ticks, 7, 0)) { ok = false; break; }
#pragma unroll
            for (int b = 0; b < NB; ++b) s_h1[b * 256 + o] = gh[b][0];
            if (!chain_sync(s_cnt, kx, lane, errw, ticks, t, 0)) { ok = false; break; }
            float am[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
              asm volatile("" ::: "memory");  // one utterance's 8 LDS reads in flight at a time (registers)
              am[b] = 0.f;
              const float* hb = s_h1 + b * 256 + 32 * mks;
#pragma unroll
              for (int i = 0; i < 8; ++i) am[b] = dot4(w2r[i], *reinterpret_cast<const f32x4*>(hb + 4 * i), am[b]);
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {   // + lane l ^ 32 (v_permlane32_swap, no LDS round trip)
              const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(am[b]), __float_as_uint(am[b]), false, false);
              am[b] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
            }
            if (lane < 32)
#pragma unroll
              for (int b = 0; b < NB; ++b) s_molp[(wave * 32 + lane) * kGMaxB + b] = am[b];
            if (!chain_sync(s_cnt, kx, lane, errw, ticks, t, 0)) { ok = false; break; }
            if (o < B * 32) {                 // thread (b, j)
              const int b = o >> 5, jj = o & 31;
              if (jj < NO)
                s_mol[b * 32 + jj] = b2[jj] + (((s_molp[(0 * 32 + jj) * kGMaxB + b] + s_molp[(1 * 32 + jj) * kGMaxB + b]) +
                                                s_molp[(2 * 32 + jj) * kGMaxB + b]) +
                                               s_molp[(3 * 32 + jj) * kGMaxB + b]);
            }
            if (!chain_sync(s_cnt, kx, lane, errw, ticks, t, 0)) { ok = false; break; }
          }
          if (wave < 2) {
            // the mixture pick on 16 lanes per utterance (mol_finish's order and tie rule)
            const int b = 4 * wave + (lane >> 4), j = lane & 15, nr = NO / 3;
            float v = -INFINITY;
            if (tp >= 0 && b < B && j < nr) {
              v = s_mol[b * 32 + j] - s_gum[b * 16 + j];
              if (!(v == v)) v = -INFINITY;
            }
            int bi = j;
#pragma unroll
            for (int mm = 8; mm >= 1; mm >>= 1) {
              const float ov = __shfl_xor(v, mm);
              const int oi = __shfl_xor(bi, mm);
              if (ov > v || (ov == v && oi < bi)) { v = ov; bi = oi; }
            }
            if (j == 0 && b < B) {
              float in_v = 0.f, smp = 0.f;
              if (tp >= 0) {
                const float mean = s_mol[b * 32 + nr + bi];
                const float ls = fmaxf(s_mol[b * 32 + 2 * nr + bi], a.log_scale_min);
                const float x = mean + expf(ls) * s_gum[b * 16 + 10];
                smp = fminf(fmaxf(x, -1.0f), 1.0f);
              }
              if (a.teacher != nullptr && t < a.teacher_len) in_v = a.teacher[(int64_t)b * a.teacher_len + t];
              else if (tp >= 0) in_v = smp;
              s_in[b] = in_v;
              if (os == 0) {
                a.yin[(int64_t)b * T + t] = in_v;
                if (tp >= 0) {
                  a.y_out[(int64_t)b * T + tp] = smp;
                  if (a.mol_out)
                    for (int qq = 0; qq < NO; ++qq) a.mol_out[((int64_t)b * T + tp) * NO + qq] = s_mol[b * 32 + qq];
                }
              }
            }
          }
          if (!chain_sync(s_cnt, kx, lane, errw, ticks, t, 0)) { ok = false; break; }
          // x_0(t)[2o], [2o + 1] = first_conv(input): the gate's x inputs; no g block
          const float wa1 = wgl[1], wa2 = wgl[2], wb1 = wgl[4], wb2 = wgl[5];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const float in_v = s_in[b];
            const float x0 = in_v * fw0 + fb0, x1 = in_v * fw1 + fb1;
            acc[b] = wa1 * x0 + wa2 * x1;
            acc[NB + b] = wb1 * x0 + wb2 * x1;
          }
        } else {
          // ---- this step's granules of layer l-1: [g_(l-1)[o] | x_(l-1)[2o], [2o + 1]]
          f32x4 gin[NB];
          if (!poll_granules<NB>(a.gring + ((int64_t)(l - 1) * RING + ts) * RB4, o, B, t + 1, gin, errw, ticks, 1, l)) {
            ok = false;
            break;
          }
          const float wa0 = wgl[0], wa1 = wgl[1], wa2 = wgl[2], wb0 = wgl[3], wb1 = wgl[4], wb2 = wgl[5];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const float g = gin[b][0], x0 = gin[b][1], x1 = gin[b][2];
            acc[b] = (wa0 * g + wa1 * x0) + wa2 * x1;
            acc[NB + b] = (wb0 * g + wb1 * x0) + wb2 * x1;
            acc[2 * NB + b] = rw0 * g;
            acc[3 * NB + b] = rw1 * g;
            acc[4 * NB + b] = rw2 * g;
          }
          if (o == os)
#pragma unroll
            for (int b = 0; b < NB; ++b) {
              s_xres[par * 2 * kGMaxB + 2 * b] = gin[b][1];
              s_xres[par * 2 * kGMaxB + 2 * b + 1] = gin[b][2];
            }
        }
        // the next phase's residual weights (layer l) fetched while the epilogue and the
        // producers run
        fetch_res(l);
        if (!reduce_park(acc)) { ok = false; break; }
        if (wave == 0 && lane < B) {
          const int b = lane;
          float pta = 0.f, ptb = 0.f;
          if (t > 0) {                        // P(0) = 0 (every past input is zero)
            Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 2, t, l};
            while (__float_as_int(pva.y) != t + 1 || __float_as_int(pvb.y) != t + 1) {   // rarely: not yet out
              if (!sp.tick()) { ok = false; break; }
              asm volatile("" ::: "memory");
              pva = ld2_l2(ptl, b * 1024 + 2 * os);
              pvb = ld2_l2(ptl, b * 1024 + 2 * (os + H));
            }
            pta = pva.x;
            ptb = pvb.x;
          }
          const float za = psum(b) + (pre_a + pta), zb = psum(NB + b) + (pre_b + ptb);
          const float gv = tanhf(za) * avc_sigmoid(zb);
          float x0n, x1n;
          if (l == 0) {
            const float in_v = s_in[b];
            x0n = in_v * fwo0 + fbo0;
            x1n = in_v * fwo1 + fbo1;
          } else {
            x0n = (psum(2 * NB + b) + bias0 + s_xres[par * 2 * kGMaxB + 2 * b]) * kSqrtHalf;
            x1n = (psum(3 * NB + b) + bias1 + s_xres[par * 2 * kGMaxB + 2 * b + 1]) * kSqrtHalf;
            const float sv = psum(4 * NB + b) + bias2;
            skip_acc = l - 1 == 0 ? sv : (a.legacy ? (skip_acc + sv) * kSqrtHalf : skip_acc + sv);
          }
          st4_sc1(a.gring + ((int64_t)l * RING + ts) * RB4, (b * 256 + os) * 4, gv, x0n, x1n, t + 1);
        }
        ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
      } else if (p == L) {
        // ---- tail: the last layer's skip row os; wave 3 then draws the next sample's noise
        f32x4 gin[NB];
        if (!poll_granules<NB>(a.gring + ((int64_t)(L - 1) * RING + ts) * RB4, o, B, t + 1, gin, errw, ticks, 1, L)) {
          ok = false;
          break;
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = rw2 * gin[b][0];
        if (!reduce_park(acc)) { ok = false; break; }
        if (wave == 0 && lane < B) {
          const float sv = psum(lane) + bsk_last;
          const float sk = L - 1 == 0 ? sv : (a.legacy ? (skip_acc + sv) * kSqrtHalf : skip_acc + sv);
          st4_sc1(a.gsk, (lane * 256 + os) * 4, sk, 0.f, 0.f, t + 1);
        }
        noise(t);
      } else {
        // ---- head: h1 row os = relu(W1[os] relu(skip) + b1[os])
        f32x4 gs[NB];
        if (!poll_granules<NB>(a.gsk, o, B, t + 1, gs, errw, ticks, 6, L + 1)) { ok = false; break; }
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = w1o * fmaxf(gs[b][0], 0.f);
        if (!reduce_park(acc)) { ok = false; break; }
        if (wave == 0 && lane < B) {
          const float h = fmaxf(psum(lane) + b1o, 0.f);
          st4_sc1(a.gh1, (lane * 256 + os) * 4, h, 0.f, 0.f, t + 1);
          a.h1[(int64_t)lane * S + os] = h;   // plain copy for the last step's sample (wn_final_sample_kernel)
        }
      }
    }
  }
  if (!ok) {
    if (os == 0 && wave == 0)
      for (int i = lane; i < B * (t1 - t0); i += 64)
        a.y_out[(int64_t)(i / (t1 - t0)) * T + t0 + i % (t1 - t0)] = __builtin_nanf("");
    if (tid == 0) __hip_atomic_fetch_or(&g_wn_fault, kGFault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ================================================================ layer-pipelined generation
// (B <= 8, the r9y9 shapes R = 512, G = 512, S = 256, 3 taps, 24 layers).  ONE persistent launch
// per autovc_wavenet_generate_f32 call, its 256 workgroups (one per CU, 8 waves) split by LAYER
// instead of by gate pair: layer l runs on ten workgroups of XCD slot l % 8 (blocks b with
// b % 8 == l % 8, ranks b / 8 in [10 (l / 8), 10 (l / 8) + 10)), so every layer-to-layer hand-off
// crosses XCDs — measured (tools/wn_pipe_trace.py, profiles/r06/wn_pipe_trace_*.txt) a same-XCD
// hop of 16-byte write-through granules took 1.6-2.6 us from the last producer's store to the
// consumer's poll, a cross-XCD hop 0.6-0.9 us.  Slot 0's ranks 30-31 run the tail (the last
// layer's skip rows and the skip sum), slot 1's the head (h1 and the MoL head's partial sums);
// placement is a speed matter only: every hand-off is a tagged write-through granule.
// A layer's ten workgroups keep its current-tap gate rows [sqrt(.5) W_2 W_out(l-1) | sqrt(.5) W_2]
// in VGPRs and layer l-1's residual rows (W_out, W_skip) in LDS for the whole call (26 gate pairs
// x 2304 floats per workgroup), so a phase moves only its 768 inputs: the previous layer's 256
// granules {g_(l-1)[o], x_(l-1)[2o], x_(l-1)[2o+1], step + 1}, published by 10 producers (not the
// 256 of wn_grid_kernel's all-gather).
//   phase (l, t, u): the 8 waves poll 32 granules each into LDS, an LDS-counter sync, each wave
//   multiplies its <= 4 gate pairs (2 gate rows over 768 inputs, 3 residual rows over 256; lane L
//   owns granules 4L..4L+3), one butterfly, and lane q publishes gate pair q's granule for layer l
//   and layer l-1's skip row {s_(l-1)[o], tag} for the tail.  Utterances are independent chains:
//   each role serves (t, u) in order, so at B > 1 the utterances travel through the layers one
//   behind the other instead of sharing every hand-off.
//   past taps: after the last utterance of step t a layer's workgroups compute P_l(t+1) = W_0
//   x_l(t+1-2d) + W_1 x_l(t+1-d) for their own rows (weights streamed from memory once per group
//   of <= 4 utterances) into LDS, where phase (l, t+1, u) adds them: no hand-off at all.
//   head: h1 rows, then the MoL head's partial sums over the workgroup's 128 h1 rows (2 x 30
//   8-byte granules per utterance).  layer 0: every wave polls those 60 partials, adds them and
//   runs the mixture pick and the draw itself (the same Philox stream, the same value in every
//   wave: no LDS, no sync); its current tap is x_0 = in fw + fb, so z = in (W_2 fw) + W_2 fb with
//   both products formed once in the prologue.
//   tail: the skip rows of layers 0..21 accumulated as they arrive, then layer 22's (published
//   with layer 23's gate outputs) and layer 23's skip rows.
// A wait that gives up (the 256 workgroups were not all resident) sets the error word every other
// wait checks, the call's samples are poisoned with NaN and bit 2 of autovc_wavenet_fault is set.
constexpr int kPW = 8;                        // waves per workgroup
constexpr int kPQ = 4;                        // gate pairs per wave (at most)
constexpr int kPLayers = 24;

struct PLds {                                 // float offsets into the dynamic LDS block
  int wr, x, red, pt, h1, cnt, total;
};
__host__ __device__ inline PLds p_lds(int NB) {
  PLds o;
  int p = 0;
  // layer l-1's residual rows of this workgroup's gate pairs [wave][q][W_out 2o, 2o + 1, W_skip
  // o][lane][4] (96 KB; read back every phase while the inputs are polled: in VGPRs for the whole
  // call they pushed the past-tap pass into spills)
  o.wr = p;   p += kPW * kPQ * 3 * 256;
  o.x = p;    p += 2 * 256 * 4;               // staged input granules [parity][256][4]
  o.red = p;  p += kPW * 32;                  // per-wave reduced values [wave][32]
  o.pt = p;   p += NB * kPW * kPQ * 2;        // past taps of the coming step [u][wave][q][2]
  o.h1 = p;   p += 128;                       // head: the workgroup's h1 rows
  o.cnt = p;  p += 4;                         // the waves' LDS sync counter
  o.total = p;
  return o;
}

// role of workgroup bid: 1 = layer `layer` (member j of 10), 2 = tail (j of 2), 3 = head (j of 2),
// 0 = idle (slots 2-7, ranks 30-31)
__host__ __device__ inline void pipe_role(int bid, int& kind, int& layer, int& j) {
  const int xs = bid & 7, rk = bid >> 3;
  kind = 0; layer = 0; j = 0;
  if (rk < 30) { kind = 1; layer = (rk / 10) * 8 + xs; j = rk % 10; }
  else if (xs == 0) { kind = 2; j = rk - 30; }
  else if (xs == 1) { kind = 3; j = rk - 30; }
}

// LDS-counter sync of the NW waves of a workgroup, bounded like chain_sync (a wave that gave up
// elsewhere never arrives; the device error word then ends the wait)
template <int NW>
__device__ __forceinline__ bool wg_sync(int* cnt, int& k, int lane, int* err, int ticks, int step, int ph) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int want = NW * ++k;
  Spin sp{__builtin_amdgcn_s_memrealtime(), err, ticks, 3, step, ph};
  int n = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
    if ((++n & 255) == 0 && !sp.tick()) return false;
  asm volatile("" ::: "memory");
  return true;
}

// N 16-byte granules per lane at base + off[i] floats (wave-uniform base) until every tag == tag;
// the error word and the clock every 32nd retry (each check is a round trip the data may arrive in)
template <int N>
__device__ __forceinline__ bool p_poll(const float* base, const int (&off)[N], int tag, f32x4 (&g)[N], Spin& sp) {
  sp.chk = 31;
  while (true) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) g[i] = ld4_l2(base, off[i]);
    int bad = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) bad |= tag_of(g[i]) ^ tag;
    if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) return true;
    sp.seen = __builtin_amdgcn_readfirstlane(tag_of(g[0]));
    if (!sp.tick()) return false;
  }
}
// one 8-byte {value, tag} granule per lane
__device__ __forceinline__ bool p_poll2(const float* base, int off, int tag, float2& v, Spin& sp) {
  sp.chk = 31;
  while (true) {
    asm volatile("" ::: "memory");
    v = ld2_l2(base, off);
    if (__builtin_amdgcn_ballot_w64(__float_as_int(v.y) != tag) == 0) return true;
    sp.seen = __builtin_amdgcn_readfirstlane(__float_as_int(v.y));
    if (!sp.tick()) return false;
  }
}

#ifdef AVC_WN_PIPE_TRACE
// diagnostic build (tools/wn_pipe_trace.py): s_memrealtime stamps of wave 0 of every workgroup
// for utterance 0 of steps kTrT0 .. kTrT0 + kTrN - 1: [step][workgroup][event]
constexpr int kTrT0 = 64, kTrN = 4, kTrE = 8;
__device__ uint64_t g_pipe_trace[kTrN * 256 * kTrE];
#define PIPE_STAMP(T, U, E)                                                                          \
  do {                                                                                              \
    if ((U) == 0 && (T) >= kTrT0 && (T) < kTrT0 + kTrN && w == 0 && lane == 0)                   \
      g_pipe_trace[(((T) - kTrT0) * 256 + bid) * kTrE + (E)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define PIPE_STAMP(T, U, E) do {} while (0)
#endif

template <int NB>
__global__ __launch_bounds__(64 * kPW, 1) void wn_pipe_kernel(WnArgs a, int t0, int t1, int* errw, int ticks) {
  // fmaf where a sum is formed; no other contraction (every utterance is computed by the same
  // instruction sequence whatever the batch: batch invariance)
#pragma clang fp contract(off)
  constexpr int R = 512, H = 256, S = 256, KX = 3 * 512 + 256, KT = 2 * 512, G = 512;
#ifndef AVC_WN_PIPE_UG
#define AVC_WN_PIPE_UG 4
#endif
  // utterances per past-tap pass: 4 (B = 8 54.2 vs 57.9 us per sample step with 2, which keeps the
  // pass in registers; 4 spills 11 VGPRs of the pass, off the chain: profiles/r06/wn_pipe_v3_ab.txt)
  constexpr int UG = NB < AVC_WN_PIPE_UG ? NB : AVC_WN_PIPE_UG;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int L = a.n_layers, B = a.B, T = a.T, RING = a.RING, NO = a.NO;
  const PLds lo = p_lds(NB);
  f32x4* s_x = reinterpret_cast<f32x4*>(lds + lo.x);
  f32x4* s_wr = reinterpret_cast<f32x4*>(lds + lo.wr);
  float* s_red = lds + lo.red;
  float* s_pt = lds + lo.pt;
  float* s_h1 = lds + lo.h1;
  int* s_cnt = reinterpret_cast<int*>(lds + lo.cnt);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x;
  int kind, layer, j;
  pipe_role(bid, kind, layer, j);
  if (kind == 0) return;
  if (tid == 0) *s_cnt = 0;
  for (int i = tid; i < NB * kPW * kPQ * 2; i += 64 * kPW) s_pt[i] = 0.f;   // P(0) = 0
  // the polls are sc1 loads: drop any stale line of the hand-off regions (as wn_grid_kernel)
  if (tid < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  const int64_t RB4 = (int64_t)B * 256 * 4;   // floats of one ring slot (all utterances)
  float* gmolp = a.gsl + (int64_t)(L - 1) * B * 256 * 2;   // the MoL partials: [u][head wg][32] granules
  int kx = 0;                                 // wg_sync rounds
  int par = 0;                                // LDS staging parity
  bool ok = true;
  const float* W1 = head_base(a);
  const float* b1 = W1 + (int64_t)S * S;
  const float* W2 = b1 + S;
  const float* b2 = W2 + (int64_t)NO * S;

  if (kind == 1) {
    // =========================== a layer's workgroup: gate pairs o0 .. o0 + no - 1
    const int o0 = j < 6 ? 26 * j : 156 + 25 * (j - 6), no = j < 6 ? 26 : 25;
    const bool l0 = layer == 0;
    const float* lb = layer_base(a, layer);
    // this wave's gate pairs: local index w + 8 q; lane q < kPQ runs pair q's epilogue
    int oq[kPQ];
    bool vq[kPQ];
#pragma unroll
    for (int q = 0; q < kPQ; ++q) {
      vq[q] = w + 8 * q < no;
      oq[q] = o0 + (vq[q] ? w + 8 * q : 0);
    }
    // lane 16 q runs gate pair q's epilogue: after the butterfly its 5 sums sit on lanes 16 q +
    // 0, 2, 4, 6, 8 of the same DPP row
    const int my_q = lane >> 4;
    const bool my_valid = (lane & 15) == 0 && w + 8 * my_q < no;
    const int my_o = o0 + (my_valid ? w + 8 * my_q : 0);
    // resident gate weights, lane L's inputs: g[4L + i], x[8L + m] (granules 4L .. 4L + 3); the
    // residual rows wait in LDS (s_wr)
    float wa[kPQ][12], wb[kPQ][12];
    float bo0 = 0.f, bo1 = 0.f, bsk = 0.f;    // lane q: layer l-1's residual biases of pair q
    float ua = 0.f, va = 0.f, ub = 0.f, vb = 0.f;   // layer 0, lane q: W_2 fw, W_2 fb of rows o, o + H
    float fw0 = 0.f, fw1 = 0.f, fb0 = 0.f, fb1 = 0.f; // layer 0, lane q: first_conv of channels 2o, 2o + 1
    float b2l = 0.f;                          // layer 0, lane j < 32: the MoL head bias of output j
#pragma unroll
    for (int q = 0; q < kPQ; ++q) {
      const float* ra = lb + (int64_t)oq[q] * KX + KT;
      const float* rb = lb + (int64_t)(oq[q] + H) * KX + KT;
      const f32x4 ga = ld4(ra + 4 * lane), gb = ld4(rb + 4 * lane);
      const f32x4 xa0 = ld4(ra + H + 8 * lane), xa1 = ld4(ra + H + 8 * lane + 4);
      const f32x4 xb0 = ld4(rb + H + 8 * lane), xb1 = ld4(rb + H + 8 * lane + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wa[q][i] = vq[q] ? ga[i] : 0.f;
        wb[q][i] = vq[q] ? gb[i] : 0.f;
        wa[q][4 + i] = vq[q] ? xa0[i] : 0.f;
        wa[q][8 + i] = vq[q] ? xa1[i] : 0.f;
        wb[q][4 + i] = vq[q] ? xb0[i] : 0.f;
        wb[q][8 + i] = vq[q] ? xb1[i] : 0.f;
      }
      if (!l0) {
        const float* pb = layer_base(a, layer - 1) + (int64_t)G * KX;
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        const f32x4 r0 = ld4(pb + (int64_t)(2 * oq[q]) * H + 4 * lane);
        const f32x4 r1 = ld4(pb + (int64_t)(2 * oq[q] + 1) * H + 4 * lane);
        const f32x4 sk = ld4(pb + (int64_t)(R + oq[q]) * H + 4 * lane);
        s_wr[((w * kPQ + q) * 3 + 0) * 64 + lane] = vq[q] ? r0 : z4;
        s_wr[((w * kPQ + q) * 3 + 1) * 64 + lane] = vq[q] ? r1 : z4;
        s_wr[((w * kPQ + q) * 3 + 2) * 64 + lane] = vq[q] ? sk : z4;
      }
    }
    if (!l0) {
      const float* pbias = layer_base(a, layer - 1) + (int64_t)G * KX + (int64_t)(R + S) * H;
      if (my_valid) { bo0 = pbias[2 * my_o]; bo1 = pbias[2 * my_o + 1]; bsk = pbias[R + my_o]; }
    } else {
      // W_2 fw and W_2 fb of this wave's gate rows (lane L: channels 8L .. 8L + 7), one butterfly
      const f32x4 f0 = ld4(a.packed + 8 * lane), f1 = ld4(a.packed + 8 * lane + 4);
      const f32x4 c0 = ld4(a.packed + R + 8 * lane), c1 = ld4(a.packed + R + 8 * lane + 4);
      float v[16];
#pragma unroll
      for (int q = 0; q < kPQ; ++q) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s0 = fmaf(wa[q][4 + i], f0[i], s0); s0 = fmaf(wa[q][8 + i], f1[i], s0);
          s1 = fmaf(wa[q][4 + i], c0[i], s1); s1 = fmaf(wa[q][8 + i], c1[i], s1);
          s2 = fmaf(wb[q][4 + i], f0[i], s2); s2 = fmaf(wb[q][8 + i], f1[i], s2);
          s3 = fmaf(wb[q][4 + i], c0[i], s3); s3 = fmaf(wb[q][8 + i], c1[i], s3);
        }
        v[4 * q] = s0; v[4 * q + 1] = s1; v[4 * q + 2] = s2; v[4 * q + 3] = s3;
      }
      const float r = wave_reduce_hw<16>(v, lane);
      if ((lane & 3) == 0) s_red[w * 32 + (lane >> 2)] = r;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if ((lane & 15) == 0) {
        ua = s_red[w * 32 + 4 * my_q]; va = s_red[w * 32 + 4 * my_q + 1];
        ub = s_red[w * 32 + 4 * my_q + 2]; vb = s_red[w * 32 + 4 * my_q + 3];
        fw0 = a.packed[2 * my_o]; fw1 = a.packed[2 * my_o + 1];
        fb0 = a.packed[R + 2 * my_o]; fb1 = a.packed[R + 2 * my_o + 1];
      }
      b2l = b2[(lane & 31) < NO ? (lane & 31) : 0];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // s_wr: wave-private slices
    const int d = 1 << (layer % a.lps);

    // P_l(tn) for every utterance into s_pt: x_l(tn - 2d) (W_0), x_l(tn - d) (W_1); per pass (tap,
    // quarter) lane L owns channels 128 quarter + 2L, + 1 (granule 64 quarter + L, components 1, 2)
    auto past = [&](int tn) -> bool {
      for (int ug = 0; ug < B; ug += UG) {
        float acc[kPQ * 2 * UG];
#pragma unroll
        for (int i = 0; i < kPQ * 2 * UG; ++i) acc[i] = 0.f;
        for (int tap = 0; tap < 2; ++tap) {
          const int s = tn - (2 - tap) * d;
          if (s < 0) continue;
          const float* xr = a.gring + ((int64_t)layer * RING + (s & (RING - 1))) * RB4;
          for (int qt = 0; qt < 4; ++qt) {
            // the pass's weights are in flight while its inputs (every utterance of the group at
            // once: one round trip, not one per utterance) are polled
            float2 wv[kPQ][2];
#pragma unroll
            for (int q = 0; q < kPQ; ++q)
#pragma unroll
              for (int ab = 0; ab < 2; ++ab)
                wv[q][ab] = *reinterpret_cast<const float2*>(lb + (int64_t)(oq[q] + ab * H) * KX + tap * R + 128 * qt +
                                                             2 * lane);
            int off[UG];
#pragma unroll
            for (int uu = 0; uu < UG; ++uu) off[uu] = ((ug + uu < B ? ug + uu : 0) * 256 + 64 * qt + lane) * 4;
            f32x4 gx[UG];
            Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 4, tn, layer};
            if (!p_poll<UG>(xr, off, s + 1, gx, sp)) return false;
#pragma unroll
            for (int q = 0; q < kPQ; ++q)
#pragma unroll
              for (int ab = 0; ab < 2; ++ab)
#pragma unroll
                for (int uu = 0; uu < UG; ++uu) {
                  float sacc = acc[(q * 2 + ab) * UG + uu];
                  sacc = fmaf(wv[q][ab].x, gx[uu][1], sacc);
                  sacc = fmaf(wv[q][ab].y, gx[uu][2], sacc);
                  acc[(q * 2 + ab) * UG + uu] = sacc;
                }
          }
        }
        constexpr int NV = kPQ * 2 * UG;      // 8, 16 or 32
        const float r = wave_reduce_hw<NV>(acc, lane);
        if ((lane & (64 / NV - 1)) == 0) {
          const int vi = lane / (64 / NV);
          const int q = vi / (2 * UG), ab = (vi / UG) & 1, uu = vi % UG;
          if (ug + uu < B) s_pt[(((ug + uu) * kPW + w) * kPQ + q) * 2 + ab] = r;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      return true;
    };
    if (t0 > 0) ok = past(t0);

    for (int t = t0; t < t1 && ok; ++t) {
      const int ts = t & (RING - 1), prow = t % a.Tch;
      for (int u = 0; u < B && ok; ++u) {
        // epilogue operands of lane q: the conditioning and the past taps of gate pair q
        float pre_a = 0.f, pre_b = 0.f, pta = 0.f, ptb = 0.f;
        if (my_valid) {
          const float* pr = a.pre + ((int64_t)prow * B + u) * ((int64_t)L * G) + (int64_t)layer * G;
          pre_a = pr[my_o];
          pre_b = pr[my_o + H];
          pta = s_pt[((u * kPW + w) * kPQ + my_q) * 2];
          ptb = s_pt[((u * kPW + w) * kPQ + my_q) * 2 + 1];
        }
        float za = 0.f, zb = 0.f, x0n = 0.f, x1n = 0.f, sv = 0.f;
        PIPE_STAMP(t, u, 0);
        if (l0) {
          // ---- the draw of sample t-1 in every wave: the head's MoL partials (lane j < 32 from
          // head workgroup 0, lane 32 + j from head workgroup 1), the mixture pick on lanes 0..15
          const int tp = t - 1;
          float in_v = 0.f, smp = 0.f, mol = 0.f;
          if (tp >= 0) {
            const int jn = lane & 15;
            float gum = 0.f;                  // the noise of sample tp, before the poll
            if (lane < 16 && (jn < NO / 3 || jn == 10)) gum = mol_noise(jn, tp, a.utt_base + u, a);
            const int jo = lane & 31;
            float2 pv;
            Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 7, t, 0};
            if (!p_poll2(gmolp + (int64_t)u * 256 * 2, ((lane >> 5) * 32 + (jo < NO ? jo : 0)) * 2, t, pv, sp)) {
              ok = false;
              break;
            }
            PIPE_STAMP(t, u, 1);
            const auto rr = __builtin_amdgcn_permlane32_swap(__float_as_uint(pv.x), __float_as_uint(pv.x), false, false);
            mol = (__uint_as_float(rr[0]) + __uint_as_float(rr[1])) + b2l;
            const int nr = NO / 3;
            float v = -INFINITY;
            if (lane < nr) {
              v = mol - gum;
              if (!(v == v)) v = -INFINITY;
            }
            int bi = jn;
#pragma unroll
            for (int mm = 8; mm >= 1; mm >>= 1) {   // ties to the lowest index (mol_finish's rule)
              const float ov = __shfl_xor(v, mm);
              const int oi = __shfl_xor(bi, mm);
              if (ov > v || (ov == v && oi < bi)) { v = ov; bi = oi; }
            }
            bi = __builtin_amdgcn_readlane(bi, 0);
            const float mn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mol), nr + bi));
            const float ls = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mol), 2 * nr + bi)),
                                   a.log_scale_min);
            const float g10 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gum), 10));
            smp = fminf(fmaxf(mn + expf(ls) * g10, -1.0f), 1.0f);
            in_v = smp;
          }
          if (a.teacher != nullptr && t < a.teacher_len) in_v = a.teacher[(int64_t)u * a.teacher_len + t];
          if (j == 0 && w == 0) {
            if (lane == 0) a.yin[(int64_t)u * T + t] = in_v;
            if (tp >= 0) {
              if (lane == 0) a.y_out[(int64_t)u * T + tp] = smp;
              if (a.mol_out && lane < NO) a.mol_out[((int64_t)u * T + tp) * NO + lane] = mol;
            }
          }
          PIPE_STAMP(t, u, 3);
          if (my_valid) {
            za = fmaf(in_v, ua, va) + (pre_a + pta);
            zb = fmaf(in_v, ub, vb) + (pre_b + ptb);
            x0n = in_v * fw0 + fb0;
            x1n = in_v * fw1 + fb1;
          }
        } else {
          // ---- layer l-1's 256 granules of this step (utterance u), staged in LDS; the residual
          // rows are read back from LDS while they are polled
          f32x4 wrv[kPQ][3];
#pragma unroll
          for (int q = 0; q < kPQ; ++q)
#pragma unroll
            for (int r = 0; r < 3; ++r) wrv[q][r] = s_wr[((w * kPQ + q) * 3 + r) * 64 + lane];
          {
            const float* src = a.gring + ((int64_t)(layer - 1) * RING + ts) * RB4 + (int64_t)u * 256 * 4;
            // (two polls in flight, staggered, measured 0.6 us per sample step slower than one:
            // profiles/r06/wn_pipe_v4_ab_dbpoll.txt)
            const int off[1] = {(32 * w + (lane & 31)) * 4};
            f32x4 g[1];
            Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 1, t, layer};
            if (!p_poll<1>(src, off, t + 1, g, sp)) { ok = false; break; }
            if (lane < 32) s_x[par * 256 + 32 * w + lane] = g[0];
          }
          PIPE_STAMP(t, u, 1);
          if (!wg_sync<kPW>(s_cnt, kx, lane, errw, ticks, t, layer)) { ok = false; break; }
          PIPE_STAMP(t, u, 2);
          f32x4 in[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) in[i] = s_x[par * 256 + 4 * lane + i];
          const f32x4 xin = s_x[par * 256 + my_o];   // x_(l-1)[2o], [2o + 1]: the residual inputs
          float v[32];
#pragma unroll
          for (int q = 0; q < kPQ; ++q) {
            float sa = 0.f, sb = 0.f, s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              sa = fmaf(wa[q][i], in[i][0], sa);
              sb = fmaf(wb[q][i], in[i][0], sb);
              s0 = fmaf(wrv[q][0][i], in[i][0], s0);
              s1 = fmaf(wrv[q][1][i], in[i][0], s1);
              s2 = fmaf(wrv[q][2][i], in[i][0], s2);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              sa = fmaf(wa[q][4 + 2 * i], in[i][1], sa);
              sa = fmaf(wa[q][5 + 2 * i], in[i][2], sa);
              sb = fmaf(wb[q][4 + 2 * i], in[i][1], sb);
              sb = fmaf(wb[q][5 + 2 * i], in[i][2], sb);
            }
            v[8 * q] = sa; v[8 * q + 1] = sb; v[8 * q + 2] = s0; v[8 * q + 3] = s1; v[8 * q + 4] = s2;
            v[8 * q + 5] = v[8 * q + 6] = v[8 * q + 7] = 0.f;
          }
          const float r = wave_reduce_hw<32>(v, lane);
          PIPE_STAMP(t, u, 3);
          // lane 16 q gathers its pair's sums from lanes + 2, 4, 6, 8 (DPP row_shl: VALU, no LDS)
          const float r_zb = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(r), 0x102, 0xf, 0xf, false));
          const float r_x0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(r), 0x104, 0xf, 0xf, false));
          const float r_x1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(r), 0x106, 0xf, 0xf, false));
          const float r_sk = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(r), 0x108, 0xf, 0xf, false));
          if (my_valid) {
            za = r + (pre_a + pta);
            zb = r_zb + (pre_b + ptb);
            x0n = (r_x0 + bo0 + xin[1]) * kSqrtHalf;
            x1n = (r_x1 + bo1 + xin[2]) * kSqrtHalf;
            sv = r_sk + bsk;
          }
        }
        if (my_valid) {
          const float gv = avc_tanh_fast(za) * avc_sigmoid_fast(zb);
          st4_sc1(a.gring + ((int64_t)layer * RING + ts) * RB4, (u * 256 + my_o) * 4, gv, x0n, x1n, t + 1);
          if (!l0) st2t_sc1(a.gsl + (int64_t)(layer - 1) * B * 256 * 2, (u * 256 + my_o) * 2, sv, t + 1);
        }
        PIPE_STAMP(t, u, 4);
        par ^= 1;
      }
      PIPE_STAMP(t, 0, 5);
      if (ok && t + 1 < t1 && t + 1 < T) ok = past(t + 1);
      PIPE_STAMP(t, 0, 6);
    }
  } else if (kind == 2) {
    // =========================== tail: skip rows r = 128 j + 16 w + i of every layer, the skip sum
    const int r0 = 128 * j + 16 * w;
    const float* pb = layer_base(a, L - 1) + (int64_t)G * KX;
    float ws[16][4];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const f32x4 v = ld4(pb + (int64_t)(R + r0 + i) * H + 4 * lane);
#pragma unroll
      for (int k = 0; k < 4; ++k) ws[i][k] = v[k];
    }
    const float bskl = pb[(int64_t)(R + S) * H + R + r0 + (lane & 15)];
    for (int t = t0; t < t1 && ok; ++t) {
      const int ts = t & (RING - 1);
      for (int u = 0; u < B && ok; ++u) {
        float acc = 0.f;                      // lane i < 16: the running skip sum of row r0 + i
        PIPE_STAMP(t, u, 0);
        {
          // layers 0 .. L-3's skip rows: every pending layer's granule re-polled at once, the
          // ready prefix folded in (in layer order) each round — one round trip when they are
          // all out (utterances queued behind another), one per arrival while the chain runs
          constexpr int NL = kPLayers - 2;
          const float* sl0 = a.gsl + (int64_t)u * 256 * 2;
          const int off = (r0 + (lane & 15)) * 2;
          int k = 0;
          Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 6, t, 0};
          sp.chk = 31;
          while (k < NL) {
            asm volatile("" ::: "memory");
            float2 v[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l)
              if (l >= k) v[l] = ld2_l2(sl0 + (int64_t)l * B * 256 * 2, off);
#pragma unroll
            for (int l = 0; l < NL; ++l) {
              if (l < k) continue;
              if (__builtin_amdgcn_ballot_w64(__float_as_int(v[l].y) != t + 1) != 0) break;
              acc = l == 0 ? v[l].x : (a.legacy ? (acc + v[l].x) * kSqrtHalf : acc + v[l].x);
              k = l + 1;
            }
            if (k < NL && !sp.tick()) { ok = false; break; }
          }
        }
        if (!ok) break;
        // layer L-2's skip rows and layer L-1's gate outputs arrive from the same phase: both
        // polled at once, the gate outputs staged in LDS (32 granules per wave)
        {
          const float* sl = a.gsl + ((int64_t)(L - 2) * B + u) * 256 * 2;
          const float* src = a.gring + ((int64_t)(L - 1) * RING + ts) * RB4 + (int64_t)u * 256 * 4;
          const int gi = 32 * w + (lane & 31);
          f32x4 g;
          float2 v;
          Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 1, t, L};
          sp.chk = 31;
          while (true) {
            asm volatile("" ::: "memory");
            g = ld4_l2(src, gi * 4);
            v = ld2_l2(sl, (r0 + (lane & 15)) * 2);
            const int bad = (__float_as_int(v.y) ^ (t + 1)) | (tag_of(g) ^ (t + 1));
            if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) break;
            if (!sp.tick()) { ok = false; break; }
          }
          if (!ok) break;
          if (lane < 32) s_x[par * 256 + gi] = g;
          acc = L - 2 == 0 ? v.x : (a.legacy ? (acc + v.x) * kSqrtHalf : acc + v.x);
        }
        PIPE_STAMP(t, u, 1);
        if (!wg_sync<kPW>(s_cnt, kx, lane, errw, ticks, t, L)) { ok = false; break; }
        PIPE_STAMP(t, u, 2);
        float gin[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) gin[i] = s_x[par * 256 + 4 * lane + i][0];
        float vals[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sacc = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) sacc = fmaf(ws[i][k], gin[k], sacc);
          vals[i] = sacc;
        }
        const float r = wave_reduce_hw<16>(vals, lane);
        if ((lane & 3) == 0) s_red[w * 32 + (lane >> 2)] = r;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 16) {
          const float svl = s_red[w * 32 + lane] + bskl;
          const float tot = a.legacy ? (acc + svl) * kSqrtHalf : acc + svl;
          st4_sc1(a.gsk, (u * 256 + r0 + lane) * 4, tot, 0.f, 0.f, t + 1);
        }
        PIPE_STAMP(t, u, 4);
        par ^= 1;
      }
    }
  } else {
    // =========================== head: h1 rows r = 128 j + 16 w + i, then the MoL partial sums
    // of this workgroup's 128 rows (wave w: outputs w + 8 m; lane L: rows 2L, 2L + 1)
    const int r0 = 128 * j + 16 * w;
    float wh[16][4];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const f32x4 v = ld4(W1 + (int64_t)(r0 + i) * S + 4 * lane);
#pragma unroll
      for (int k = 0; k < 4; ++k) wh[i][k] = v[k];
    }
    const float b1r = b1[r0 + (lane & 15)];
    float w2c[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int jo = w + 8 * m < NO ? w + 8 * m : 0;
      w2c[m][0] = W2[(int64_t)jo * S + 128 * j + 2 * lane];
      w2c[m][1] = W2[(int64_t)jo * S + 128 * j + 2 * lane + 1];
    }
    for (int t = t0; t < t1 && ok; ++t) {
      for (int u = 0; u < B && ok; ++u) {
        PIPE_STAMP(t, u, 0);
        {
          const float* src = a.gsk + (int64_t)u * 256 * 4;
          const int off[1] = {(32 * w + (lane & 31)) * 4};
          f32x4 g[1];
          Spin sp{__builtin_amdgcn_s_memrealtime(), errw, ticks, 6, t, L + 1};
          if (!p_poll<1>(src, off, t + 1, g, sp)) { ok = false; break; }
          if (lane < 32) s_x[par * 256 + 32 * w + lane] = g[0];
        }
        PIPE_STAMP(t, u, 1);
        if (!wg_sync<kPW>(s_cnt, kx, lane, errw, ticks, t, L + 1)) { ok = false; break; }
        PIPE_STAMP(t, u, 2);
        float sk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sk[i] = fmaxf(s_x[par * 256 + 4 * lane + i][0], 0.f);
        float vals[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sacc = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) sacc = fmaf(wh[i][k], sk[k], sacc);
          vals[i] = sacc;
        }
        const float r = wave_reduce_hw<16>(vals, lane);
        if ((lane & 3) == 0) s_red[w * 32 + (lane >> 2)] = r;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 16) {
          const float h = fmaxf(s_red[w * 32 + lane] + b1r, 0.f);
          s_h1[16 * w + lane] = h;
          a.h1[(int64_t)u * S + r0 + lane] = h;   // plain copy for the last step's sample (wn_final_sample_kernel)
        }
        if (!wg_sync<kPW>(s_cnt, kx, lane, errw, ticks, t, L + 1)) { ok = false; break; }
        const float h0 = s_h1[2 * lane], h1v = s_h1[2 * lane + 1];
        float mv[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) mv[m] = fmaf(w2c[m][1], h1v, w2c[m][0] * h0);
        const float p = wave_reduce_hw<4>(mv, lane);
        if ((lane & 15) == 0) {
          const int jo = w + 8 * (lane >> 4);
          if (jo < NO) st2t_sc1(gmolp + (int64_t)u * 256 * 2, (j * 32 + jo) * 2, p, t + 1);
        }
        PIPE_STAMP(t, u, 4);
        par ^= 1;
      }
    }
  }
  if (!ok) {
    if (bid == 0 && w == 0)
      for (int i = lane; i < B * (t1 - t0); i += 64)
        a.y_out[(int64_t)(i / (t1 - t0)) * T + t0 + i % (t1 - t0)] = __builtin_nanf("");
    if (tid == 0) __hip_atomic_fetch_or(&g_wn_fault, kGFault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- graph cache: a captured S-step graph depends only on WnArgs and S.
struct GraphKey {
  WnArgs a;
  int steps;
  int slot0;      // ring slot of the graph's first step
  int prow0;      // conditioning row of the graph's first step
  int device;
  bool operator<(const GraphKey& o) const { return memcmp(this, &o, sizeof(GraphKey)) < 0; }
};
std::mutex g_mu;
std::map<GraphKey, hipGraphExec_t> g_graphs;
std::vector<GraphKey> g_order;
hipStream_t g_capture_stream[64] = {};

// one sample step: ring slot, conditioning row, and t (direct launch) or -1 (graph replay)
int enqueue_step(const WnArgs& a, hipStream_t s, int slot, int prow, int targ) {
  const int H = a.G / 2;
  const int nbt = (a.B + kBT - 1) / kBT;
  const dim3 lgrid(H / kRP, (a.B + kUB - 1) / kUB);
  for (int l = 0; l < a.n_layers; ++l) {
    if (l == 0) hipLaunchKernelGGL((wn_layer_kernel<true>), lgrid, dim3(kLayerThreads), 0, s, a, 0, slot, prow, targ);
    else hipLaunchKernelGGL((wn_layer_kernel<false>), lgrid, dim3(kLayerThreads), 0, s, a, l, slot, prow, targ);
  }
  const int own = (a.S + kTailWaves - 1) / kTailWaves;
  hipLaunchKernelGGL((wn_tail_kernel<kTailWaves>), dim3(own + past_tap_blocks(a, a.n_layers / 2), nbt),
                     dim3(64 * kTailWaves), 0, s, a, slot);
  hipLaunchKernelGGL((wn_head_kernel<kTailWaves>), dim3(a.S / kHR + past_tap_blocks(a, a.n_layers - a.n_layers / 2), nbt),
                     dim3(64 * kTailWaves), 0, s, a, slot, targ);
  AVC_CHECK_LAUNCH("autovc_wavenet_generate_f32");
  return avc::kOk;
}

// a graph of `steps` sample steps starting at ring slot slot0 and conditioning row prow0:
// every kernel argument is static (slot (slot0 + i) & (RING-1), row prow0 + i)
int get_graph(const WnArgs& a, int steps, int slot0, int prow0, hipGraphExec_t* out) {
  int dev = 0;
  AVC_HIP(hipGetDevice(&dev), "hipGetDevice");
  GraphKey key;
  memset(&key, 0, sizeof(key));
  key.a = a;
  key.steps = steps;
  key.slot0 = slot0;
  key.prow0 = prow0;
  key.device = dev;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_graphs.find(key);
  if (it != g_graphs.end()) { *out = it->second; return avc::kOk; }
  if (dev < 0 || dev >= 64) { avc::set_error("wavenet: device index %d", dev); return avc::kErrArg; }
  if (!g_capture_stream[dev]) AVC_HIP(hipStreamCreateWithFlags(&g_capture_stream[dev], hipStreamNonBlocking), "hipStreamCreate");
  hipStream_t cs = g_capture_stream[dev];
  AVC_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
  int rc = avc::kOk;
  for (int i = 0; i < steps && rc == avc::kOk; ++i) rc = enqueue_step(a, cs, (slot0 + i) & (a.RING - 1), prow0 + i, -1);
  hipGraph_t graph = nullptr;
  const hipError_t e = hipStreamEndCapture(cs, &graph);
  if (rc != avc::kOk) { if (graph) (void)hipGraphDestroy(graph); return rc; }
  AVC_HIP(e, "hipStreamEndCapture");
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  AVC_HIP(ei, "hipGraphInstantiate");
  if (g_order.size() >= 16) {  // bounded cache: drop the oldest graph
    auto old = g_graphs.find(g_order.front());
    if (old != g_graphs.end()) { (void)hipGraphExecDestroy(old->second); g_graphs.erase(old); }
    g_order.erase(g_order.begin());
  }
  g_graphs[key] = exec;
  g_order.push_back(key);
  *out = exec;
  return avc::kOk;
}

int g_wn_timeout_ticks = 100000000;   // 1 s of s_memrealtime (100 MHz) per phase wait

// All-CU weight-resident generation (wn_grid_kernel): 0 never, 1 every eligible batch, 2 (the
// default) up to two utterances — the measured crossover: B = 1 86.5, B = 2 101.1 us per sample
// step against 103.8 / 104.6 for the launches, B = 4 and up slower (profiles/r04/wn_grid_ab.txt).
// 3: the layer-pipelined kernel (wn_pipe_kernel) for every eligible batch (B <= 8, 24 layers).
// AVC_WN_GRID outside 0..3 is rejected by the first generate call (g_wn_grid_bad), as
// autovc_wavenet_set_grid rejects it, rather than read as "every batch" with its fault unread
// Default 3: the layer-pipelined kernel beats both others at every B <= 8 (B = 1 54.6 vs 86.2
// (mode 2) vs 104.7 us per sample step for the launches, B = 8 54.2 vs 109.3 and 129.2 (mode 1);
// profiles/r06/wn_pipe_v3_ab.txt).
constexpr int kWnGridDefault = 3;
int g_wn_grid_bad = 0;
int g_wn_grid = [] {
  const char* e = getenv("AVC_WN_GRID");
  if (!e) return kWnGridDefault;
  if (e[0] >= '0' && e[0] <= '3' && e[1] == 0) return e[0] - '0';
  g_wn_grid_bad = 1;
  return kWnGridDefault;
}();
int g_wn_grid_explicit = getenv("AVC_WN_GRID") != nullptr;   // the mode was chosen, not defaulted
// which path the last autovc_wavenet_generate_f32 call took: 0 the per-layer launches, 1 the
// all-CU persistent kernel, 2 the layer-pipelined persistent kernel (1, 2: the caller must read
// the fault word)
int g_wn_last_path = 0;

template <int NB>
bool pipe_attr(int bytes) {
  int per = 0;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(wn_pipe_kernel<NB>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess &&
         hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, wn_pipe_kernel<NB>, 64 * kPW, bytes) == hipSuccess &&
         per >= 1;
}

bool pipe_eligible(int B, int n_layers, int taps, int R, int G, int S, int NO) {
  if (g_wn_grid != 3 || B > 8 || n_layers != kPLayers || taps != 3 || R != 512 || G != 512 || S != 256 || NO > kMaxNO)
    return false;
  static int ok = -1;
  if (ok < 0) {
    ok = 0;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus == 256 &&
        pipe_attr<1>(4 * p_lds(1).total) && pipe_attr<2>(4 * p_lds(2).total) && pipe_attr<4>(4 * p_lds(4).total) &&
        pipe_attr<8>(4 * p_lds(8).total))
      ok = 1;
  }
  return ok == 1;
}

template <int NB>
bool grid_attr(int bytes) {
  int per = 0;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(wn_grid_kernel<NB>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess &&
         hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, wn_grid_kernel<NB>, 64 * kGrW, bytes) == hipSuccess &&
         per >= 1;
}

bool grid_eligible(int B, int n_layers, int taps, int R, int G, int S, int NO) {
  if (!g_wn_grid || g_wn_grid == 3 || (g_wn_grid == 2 && B > 2) || B > kGMaxB || n_layers < 8 || n_layers > kGMaxL || taps != 3 || R != 512 || G != 512 ||
      S != 256 || NO > kMaxNO)
    return false;
  static int ok = -1;
  static int lds_ok_for = -1;
  const int bytes = 4 * g_lds(n_layers, NO).total;
  if (ok < 0 || lds_ok_for != bytes) {
    ok = 0;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus == 256 &&
        grid_attr<1>(bytes) && grid_attr<2>(bytes) && grid_attr<4>(bytes) && grid_attr<8>(bytes))
      ok = 1;
    lds_ok_for = bytes;
  }
  return ok == 1;
}

int64_t ring_frames(int n_layers, int lps, int K) {
  const int64_t dmax = (int64_t)1 << (std::min(n_layers, lps) - 1);
  const int64_t need = (K - 1) * dmax + 1;
  int64_t r = 1;
  while (r < need) r <<= 1;
  return r;
}

}  // namespace

extern "C" {


int autovc_wavenet_set_grid(int on) {
  AVC_CHECK_ARG(on >= 0 && on <= 3, "autovc_wavenet_set_grid: 0 (off), 1 (B <= 8), 2 (B <= 2) or 3 (layer-pipelined, B <= 8)");
  g_wn_grid = on;
  g_wn_grid_bad = 0;
  g_wn_grid_explicit = 1;
  return avc::kOk;
}

int autovc_wavenet_get_grid(void) { return g_wn_grid; }

int autovc_wavenet_grid_explicit(void) { return g_wn_grid_explicit; }

int autovc_wavenet_reset_grid(void) {
  g_wn_grid = kWnGridDefault;
  g_wn_grid_bad = 0;
  g_wn_grid_explicit = 0;
  return avc::kOk;
}

int autovc_wavenet_last_path(void) { return g_wn_last_path; }


int autovc_wavenet_grid_diag(int clear, int* out5) {
  AVC_CHECK_ARG(out5 != nullptr, "autovc_wavenet_grid_diag: null out");
  AVC_HIP(hipDeviceSynchronize(), "hipDeviceSynchronize");
  AVC_HIP(hipMemcpyFromSymbol(out5, HIP_SYMBOL(g_wn_grid_diag), 5 * sizeof(int)), "hipMemcpyFromSymbol");
  if (clear) {
    const int zero[5] = {};
    AVC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wn_grid_diag), zero, 5 * sizeof(int)), "hipMemcpyToSymbol");
  }
  return avc::kOk;
}

#ifdef AVC_WN_PIPE_TRACE
int autovc_wavenet_pipe_trace(uint64_t* out) {   // trace build only (tools/wn_pipe_trace.py)
  AVC_HIP(hipDeviceSynchronize(), "hipDeviceSynchronize");
  AVC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pipe_trace), sizeof(g_pipe_trace)), "hipMemcpyFromSymbol");
  return avc::kOk;
}
#endif

int autovc_wavenet_set_timeout_ticks(int ticks) {
  AVC_CHECK_ARG(ticks >= 0, "autovc_wavenet_set_timeout_ticks: ticks >= 0");
  g_wn_timeout_ticks = ticks > 0 ? ticks : 100000000;
  return avc::kOk;
}

int autovc_wavenet_fault(int clear, int* out) {
  AVC_CHECK_ARG(out != nullptr, "autovc_wavenet_fault: null out");
  AVC_HIP(hipDeviceSynchronize(), "hipDeviceSynchronize");
  AVC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wn_fault), sizeof(int)), "hipMemcpyFromSymbol");
  if (clear) {
    const int zero = 0;
    AVC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wn_fault), &zero, sizeof(int)), "hipMemcpyToSymbol");
  }
  return avc::kOk;
}

int64_t autovc_wavenet_ring_frames(int n_layers, int layers_per_stack, int taps) {
  if (n_layers <= 0 || layers_per_stack <= 0 || layers_per_stack > 16 || taps <= 0) return -1;
  return ring_frames(n_layers, layers_per_stack, taps);
}

int64_t autovc_wavenet_packed_floats(int n_layers, int taps, int R, int G, int S, int n_out) {
  if (n_layers <= 0 || taps <= 0 || R <= 0 || G <= 0 || S <= 0 || n_out <= 0) return -1;
  const int64_t H = G / 2;
  const int64_t per = (int64_t)G * (taps * R + H) + (int64_t)(R + S) * H + (R + S);
  return 2 * (int64_t)R + n_layers * per + (int64_t)S * S + S + (int64_t)n_out * S + n_out;
}

int64_t autovc_wavenet_workspace_bytes(int B, int T, int n_layers, int layers_per_stack, int taps, int R, int G,
                                       int S) {
  if (B <= 0 || T <= 0 || n_layers <= 0 || layers_per_stack <= 0 || taps <= 0) return -1;
  const int64_t ring = (int64_t)(n_layers + 1) * ring_frames(n_layers, layers_per_stack, taps) * B * R;
  const int64_t floats = ring + (int64_t)B * T + 2 * (int64_t)B * S + 2 * (int64_t)B * (G / 2) +
                         2 * (int64_t)n_layers * B * G + (int64_t)(S / kHR) * B * kMaxNO + 7 * 64;
  const int64_t grid = 16 * ((int64_t)n_layers * ring_frames(n_layers, layers_per_stack, taps) * B * 256 + 2 * (int64_t)B * 256) +
                       8 * 2 * (int64_t)n_layers * B * 512 +  // wn_grid_kernel's tagged granules
                       8 * (int64_t)n_layers * B * 256;       // wn_pipe_kernel's skip-row granules
  return floats * 4 + kCtrSlots * 4 + kGErrInts * 4 + grid + 1024;
}

int autovc_wavenet_upsample_f32(int B, int Tc, int C, int n_stages, const int* scales, const float* c,
                                const float* w, const float* bias, float* out, hipStream_t stream) {
  AVC_CHECK_ARG(B > 0 && Tc > 0 && C > 0 && n_stages > 0 && n_stages <= kUpMaxStages,
                "autovc_wavenet_upsample_f32: bad dims B=%d Tc=%d C=%d n=%d", B, Tc, C, n_stages);
  AVC_CHECK_ARG(scales && c && w && bias && out, "autovc_wavenet_upsample_f32: null pointer");
  UpArgs u;
  memset(&u, 0, sizeof(u));
  u.B = B; u.Tc = Tc; u.C = C; u.n = n_stages; u.P = 1;
  int off = 0;
  for (int i = 0; i < n_stages; ++i) {
    AVC_CHECK_ARG(scales[i] > 0, "autovc_wavenet_upsample_f32: scale %d", scales[i]);
    u.s[i] = scales[i];
    u.woff[i] = off;
    off += 3 * scales[i];
    u.P *= scales[i];
  }
  const int64_t lds = (int64_t)C * (u.P / u.s[n_stages - 1]) * 2 * 4;
  AVC_CHECK_ARG(lds <= 160 * 1024, "autovc_wavenet_upsample_f32: C * prod(scales[:-1]) too large for LDS");
  hipLaunchKernelGGL(wn_upsample_kernel, dim3(Tc, B), dim3(256), (size_t)lds, stream, u, c, w, bias, out);
  AVC_CHECK_LAUNCH("autovc_wavenet_upsample_f32");
  return avc::kOk;
}

int autovc_wavenet_generate_f32(int B, int T, int t0, int t1, int n_layers, int layers_per_stack, int taps, int R,
                                int G, int S, int n_out, int legacy, const float* packed, const float* pre, int Tch,
                                uint64_t seed, int utt_base, float log_scale_min, const float* teacher,
                                int teacher_len, float* y_out, float* mol_out, void* workspace, int graph_steps,
                                hipStream_t stream) {
  static const char* fn = "autovc_wavenet_generate_f32";
  AVC_CHECK_ARG(!g_wn_grid_bad, "%s: AVC_WN_GRID must be 0 (per-layer launches), 1 (all-CU kernel for B <= 8), 2 "
                "(all-CU kernel for B <= 2, the default) or 3 (layer-pipelined kernel for B <= 8)", fn);
  AVC_CHECK_ARG(B > 0 && T > 0 && 0 <= t0 && t0 < t1 && t1 <= T, "%s: bad range B=%d T=%d t=[%d,%d)", fn, B, T, t0, t1);
  AVC_CHECK_ARG(Tch > 0 && t1 - t0 <= Tch, "%s: chunk [%d,%d) longer than the conditioning chunk %d", fn, t0, t1, Tch);
  AVC_CHECK_ARG(n_layers >= 1 && n_layers + 2 < kCtrSlots && layers_per_stack >= 1 && layers_per_stack <= 16 &&
                    taps >= 1,
                "%s: bad layer structure layers=%d per_stack=%d taps=%d", fn, n_layers, layers_per_stack, taps);
  AVC_CHECK_ARG(R > 0 && R % 256 == 0 && G > 0 && G % 512 == 0 && S > 0 && S % 256 == 0 &&
                    R % (G / 2) == 0 && S % (G / 2) == 0 && G / 2 == 256 && S == 256 &&
                    kRP * ((R + S) / (G / 2)) <= kRW * kResRows && taps >= 2,
                "%s: need G/2 == S == 256, R a multiple of 256 with (R + S) / (G/2) <= %d, taps >= 2 "
                "(R=%d, G/2=%d, S=%d)", fn, kRW * kResRows / kRP,
                R, G / 2, S);
  AVC_CHECK_ARG(n_out % 3 == 0 && n_out / 3 >= 1 && n_out / 3 <= 10 && n_out <= kMaxNO,
                "%s: out_channels %d is not 3 x (1..10) logistic mixtures", fn, n_out);
  AVC_CHECK_ARG(packed && pre && y_out && workspace, "%s: null pointer", fn);
  AVC_CHECK_ARG(AVC_ALIGNED16(packed) && AVC_ALIGNED16(workspace), "%s: packed/workspace must be 16-byte aligned", fn);
  AVC_CHECK_ARG(teacher == nullptr || (teacher_len >= 0 && teacher_len <= T), "%s: teacher_len %d", fn, teacher_len);
  AVC_CHECK_ARG(graph_steps >= 0 && graph_steps <= 4096, "%s: graph_steps %d", fn, graph_steps);

  auto round64 = [](int64_t n) { return (n + 63) / 64 * 64; };
  const int RING = (int)ring_frames(n_layers, layers_per_stack, taps);
  float* ws = static_cast<float*>(workspace);
  WnArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.T = T; a.R = R; a.G = G; a.S = S; a.NO = n_out; a.K = taps; a.RING = RING;
  a.n_layers = n_layers; a.lps = layers_per_stack; a.Tch = Tch; a.legacy = legacy ? 1 : 0;
  a.packed = packed; a.pre = pre;
  a.ring = ws;                 ws += round64((int64_t)(n_layers + 1) * RING * B * R);
  a.yin = ws;                  ws += round64((int64_t)B * T);
  a.skip = ws;                 ws += round64((int64_t)B * S);
  a.h1 = ws;                   ws += round64((int64_t)B * S);
  a.gbuf = ws;                 ws += round64(2 * (int64_t)B * (G / 2));
  a.ptap = ws;                 ws += round64(2 * (int64_t)n_layers * B * G);
  a.molp = ws;                 ws += round64((int64_t)(S / kHR) * B * kMaxNO);
  a.ctr = reinterpret_cast<int*>(ws);
  int* gerr = a.ctr + kCtrSlots;   // the all-CU generation's error word (one line)
  {
    float* g = reinterpret_cast<float*>(gerr + kGErrInts);
    a.gring = g;  g += 4 * (int64_t)n_layers * RING * B * 256;
    a.gsk = g;    g += 4 * (int64_t)B * 256;
    a.gh1 = g;    g += 4 * (int64_t)B * 256;
    a.gpt = g;    g += 2 * 2 * (int64_t)n_layers * B * 512;
    a.gsl = g;    g += 2 * (int64_t)n_layers * B * 256;
  }
  a.teacher = teacher; a.teacher_len = teacher ? teacher_len : 0;
  a.y_out = y_out; a.mol_out = mol_out;
  a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32);
  a.utt_base = utt_base; a.log_scale_min = log_scale_min;
  const int64_t used = reinterpret_cast<char*>(a.gsl + 2 * (int64_t)n_layers * B * 256) - static_cast<char*>(workspace);
  AVC_CHECK_ARG(used <= autovc_wavenet_workspace_bytes(B, T, n_layers, layers_per_stack, taps, R, G, S),
                "%s: workspace layout overflow", fn);

  if (t0 == 0) AVC_HIP(avc::zero_async(workspace, (size_t)used, stream), "zero_async");
  g_wn_last_path = 0;
  if (pipe_eligible(B, n_layers, taps, R, G, S, n_out)) {
    // one persistent launch for the whole call, each layer's current-tap and residual rows on
    // ten CUs of their own, utterances flowing through the layers (wn_pipe_kernel)
    g_wn_last_path = 2;
    AVC_HIP(avc::zero_async(gerr, (size_t)kGErrInts * 4, stream), "zero_async");
    const int lds = 4 * p_lds(B == 1 ? 1 : B == 2 ? 2 : B <= 4 ? 4 : 8).total;
    if (B == 1) hipLaunchKernelGGL(wn_pipe_kernel<1>, dim3(256), dim3(64 * kPW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else if (B == 2) hipLaunchKernelGGL(wn_pipe_kernel<2>, dim3(256), dim3(64 * kPW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else if (B <= 4) hipLaunchKernelGGL(wn_pipe_kernel<4>, dim3(256), dim3(64 * kPW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else hipLaunchKernelGGL(wn_pipe_kernel<8>, dim3(256), dim3(64 * kPW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    AVC_CHECK_LAUNCH(fn);
    if (t1 == T) {
      hipLaunchKernelGGL(wn_final_sample_kernel, dim3(1, (B + kBT - 1) / kBT), dim3(256), 0, stream, a, T);
      AVC_CHECK_LAUNCH(fn);
    }
    return avc::kOk;
  }
  if (grid_eligible(B, n_layers, taps, R, G, S, n_out)) {
    // one persistent launch for the whole call, every gate weight of the chain on chip (wn_grid_kernel)
    g_wn_last_path = 1;
    AVC_HIP(avc::zero_async(gerr, (size_t)kGErrInts * 4, stream), "zero_async");
    const int lds = 4 * g_lds(n_layers, n_out).total;
    if (B == 1) hipLaunchKernelGGL(wn_grid_kernel<1>, dim3(256), dim3(64 * kGrW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else if (B == 2) hipLaunchKernelGGL(wn_grid_kernel<2>, dim3(256), dim3(64 * kGrW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else if (B <= 4) hipLaunchKernelGGL(wn_grid_kernel<4>, dim3(256), dim3(64 * kGrW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    else hipLaunchKernelGGL(wn_grid_kernel<8>, dim3(256), dim3(64 * kGrW), lds, stream, a, t0, t1, gerr, g_wn_timeout_ticks);
    AVC_CHECK_LAUNCH(fn);
    if (t1 == T) {
      hipLaunchKernelGGL(wn_final_sample_kernel, dim3(1, (B + kBT - 1) / kBT), dim3(256), 0, stream, a, T);
      AVC_CHECK_LAUNCH(fn);
    }
    return avc::kOk;
  }
  hipLaunchKernelGGL(wn_set_ctr_kernel, dim3(1), dim3(1), 0, stream, a.ctr, t0);
  AVC_CHECK_LAUNCH(fn);
  // graph replays cover runs of graph_steps steps inside the conditioning chunk (a graph
  // per (ring slot, chunk row) of its first step: callers keep Tch a small multiple of
  // graph_steps and of the ring, so a few graphs serve every chunk); the rest launch directly
  int t = t0;
  while (t < t1) {
    if (graph_steps > 0 && t + graph_steps <= t1 && t % Tch + graph_steps <= Tch) {
      hipGraphExec_t exec = nullptr;
      const int rc = get_graph(a, graph_steps, t & (RING - 1), t % Tch, &exec);
      if (rc != avc::kOk) return rc;
      AVC_HIP(hipGraphLaunch(exec, stream), "hipGraphLaunch");
      t += graph_steps;
      continue;
    }
    const int rc = enqueue_step(a, stream, t & (RING - 1), t % Tch, t);
    if (rc != avc::kOk) return rc;
    ++t;
  }
  if (t1 == T) {
    hipLaunchKernelGGL(wn_final_sample_kernel, dim3(1, (B + kBT - 1) / kBT), dim3(256), 0, stream, a, T);
    AVC_CHECK_LAUNCH(fn);
  }
  return avc::kOk;
}

}  // extern "C"
