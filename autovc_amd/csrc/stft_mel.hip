// Fused STFT + mel filterbank + log/normalise front end (gfx950).
//
// Replaces, for a batch of utterances at once:
//   make_spect.py:36-48   Spect.pySTFT  (reflect pad 512, 1024-pt frames at hop 256,
//                                        periodic Hann, |rfft|)
//   make_spect.py:79-83   spmel branch  (D.T @ mel_basis -> 20*log10(max(1e-5, .)) - 16
//                                        -> clip((.+100)/100, 0, 1))
//   make_spect.py:84-86   stft branch   (same without the mel projection)
//
// One WAVEFRONT transforms a contiguous run of frames (4 waves per 256-thread workgroup;
// the only workgroup barrier is after the sparse mel basis is staged into LDS).
// The 1024 real windowed samples are packed as 512 complex values z[n] = x[2n] + i x[2n+1]
// (real-FFT trick), transformed by a 512-point FFT done as three radix-8 passes in
// registers (8 complex values per lane, 64 lanes) with two wave-local LDS exchanges, and
// unpacked to the 513 one-sided bins X[k] = E[k] + W^k O[k].  Reflect padding is an
// index fold, never materialised.  Twiddles and the periodic Hann window come from one
// float64 table exp(-2 pi i e / 1024) (twiddle1024.h), so no transcendental is evaluated
// per butterfly.  Arithmetic is float64 like the reference (numpy pocketfft on the f64
// dithered signal): an fp32 FFT misses the 1e-4 bound on quiet bins of loud frames (the
// rounding noise of the loudest bin lands above the -84 dB clip floor).
// HBM traffic per frame = 256 new f64 input samples (the other 768 are cache hits from
// the neighbouring frames) + the f32 output row: 2,368 B for spmel, 4,100 B for stft.
#include <algorithm>

#include "common.h"
#include "twiddle1024.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int kN = 1024;      // fft_length (make_spect.py:24)
constexpr int kHop = 256;     // hop_length (make_spect.py:25)
constexpr int kBins = kN / 2 + 1;
constexpr int kWaves = 4;     // frames per workgroup
constexpr int kThreads = 64 * kWaves;

struct cd { double x, y; };

__device__ __forceinline__ cd cmul(cd a, cd b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cd cadd(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd csub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd mul_mi(cd a) { return {a.y, -a.x}; }   // a * (-i)
__device__ __forceinline__ cd tw(const avc_c64* T, int e) {
  const avc_c64 t = T[e & (kN - 1)];
  return {t.x, t.y};
}

// numpy.pad(mode='reflect') index fold (edge sample not repeated); handles pads
// longer than the signal the way numpy's iterated reflection does.
// (int32 within one utterance: utterances must be shorter than 2^31 - 1024 samples,
// 37 hours at 16 kHz; the batch offsets themselves are int64)
__device__ __forceinline__ int reflect_idx(int i, int L) {
  if ((unsigned)i < (unsigned)L) return i;
  if (L <= 1) return 0;
  const int P = 2 * (L - 1);
  i %= P;
  if (i < 0) i += P;
  return i < L ? i : P - i;
}

// In-register radix-8 DFT, natural order in and out: a[k] <- sum_n a[n] exp(-2 pi i nk/8).
__device__ __forceinline__ void dft8(cd (&a)[8]) {
  constexpr double r = 0.70710678118654752440;  // 1/sqrt(2)
  cd b[4], c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    b[k] = cadd(a[k], a[k + 4]);
    c[k] = csub(a[k], a[k + 4]);
  }
  // odd half times W8^k, W8 = (1 - i)/sqrt2
  c[1] = {(c[1].x + c[1].y) * r, (c[1].y - c[1].x) * r};
  c[2] = mul_mi(c[2]);
  c[3] = {(c[3].y - c[3].x) * r, -(c[3].x + c[3].y) * r};
  const cd e0 = cadd(b[0], b[2]), e2 = csub(b[0], b[2]), e1 = cadd(b[1], b[3]), e3 = mul_mi(csub(b[1], b[3]));
  const cd f0 = cadd(c[0], c[2]), f2 = csub(c[0], c[2]), f1 = cadd(c[1], c[3]), f3 = mul_mi(csub(c[1], c[3]));
  a[0] = cadd(e0, e1); a[4] = csub(e0, e1); a[2] = cadd(e2, e3); a[6] = csub(e2, e3);
  a[1] = cadd(f0, f1); a[5] = csub(f0, f1); a[3] = cadd(f2, f3); a[7] = csub(f2, f3);
}

// The wave's outstanding LDS operations are complete, and the compiler may not move LDS
// accesses across this point.  Each frame's buffers belong to one wave, and one wave's
// LDS operations execute in issue order, so this is the whole exchange protocol.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// 20*log10(max(min_level, v)) - 16 -> clip((. + 100)/100, 0, 1)   (make_spect.py:52,81-83).
// Magnitudes, mel sums and the dB map run in fp32: after the fp64 transform each value
// only needs ~1e-3 relative accuracy for the 1e-4 absolute output bound (d out / d ln v =
// 20 / (100 ln 10) = 0.087), and fp32 keeps ~1e-7.
__device__ __forceinline__ float normalise(float v) {
  const float db = 20.0f * log10f(fmaxf(1e-5f, v)) - 16.0f;   // min_level = exp(-100/20 ln 10)
  return fminf(fmaxf((db + 100.0f) * 0.01f, 0.0f), 1.0f);
}

// 2 waves per SIMD: the per-wave frame loop keeps the window, the prefetched next frame
// and the hoisted twiddles in registers (256 VGPRs).  Measured on MI355X (44k frames):
// 0.116 / 0.173 ms (stft / spmel) vs 0.13 / 0.17 ms for one frame per wave at 5 waves per
// SIMD and 0.5 ms for the first version (radix-4 Stockham over the workgroup, fp64 sincos
// per butterfly).
constexpr int kWavesPerEU = 2;

constexpr int kMaxMels = 128;    // n_mels limit of the LDS-staged sparse basis
constexpr int kMaxNnz = 2048;    // basis nonzeros staged in LDS (librosa 80-mel: 941)
struct MelLDS {
  int* lo;
  int* len;
  int* woff;
  float* w;
};

// Everything after windowing for one frame: the three radix-8 passes, the real-transform
// unpack, |X|, and the stft row or the mel / log / clip row.  a[j] = windowed z[l + 64 j].
__device__ __forceinline__ void frame_body(cd (&a)[8], int lane, double* __restrict__ Re, double* __restrict__ Im,
                                           const MelLDS& ml, const float* __restrict__ mel_w, int n_mels, int mode,
                                           float* __restrict__ out, int64_t f) {
  const avc_c64* TW = kTw1024;
  dft8(a);   // over j (n = l + 64 j) -> k2
  // exchange 1: element (k2, l) at 64 k2 + (l ^ 8 k2)
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    const cd v = k2 ? cmul(a[k2], tw(TW, 2 * lane * k2)) : a[k2];  // W512^{l k2}
    const int ix = 64 * k2 + (lane ^ (8 * k2));
    Re[ix] = v.x;
    Im[ix] = v.y;
  }
  wave_lds_sync();

  // pass 2: the 64-point DFT over l of every k2, as 8 x 8; lane = (k2, l0), l = l0 + 8 l1
  {
    const int k2 = lane >> 3, l0 = lane & 7;
#pragma unroll
    for (int l1 = 0; l1 < 8; ++l1) {
      const int ix = 64 * k2 + ((l0 + 8 * l1) ^ (8 * k2));
      a[l1] = {Re[ix], Im[ix]};
    }
    wave_lds_sync();
    dft8(a);   // -> q
    // exchange 2: element (k2, q, l0) at 64 k2 + 8 ((q + k2) & 7) + ((l0 + q) & 7)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const cd v = q ? cmul(a[q], tw(TW, 16 * l0 * q)) : a[q];     // W64^{l0 q}
      const int ix = 64 * k2 + 8 * ((q + k2) & 7) + ((l0 + q) & 7);
      Re[ix] = v.x;
      Im[ix] = v.y;
    }
  }
  wave_lds_sync();

  // pass 3: lane = (k2, q); the DFT over l0 gives Z[64 p + 8 q + k2], p = 0..7
  {
    const int k2 = lane >> 3, q = lane & 7;
#pragma unroll
    for (int l0 = 0; l0 < 8; ++l0) {
      const int ix = 64 * k2 + 8 * ((q + k2) & 7) + ((l0 + q) & 7);
      a[l0] = {Re[ix], Im[ix]};
    }
    wave_lds_sync();
    dft8(a);
    // exchange 3: Z[k] at k ^ (bit 5 of k moved onto bit 2)
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int k = 64 * p + 8 * q + k2;
      const int ix = k ^ (((k >> 5) & 1) << 2);
      Re[ix] = a[p].x;
      Im[ix] = a[p].y;
    }
  }
  wave_lds_sync();
  auto zat = [&](int k) {
    const int ix = k ^ (((k >> 5) & 1) << 2);
    return cd{Re[ix], Im[ix]};
  };

  // real-transform unpack: E = (Z_k + conj Z_{-k})/2, O = (Z_k - conj Z_{-k})/(2i),
  // X_k = E + W1024^k O for k < 512, X_512 = Re Z_0 - Im Z_0
  float mg[8];
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) {
    const int k = lane + 64 * qq;
    const cd zk = zat(k), zm = zat((kN / 2 - k) & (kN / 2 - 1));
    const cd e = {0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y)};
    const cd o = {0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x)};
    const cd x = cadd(e, cmul(tw(TW, k), o));
    mg[qq] = sqrtf((float)(x.x * x.x + x.y * x.y));
  }
  const cd z0 = zat(0);
  const float mg512 = (float)fabs(z0.x - z0.y);

  if (mode == AUTOVC_FE_STFT) {
    float* o = out + f * kBins;
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) o[lane + 64 * qq] = normalise(mg[qq]);
    if (lane == 0) o[kN / 2] = normalise(mg512);
    return;
  }
  wave_lds_sync();   // every read of Z has completed before the magnitudes overwrite it
  float* Mg = reinterpret_cast<float*>(Re);
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) Mg[lane + 64 * qq] = mg[qq];
  if (lane == 0) Mg[kN / 2] = mg512;
  wave_lds_sync();
  for (int m = lane; m < n_mels; m += 64) {
    const int k0 = ml.lo[m], nk = ml.len[m], wo = ml.woff[m];
    // weights from the workgroup's LDS copy (global only past its capacity); 8 independent
    // loads per round, partial sums combined in a fixed order
    auto wt = [&](int i) { return i < kMaxNnz ? ml.w[i] : mel_w[i]; };
    float acc = 0.f;
    int q = 0;
    for (; q + 8 <= nk; q += 8) {
      float wq[8], mq[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) { wq[r] = wt(wo + q + r); mq[r] = Mg[k0 + q + r]; }
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int r = 0; r < 8; r += 2) { s0 = fmaf(mq[r], wq[r], s0); s1 = fmaf(mq[r + 1], wq[r + 1], s1); }
      acc += s0 + s1;
    }
    for (; q < nk; ++q) acc = fmaf(Mg[k0 + q], wt(wo + q), acc);
    out[f * n_mels + m] = normalise(acc);
  }
  wave_lds_sync();   // the mel reads of Mg are done before the next frame's exchange 1
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kWavesPerEU, kWavesPerEU)))
void stft_mel_kernel(
    const double* __restrict__ wav, const int64_t* __restrict__ wav_off,
    const int64_t* __restrict__ frame_off, int n_utt, int64_t total_frames,
    const int* __restrict__ mel_lo, const int* __restrict__ mel_len,
    const int* __restrict__ mel_woff, const float* __restrict__ mel_w, int n_mels,
    int mode, float* __restrict__ out) {
  // per wave: the 512 complex values as separate re / im float64 arrays (8 KB); reused
  // for the 513 magnitudes of the mel stage.  Each exchange stores through its own
  // XOR/rotate index map so that every 32-lane half of a ds_read_b64 / ds_write_b64
  // touches 32 distinct 8-byte bank slots (bank = (addr/4) % 64).
  __shared__ double zbuf[kWaves][kN];
  __shared__ int s_lo[kMaxMels], s_len[kMaxMels], s_woff[kMaxMels];
  __shared__ float s_w[kMaxNnz];

  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* Re = zbuf[wv];
  double* Im = zbuf[wv] + kN / 2;
  const MelLDS ml{s_lo, s_len, s_woff, s_w};
  if (mode == AUTOVC_FE_SPMEL) {   // the sparse mel basis, once per workgroup, into LDS
    for (int i = threadIdx.x; i < n_mels; i += kThreads) {
      s_lo[i] = mel_lo[i];
      s_len[i] = mel_len[i];
      s_woff[i] = mel_woff[i];
    }
    const int nnz = mel_woff[n_mels - 1] + mel_len[n_mels - 1];
    for (int i = threadIdx.x; i < nnz && i < kMaxNnz; i += kThreads) s_w[i] = mel_w[i];
    __syncthreads();   // before any wave's early exit: every wave of the block reaches it
  }
  // each wave transforms a contiguous run of frames (consecutive frames share 3/4 of
  // their samples), prefetching the next frame's samples while the current one computes
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  const int64_t per = (total_frames + nw - 1) / nw;
  int64_t f = ((int64_t)blockIdx.x * kWaves + wv) * per;
  const int64_t fend = f + per < total_frames ? f + per : total_frames;
  if (f >= fend) return;   // wave-uniform exit; the kernel has no workgroup barrier

  // utterance of the first frame: largest u with frame_off[u] <= f
  int u = 0;
  {
    int hi = n_utt;   // invariant frame_off[u] <= f < frame_off[hi]
    while (hi - u > 1) {
      const int mid = (u + hi) >> 1;
      if (frame_off[mid] <= f) u = mid; else hi = mid;
    }
  }
  int t = (int)(f - frame_off[u]);
  const double* src = wav + wav_off[u];
  int L = (int)(wav_off[u + 1] - wav_off[u]);
  // frame sample n sits at padded position hop*t + n, original index hop*t + n - N/2
  // (make_spect.py:38-42); lane l holds z[l + 64 j] = x[2n'] + i x[2n'+1], n' = l + 64 j
  int nfr = (int)(frame_off[u + 1] - frame_off[u]);
  double hw[16];   // this lane's 16 window values, held for the whole run
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hw[2 * j] = kHann1024[2 * (lane + 64 * j)];
    hw[2 * j + 1] = kHann1024[2 * (lane + 64 * j) + 1];
  }
  double xs[16];
  auto load_frame = [&](const double* s, int tt, int LL) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = kHop * tt + 2 * (lane + 64 * j) - kN / 2;
      xs[2 * j] = s[reflect_idx(p, LL)];
      xs[2 * j + 1] = s[reflect_idx(p + 1, LL)];
    }
  };
  load_frame(src, t, L);
  for (; f < fend; ++f) {
    cd a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = {xs[2 * j] * hw[2 * j], xs[2 * j + 1] * hw[2 * j + 1]};
    if (f + 1 < fend) {   // next frame (wave-uniform bookkeeping), loads in flight during this one
      if (++t == nfr) {
        ++u;
        t = 0;
        nfr = (int)(frame_off[u + 1] - frame_off[u]);
        src = wav + wav_off[u];
        L = (int)(wav_off[u + 1] - wav_off[u]);
      }
      load_frame(src, t, L);
    }
    frame_body(a, lane, Re, Im, ml, mel_w, n_mels, mode, out, f);
    wave_lds_sync();   // this frame's LDS reads are done before the next frame's exchange 1
  }
}

}  // namespace

extern "C" int autovc_stft_mel_f32(const double* wav, const int64_t* wav_off,
                                   const int64_t* frame_off, int n_utt,
                                   int64_t total_frames, const int* mel_lo,
                                   const int* mel_len, const int* mel_woff,
                                   const float* mel_w, int n_mels, int mode,
                                   float* out, hipStream_t stream) {
  AVC_CHECK_ARG(n_utt >= 1, "autovc_stft_mel_f32: n_utt must be >= 1 (got %d)", n_utt);
  AVC_CHECK_ARG(total_frames >= 0, "autovc_stft_mel_f32: negative total_frames");
  AVC_CHECK_ARG(wav && wav_off && frame_off && out, "autovc_stft_mel_f32: null pointer");
  AVC_CHECK_ARG(mode == AUTOVC_FE_SPMEL || mode == AUTOVC_FE_STFT,
                "autovc_stft_mel_f32: unknown mode %d", mode);
  if (mode == AUTOVC_FE_SPMEL)
    AVC_CHECK_ARG(n_mels > 0 && n_mels <= kMaxMels && mel_lo && mel_len && mel_woff && mel_w,
                  "autovc_stft_mel_f32: spmel mode needs the sparse mel basis with 1..%d mel rows", kMaxMels);
  if (total_frames == 0) return avc::kOk;
  AVC_CHECK_ARG(total_frames < (int64_t)INT32_MAX, "autovc_stft_mel_f32: too many frames");
  // one resident wave per slot (kWavesPerEU per SIMD, 256 CUs x 4 SIMDs), >= 2 frames each
  const int64_t waves = std::min<int64_t>((total_frames + 1) / 2, (int64_t)kWavesPerEU * 1024);
  hipLaunchKernelGGL(stft_mel_kernel, dim3((unsigned)((waves + kWaves - 1) / kWaves)), dim3(kThreads), 0,
                     stream, wav, wav_off, frame_off, n_utt, total_frames, mel_lo, mel_len, mel_woff, mel_w,
                     n_mels, mode, out);
  AVC_CHECK_LAUNCH("autovc_stft_mel_f32");
  return avc::kOk;
}
