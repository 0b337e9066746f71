// Fused STFT + mel filterbank + log/normalise front end (gfx950).
//
// Replaces, for a batch of utterances at once:
//   make_spect.py:36-48   Spect.pySTFT  (reflect pad 512, 1024-pt frames at hop 256,
//                                        periodic Hann, |rfft|)
//   make_spect.py:79-83   spmel branch  (D.T @ mel_basis -> 20*log10(max(1e-5, .)) - 16
//                                        -> clip((.+100)/100, 0, 1))
//   make_spect.py:84-86   stft branch   (same without the mel projection)
//
// One workgroup = one frame.  The 1024 windowed samples are read coalesced straight
// from the utterance (reflect padding is an index fold, never materialised), the
// transform is a radix-4 Stockham FFT in LDS (5 stages, one butterfly per thread per
// stage, natural-order output), and the magnitude / sparse mel / log / clip epilogue
// runs from LDS.  Arithmetic is float64 like the reference (numpy pocketfft on the f64
// dithered signal): an fp32 FFT misses the 1e-4 bound on quiet STFT bins of loud
// frames, and f64 costs nothing here (the kernel is bandwidth/latency bound and gfx950
// runs f64 FMA at half the f32 rate).  HBM traffic per frame = 256 new f64 input
// samples (the other 768 are L2 hits from the neighbouring frames) + the f32 output
// row: 2,368 B for spmel.
#include "common.h"
#include "../../include/autovc_hip.h"

namespace {

constexpr int kN = 1024;      // fft_length (make_spect.py:24)
constexpr int kHop = 256;     // hop_length (make_spect.py:25)
constexpr int kBins = kN / 2 + 1;
constexpr int kThreads = 256;

struct cf { double x, y; };

__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }

// numpy.pad(mode='reflect') index fold (edge sample not repeated); handles pads
// longer than the signal the way numpy's iterated reflection does.
__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t L) {
  if (L <= 1) return 0;
  const int64_t P = 2 * (L - 1);
  i %= P;
  if (i < 0) i += P;
  return i < L ? i : P - i;
}

__global__ __launch_bounds__(kThreads) void stft_mel_kernel(
    const double* __restrict__ wav, const int64_t* __restrict__ wav_off,
    const int64_t* __restrict__ frame_off, int n_utt,
    const int* __restrict__ mel_lo, const int* __restrict__ mel_len,
    const int* __restrict__ mel_woff, const float* __restrict__ mel_w, int n_mels,
    int mode, float* __restrict__ out) {
  __shared__ cf buf[2][kN];
  __shared__ double mag[kBins + 3];

  const int64_t f = blockIdx.x;
  const int tid = threadIdx.x;

  // utterance of this frame: largest u with frame_off[u] <= f
  int lo = 0, hi = n_utt;  // invariant frame_off[lo] <= f < frame_off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (frame_off[mid] <= f) lo = mid; else hi = mid;
  }
  const int u = lo;
  const int64_t t = f - frame_off[u];
  const int64_t base = wav_off[u];
  const int64_t L = wav_off[u + 1] - base;

  // windowed frame -> buf[0]; padded index p = hop*t + n, original index p - N/2
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = tid + r * kThreads;
    const int64_t src = reflect_idx(kHop * t + n - kN / 2, L);
    // periodic Hann = scipy get_window('hann', N, fftbins=True)
    const double w = 0.5 - 0.5 * cospi(2.0 * (double)n / (double)kN);
    buf[0][n] = {wav[base + src] * w, 0.0};
  }
  __syncthreads();

  // radix-4 Stockham, Ns = 1, 4, 16, 64, 256
  int src_b = 0;
#pragma unroll
  for (int Ns = 1; Ns < kN; Ns *= 4) {
    const int j = tid;
    const int k = j % Ns;
    cf v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = buf[src_b][j + r * (kN / 4)];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        // exp(-2*pi*i * r*k / (4*Ns)), evaluated in double then rounded
        double s, c;
        sincospi(-2.0 * (double)(r * k) / (double)(4 * Ns), &s, &c);
        v[r] = cmul(v[r], cf{c, s});
      }
    }
    const cf a0 = cadd(v[0], v[2]);
    const cf a1 = csub(v[0], v[2]);
    const cf a2 = cadd(v[1], v[3]);
    const cf d = csub(v[1], v[3]);
    const cf a3 = {d.y, -d.x};  // (v1 - v3) * (-i)
    const int idxD = (j / Ns) * Ns * 4 + k;
    buf[src_b ^ 1][idxD + 0 * Ns] = cadd(a0, a2);
    buf[src_b ^ 1][idxD + 1 * Ns] = cadd(a1, a3);
    buf[src_b ^ 1][idxD + 2 * Ns] = csub(a0, a2);
    buf[src_b ^ 1][idxD + 3 * Ns] = csub(a1, a3);
    src_b ^= 1;
    __syncthreads();
  }

  const double min_level = exp(-100.0 / 20.0 * log(10.0));  // make_spect.py:52
  if (mode == AUTOVC_FE_STFT) {
    for (int kb = tid; kb < kBins; kb += kThreads) {
      const cf z = buf[src_b][kb];
      const double db = 20.0 * log10(fmax(min_level, hypot(z.x, z.y))) - 16.0;
      out[f * kBins + kb] = (float)fmin(fmax((db + 100.0) / 100.0, 0.0), 1.0);
    }
    return;
  }
  for (int kb = tid; kb < kBins; kb += kThreads) {
    const cf z = buf[src_b][kb];
    mag[kb] = hypot(z.x, z.y);
  }
  __syncthreads();
  for (int m = tid; m < n_mels; m += kThreads) {
    const int k0 = mel_lo[m], nk = mel_len[m], wo = mel_woff[m];
    double acc = 0.0;
    for (int q = 0; q < nk; ++q) acc = fma(mag[k0 + q], (double)mel_w[wo + q], acc);
    const double db = 20.0 * log10(fmax(min_level, acc)) - 16.0;
    out[f * n_mels + m] = (float)fmin(fmax((db + 100.0) / 100.0, 0.0), 1.0);
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
    AVC_CHECK_ARG(n_mels > 0 && mel_lo && mel_len && mel_woff && mel_w,
                  "autovc_stft_mel_f32: spmel mode needs the sparse mel basis");
  if (total_frames == 0) return avc::kOk;
  AVC_CHECK_ARG(total_frames < (int64_t)INT32_MAX, "autovc_stft_mel_f32: too many frames");
  hipLaunchKernelGGL(stft_mel_kernel, dim3((unsigned)total_frames), dim3(kThreads), 0, stream,
                     wav, wav_off, frame_off, n_utt, mel_lo, mel_len, mel_woff, mel_w, n_mels,
                     mode, out);
  AVC_CHECK_LAUNCH("autovc_stft_mel_f32");
  return avc::kOk;
}
