// Waveform preprocessing of the front end (gfx950): Butterworth high-pass filtfilt and
// the MT19937 dither, bit-exact with the reference's scipy / numpy host code.
//
// Replaces, for a batch of utterances at once:
//   make_spect.py:30-34  butter_highpass (order 5, 30 Hz, fs 16 kHz; coefficients come
//                        from the host, they are 12 constants)
//   make_spect.py:74     y = signal.filtfilt(b, a, x)   (scipy: padtype 'odd', padlen
//                        3*max(len(a), len(b)) = 18, lfilter_zi initial state scaled by the
//                        first sample of each pass, direct form II transposed)
//   make_spect.py:76     wav = y * 0.96 + (prng.rand(len(y)) - 0.5) * 1e-06 with
//                        prng = RandomState(int(spk[1:])) shared by a speaker's files in
//                        sorted order (make_spect.py:68-70)
//
// filtfilt: one thread per utterance runs the IIR recurrence sequentially in float64 in
// scipy's exact operation order (lfilter's inner loop: y = z0 + b0 x; z_i = (z_{i+1} +
// x b_{i+1}) - y a_{i+1}; z_last = x b_last - y a_last), with FP contraction off, so the
// result equals scipy's to the bit.  A parallel (chunked-scan) formulation would
// reassociate the recurrence and lose that; the recurrence is latency-bound (three
// dependent f64 operations per sample), every utterance of the batch runs concurrently,
// and the loads/stores are batched 8 samples at a time so that HBM latency stays off the
// chain.  The odd extension (2 x0 - x[18-i], in the input's own precision as numpy
// computes it) is an index fold; the forward pass writes the kept samples straight into
// the output and holds the 18 right-pad outputs in registers; the backward pass runs in
// place and stops at the first kept sample (the left-pad outputs are discarded by scipy).
//
// dither: one workgroup per RandomState stream.  The MT19937 state lives in LDS; a twist
// of 624 words runs as the four dependency phases of the sequential update ([0,227),
// [227,454), [454,623), 623) with registers holding each phase's reads; thread k tempers
// word k, and 312 threads form the 53-bit doubles (a >> 5, b >> 6) of numpy's
// random_sample from word pairs (a stream starts at word 0 and consumes 2 words per
// sample, so a pair never straddles two twists) and apply y*0.96 + (u-0.5)*1e-6.
#include "common.h"
#include "../../include/autovc_hip.h"

#pragma clang fp contract(off)

namespace {

constexpr int kOrd = 5;                  // make_spect.py:31 order=5
constexpr int kPad = 3 * (kOrd + 1);     // scipy filtfilt padlen = 3 * max(len(a), len(b))
constexpr int kU = 8;                    // samples per batched load/store group

struct FiltCoef {
  double b[kOrd + 1], a[kOrd + 1], zi[kOrd];
};

struct Df2t {
  double z[kOrd];
  __device__ __forceinline__ double step(const FiltCoef& c, double x) {
    const double y = z[0] + c.b[0] * x;
#pragma unroll
    for (int i = 0; i < kOrd - 1; ++i) z[i] = (z[i + 1] + x * c.b[i + 1]) - y * c.a[i + 1];
    z[kOrd - 1] = x * c.b[kOrd] - y * c.a[kOrd];
    return y;
  }
  __device__ __forceinline__ void init(const FiltCoef& c, double s) {
#pragma unroll
    for (int i = 0; i < kOrd; ++i) z[i] = c.zi[i] * s;
  }
};

template <typename T>
__global__ __launch_bounds__(64) void filtfilt_kernel(const T* __restrict__ x, const int64_t* __restrict__ off,
                                                      int n_utt, FiltCoef c, double* __restrict__ out) {
  const int u = blockIdx.x * 64 + threadIdx.x;
  if (u >= n_utt) return;
  const int64_t o = off[u], n = off[u + 1] - o;
  if (n <= kPad) return;                 // rejected on the host (scipy raises ValueError)
  const T* xs = x + o;
  double* ys = out + o;
  const T x0 = xs[0], xl = xs[n - 1];
  // left odd extension: ext[i] = 2 x0 - x[18 - i], i = 0..17 (in T, as numpy does)
  Df2t f;
  const T e0 = T(2) * x0 - xs[kPad];
  f.init(c, (double)e0);
  {
    T e[kPad];
#pragma unroll
    for (int i = 0; i < kPad; ++i) e[i] = T(2) * x0 - xs[kPad - i];
#pragma unroll
    for (int i = 0; i < kPad; ++i) f.step(c, (double)e[i]);
  }
  // body: ext[18 + k] = x[k] -> forward outputs kept at out[k]
  int64_t k = 0;
  for (; k + kU <= n; k += kU) {
    T v[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) v[j] = xs[k + j];
    double r[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) r[j] = f.step(c, (double)v[j]);
#pragma unroll
    for (int j = 0; j < kU; ++j) ys[k + j] = r[j];
  }
  for (; k < n; ++k) ys[k] = f.step(c, (double)xs[k]);
  // right odd extension: ext[n + 18 + j] = 2 x[n-1] - x[n-2-j]; its outputs stay in registers
  double tail[kPad];
  {
    T e[kPad];
#pragma unroll
    for (int j = 0; j < kPad; ++j) e[j] = T(2) * xl - xs[n - 2 - j];
#pragma unroll
    for (int j = 0; j < kPad; ++j) tail[j] = f.step(c, (double)e[j]);
  }
  // backward pass over the reversed forward output, initial state zi * y[-1]
  Df2t g;
  g.init(c, tail[kPad - 1]);
#pragma unroll
  for (int j = kPad - 1; j >= 0; --j) g.step(c, tail[j]);
  k = n;
  for (; k - kU >= 0; k -= kU) {
    double v[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) v[j] = ys[k - 1 - j];
#pragma unroll
    for (int j = 0; j < kU; ++j) v[j] = g.step(c, v[j]);
#pragma unroll
    for (int j = 0; j < kU; ++j) ys[k - 1 - j] = v[j];
  }
  for (; k > 0; --k) ys[k - 1] = g.step(c, ys[k - 1]);
}

// ------------------------------------------------------------------ MT19937 dither
constexpr int kMtN = 624, kMtM = 397;
constexpr unsigned kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
constexpr int kDitherThreads = 640;      // >= 624, whole waves

__device__ __forceinline__ unsigned mt_mix(unsigned cur, unsigned next, unsigned far) {
  const unsigned y = (cur & kUpper) | (next & kLower);
  return far ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
}

// out[s_off[s] .. s_off[s+1]) = out * 0.96 + (RandomState(seed[s]).rand(len) - 0.5) * 1e-6
__global__ __launch_bounds__(kDitherThreads) void mt_dither_kernel(const int64_t* __restrict__ s_off,
                                                                   const unsigned* __restrict__ seed,
                                                                   double scale, double amp,
                                                                   double* __restrict__ out) {
  __shared__ unsigned mt[kMtN];
  __shared__ unsigned tw[kMtN];
  const int s = blockIdx.x, k = threadIdx.x;
  const int64_t o = s_off[s], len = s_off[s + 1] - o;
  if (k == 0) {                          // numpy mt19937_seed (init_genrand)
    unsigned v = seed[s];
    mt[0] = v;
    for (int i = 1; i < kMtN; ++i) {
      v = 1812433253u * (v ^ (v >> 30)) + (unsigned)i;
      mt[i] = v;
    }
  }
  __syncthreads();
  const int64_t nblk = (2 * len + kMtN - 1) / kMtN;
  for (int64_t blk = 0; blk < nblk; ++blk) {
    // twist: the sequential in-place update as four phases of independent words
    unsigned r = 0;
    if (k < kMtN - kMtM) r = mt_mix(mt[k], mt[k + 1], mt[k + kMtM]);
    __syncthreads();
    if (k < kMtN - kMtM) mt[k] = r;
    __syncthreads();
    if (k >= kMtN - kMtM && k < 2 * (kMtN - kMtM)) r = mt_mix(mt[k], mt[k + 1], mt[k + kMtM - kMtN]);
    __syncthreads();
    if (k >= kMtN - kMtM && k < 2 * (kMtN - kMtM)) mt[k] = r;
    __syncthreads();
    if (k >= 2 * (kMtN - kMtM) && k < kMtN - 1) r = mt_mix(mt[k], mt[k + 1], mt[k + kMtM - kMtN]);
    __syncthreads();
    if (k >= 2 * (kMtN - kMtM) && k < kMtN - 1) mt[k] = r;
    __syncthreads();
    if (k == kMtN - 1) {
      const unsigned w = mt_mix(mt[kMtN - 1], mt[0], mt[kMtM - 1]);
      mt[kMtN - 1] = w;
    }
    __syncthreads();
    if (k < kMtN) {                      // tempering
      unsigned y = mt[k];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      tw[k] = y;
    }
    __syncthreads();
    const int64_t d = blk * (kMtN / 2) + k;
    if (k < kMtN / 2 && d < len) {
      const double a = (double)(tw[2 * k] >> 5), b = (double)(tw[2 * k + 1] >> 6);
      const double uni = (a * 67108864.0 + b) / 9007199254740992.0;
      double* p = out + o + d;
      *p = *p * scale + (uni - 0.5) * amp;
    }
    // the next twist's first barrier orders these tw reads before tw is rewritten
  }
}

}  // namespace

extern "C" int autovc_preprocess_f64(const void* x, int x_is_f64, const int64_t* wav_off, int n_utt,
                                     const double* b, const double* a, const double* zi, int order,
                                     const int64_t* stream_off, const unsigned* seeds, int n_streams,
                                     double* out, hipStream_t stream) {
  AVC_CHECK_ARG(n_utt >= 0 && n_streams >= 0, "autovc_preprocess_f64: negative count");
  if (n_utt == 0) return avc::kOk;
  AVC_CHECK_ARG(x && wav_off && out, "autovc_preprocess_f64: null pointer");
  AVC_CHECK_ARG(order == kOrd, "autovc_preprocess_f64: order %d (only the reference's order %d)", order, kOrd);
  AVC_CHECK_ARG(b && a && zi, "autovc_preprocess_f64: null filter coefficients");
  AVC_CHECK_ARG(a[0] == 1.0, "autovc_preprocess_f64: a[0] must be 1 (normalised filter)");
  AVC_CHECK_ARG(n_streams == 0 || (stream_off && seeds), "autovc_preprocess_f64: null dither stream arrays");
  FiltCoef c;
  for (int i = 0; i <= kOrd; ++i) { c.b[i] = b[i]; c.a[i] = a[i]; }
  for (int i = 0; i < kOrd; ++i) c.zi[i] = zi[i];
  const dim3 grid((unsigned)((n_utt + 63) / 64));
  if (x_is_f64)
    hipLaunchKernelGGL(filtfilt_kernel<double>, grid, dim3(64), 0, stream, static_cast<const double*>(x), wav_off,
                       n_utt, c, out);
  else
    hipLaunchKernelGGL(filtfilt_kernel<float>, grid, dim3(64), 0, stream, static_cast<const float*>(x), wav_off,
                       n_utt, c, out);
  AVC_CHECK_LAUNCH("autovc_preprocess_f64 (filtfilt)");
  if (n_streams > 0) {
    hipLaunchKernelGGL(mt_dither_kernel, dim3((unsigned)n_streams), dim3(kDitherThreads), 0, stream, stream_off,
                       seeds, 0.96, 1e-06, out);
    AVC_CHECK_LAUNCH("autovc_preprocess_f64 (dither)");
  }
  return avc::kOk;
}
