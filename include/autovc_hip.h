/*
 * autovc_hip.h — C-ABI of libautovc_hip.so, the MI355X (gfx950) hot path of AutoVC.
 *
 * The reference (sebakeaaen/autovc) has no FFI layer: its hot path is Python calling
 * numpy/ATen/cuDNN.  Each entry point below replaces the reference call named in its
 * comment (file:line in the reference tree); the Python host modules in autovc_amd/
 * keep the reference's Python API and call these through ctypes.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer unless the comment says "host";
 *   - the caller owns every buffer (the library never allocates caller memory);
 *     scratch is passed in as an explicit workspace pointer;
 *   - fp32 everywhere ("f32" suffix); activations are frame-major / channel-last:
 *     a (B, T, C) tensor is contiguous with C fastest ("NTC");
 *   - all work is enqueued on `stream` (hipStream_t); nothing synchronises;
 *   - return 0 on success, < 0 on error; autovc_last_error() (thread-local) says why.
 */
#ifndef AUTOVC_HIP_H_
#define AUTOVC_HIP_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AUTOVC_HIP_ABI_VERSION 1

/* ---------------------------------------------------------------- core */
const char* autovc_last_error(void);
int autovc_abi_version(void);
int autovc_device_sync(void);

/* ---------------------------------------------------------------- front end
 * Replaces make_spect.py:36-48 (Spect.pySTFT) + :51-52,79-86 (mel projection,
 * 20*log10 - 16, clip((.+100)/100, 0, 1)).
 *   wav        : concatenated utterances (after the host filtfilt + dither of
 *                make_spect.py:74-76), float64 as the reference computes it
 *   wav_off    : [n_utt+1] int64 sample offsets
 *   frame_off  : [n_utt+1] int64 frame offsets, frames_u = L_u // 256 + 1
 *   mel_*      : sparse mel basis (librosa Slaney 80x513): per mel m the first bin,
 *                the bin count and the offset of its weights in mel_w; n_mels <= 128
 *                (the basis is staged in LDS per workgroup)
 *   The transform runs in float64 (an fp32 FFT misses the 1e-4 bound on quiet stft
 *   bins of loud frames); magnitudes, mel sums and the dB map in fp32.
 *   out        : (total_frames, n_mels) for AUTOVC_FE_SPMEL,
 *                (total_frames, 513)    for AUTOVC_FE_STFT (frame-major)
 */
#define AUTOVC_FE_SPMEL 0
#define AUTOVC_FE_STFT 1
int autovc_stft_mel_f32(const double* wav, const int64_t* wav_off, const int64_t* frame_off,
                        int n_utt, int64_t total_frames, const int* mel_lo, const int* mel_len,
                        const int* mel_woff, const float* mel_w, int n_mels, int mode,
                        float* out, hipStream_t stream);

/* Replaces make_spect.py:74 (scipy.signal.filtfilt of the make_spect.py:30-34 order-5
 * Butterworth high-pass: odd extension of 18 samples, lfilter_zi initial states, direct
 * form II transposed) and make_spect.py:76 (y * 0.96 + (RandomState(seed).rand(n) - 0.5)
 * * 1e-06), bit-exact with scipy / numpy, for a batch of utterances.
 *   x          : concatenated raw utterances, float32 (x_is_f64 = 0, what load_wav
 *                returns; the odd extension is then computed in float32 like numpy) or
 *                float64; every utterance must be longer than 18 samples (scipy raises)
 *   wav_off    : [n_utt+1] int64 sample offsets (device)
 *   b, a, zi   : HOST arrays, order+1 / order+1 / order doubles (butter + lfilter_zi);
 *                order must be 5 and a[0] == 1
 *   stream_off : [n_streams+1] int64 sample offsets of the dither streams (device): each
 *                stream is one RandomState(seeds[s]) consumed over out[stream_off[s] ..
 *                stream_off[s+1]) in order (a speaker's files in sorted order); seeds
 *                (device, uint32).  n_streams = 0 skips the dither (filtfilt only).
 *   out        : float64, same length as x (may not alias x)
 */
int autovc_preprocess_f64(const void* x, int x_is_f64, const int64_t* wav_off, int n_utt,
                          const double* b, const double* a, const double* zi, int order,
                          const int64_t* stream_off, const unsigned* seeds, int n_streams,
                          double* out, hipStream_t stream);

/* ---------------------------------------------------------------- GEMM (fp32 MFMA)
 * Replaces the ATen/cuDNN GEMMs behind nn.Conv1d (implicit im2col, model_vc_mel.py:28-38),
 * nn.LSTM input projections (model_vc_mel.py:61,90,104) and nn.Linear (:10,106), forward
 * and backward.  C[M,N] (ldc) = sum_k A(m,k) B(k,n) (+ bias1[n] + bias2[n]) (+ C if
 * accumulate).  a_trans=0: A[m*lda+k], 1: A[k*lda+m].  b_trans=0: B[n*ldb+k], 1: B[k*ldb+n].
 * *_conv_T > 0 turns the operand into the im2col view of an NTC activation with T frames
 * per sequence, C channels and first tap offset tap0 (-2 for k=5/pad=2; -1 = "previous
 * frame").  splits > 1 = split-K with a workspace of autovc_gemm_workspace_floats floats
 * (partial slabs, summed in split order by a reduce launch: deterministic).
 */
int64_t autovc_gemm_workspace_floats(int M, int N, int splits);
int autovc_gemm_f32(int M, int N, int K,
                    const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                    const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                    float* C, int64_t ldc, const float* bias1, const float* bias2,
                    int accumulate, int splits, float* workspace, hipStream_t stream);
/* How autovc_gemm_f32 and the fp32 batched GEMMs compute (returns the previous mode):
 * 0 = fp32 MFMA (v_mfma_f32_32x32x2_f32); 1 = bf16 MFMA on each operand's three-plane split
 * (fp32 = hi + mid + lo bf16, exact), the six products above 2^-24 |a b| accumulated as a
 * large and a small partial: an fp32 GEMM to fp32 rounding, on the 16x faster bf16 units. */
int autovc_gemm_set_fp32_x6(int on);
int autovc_gemm_fp32_x6(void);   /* the current mode */
/* The split-K factor autovc_gemm_f32 uses for `requested` (the bf16-plane mode plans its own
 * split for large outputs, never above the request): size the workspace with it. */
int autovc_gemm_f32_splits(int M, int N, int K, int requested);
/* LDS bytes per CU that GEMM launches (fp32 and bf16) leave free from now on (0 = none):
 * their workgroups are padded so that no more of them share a CU than fit beside that
 * reserve — a latency-bound kernel on another stream keeps a slot on every CU. */
int autovc_gemm_set_lds_reserve(int bytes);
/* A stream whose kernels only run on the CUs set in `mask` (n_words 32-bit words, bit i =
 * CU i as hipExtStreamCreateWithCUMask numbers them): throughput work (weight-gradient
 * GEMMs) kept off the CUs a latency-bound recurrence on another stream needs.  No
 * reference counterpart (torch.cuda streams are unmasked). */
int autovc_stream_create_cu_mask(int n_words, const uint32_t* mask, hipStream_t* out);
int autovc_stream_destroy(hipStream_t stream);
/* Gradient-ready marks of the data-parallel step (not in the reference, which is
 * single-device: solver_encoder.py:101,128 / :293-300 backward then step).  The step's
 * backward records an event whenever a group of parameter gradients is complete;
 * autovc_event_record_any adds an event-record node when `stream` is being captured into a
 * hipGraph (so every replay records it) and is hipEventRecord otherwise.  The eager
 * gradient exchange waits on those events (autovc_stream_wait_event) before each bucket's
 * collective, overlapping the exchange with the rest of the backward (autovc_amd/ddp.py). */
int autovc_event_create(hipEvent_t* out);
int autovc_event_destroy(hipEvent_t ev);
int autovc_event_record_any(hipEvent_t ev, hipStream_t stream);
int autovc_stream_wait_event(hipStream_t stream, hipEvent_t ev);
/* Measurement only (no reference counterpart): a one-thread kernel that stores the chip's
 * 100 MHz s_memrealtime clock into *dst when `stream` reaches it — a kernel node inside a
 * captured graph, so a replay's streams can be time-stamped without a tracer (which
 * serialises them). */
int autovc_stamp(uint64_t* dst, hipStream_t stream);
/* Same contract, bf16 compute (BASELINE config 3, "bf16 with fp32 master"): the fp32
 * operands are rounded to bf16 (RNE) as they are staged, v_mfma_f32_32x32x16_bf16
 * accumulates in fp32, C / bias / accumulate stay fp32 — the numerics of a torch.autocast
 * bf16 matmul whose output is kept in fp32. */
int autovc_gemm_bf16_f32(int M, int N, int K,
                         const float* A, int64_t lda, int a_trans, int a_conv_T, int a_conv_C, int a_tap0,
                         const float* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                         float* C, int64_t ldc, const float* bias1, const float* bias2,
                         int accumulate, int splits, float* workspace, hipStream_t stream);
/* autovc_gemm_bf16_f32 with A (src bit 0) and / or B (bit 1) held as bf16 (such an operand
 * plain, its ld in bf16 elements, ld and contiguous dimension multiples of 8): a producer's
 * own bf16 copy (the LSTM backward's dGb = RNE(dG), a per-step bf16 weight copy) read as is —
 * half of that operand's bytes, the same result as autovc_gemm_bf16_f32 on the fp32
 * operand.  The rest as autovc_gemm_bf16_f32
 * (the reference computes these as torch.autocast bf16 matmuls inside nn.LSTM's backward,
 * model_vc_mel.py:115-116,122 under BASELINE config 3). */
int autovc_gemm_bf16src_f32(int M, int N, int K, const void* A, int64_t lda, int a_trans,
                            const void* B, int64_t ldb, int b_trans, int b_conv_T, int b_conv_C, int b_tap0,
                            float* C, int64_t ldc, const float* bias1, const float* bias2,
                            int accumulate, int splits, float* workspace, int src, hipStream_t stream);
/* The split-K count autovc_gemm_bf16_f32 uses for this shape when the caller asks for
 * `requested` splits: large outputs run one workgroup per CU on 256-row tiles with the
 * library's own split (so the workspace must be autovc_gemm_workspace_floats(M, N, returned
 * value) floats), smaller ones keep `requested`. */
int autovc_gemm_bf16_splits(int M, int N, int K, int requested);

/* batch independent GEMMs C_z = A_z B_z (same layouts as autovc_gemm_f32, plain operands,
 * no bias/accumulate/split-K) in one launch; A_z / B_z / C_z start z * (a_bstride,
 * b_bstride, c_bstride) floats after the first.  bf16 != 0: bf16 MFMA operands. */
int autovc_gemm_batched_f32(int batch, int M, int N, int K, const float* A, int64_t lda, int64_t a_bstride,
                            int a_trans, const float* B, int64_t ldb, int64_t b_bstride, int b_trans, float* C,
                            int64_t ldc, int64_t c_bstride, int bf16, hipStream_t stream);

/* ---------------------------------------------------------------- Winograd F(4,5) conv
 * ConvNorm (Conv1d k=5, pad=2, model_vc_mel.py:20-38) as 8 batched GEMMs over 4-frame
 * tiles (0.4 of the im2col multiply-adds).  weights: W (Co,Ci,5) -> out (8,Co,Ci) (flip=0)
 * or (8,Ci,Co) with the kernel reversed (flip=1: the input-gradient correlation).  input:
 * x (B,T,C) rows of ldx -> (8, B*T/4, C), zero outside each sequence.  output: (8,
 * B*T/4, C) -> y (B,T,C) rows of ldy, + bias (nullable).  T and C multiples of 4. */
int autovc_wino5_weights_f32(int Co, int Ci, const float* W, int flip, float* out, hipStream_t stream);
/* Every conv weight transform of a training step in one launch: job j turns W[j] (Co[j],
 * Ci[j], 5) into out[j] by kinds[j]: 0 / 1 = autovc_wino5_weights_f32 with flip 0 / 1,
 * 2 / 3 = autovc_conv_pack_f32's Wf / Wd, 4 / 5 = the same packs as bf16 (RNE); for a 2-D
 * W (Co rows x Ci cols: the LSTM weights) 6 = its bf16 copy, 7 = its transpose (Ci x Co, as
 * autovc_transpose_f32), 8 = the bf16 transpose.  Host arrays of n entries.  Replaces the
 * per-layer transforms of the ConvNorm calls (model_vc_mel.py:20-38) in one Solver step. */
int autovc_conv_weights_batched_f32(int n, const int* kinds, const int* Co, const int* Ci,
                                    const float* const* W, float* const* out, hipStream_t stream);
int autovc_wino5_input_f32(int B, int T, int C, const float* x, int64_t ldx, float* out, hipStream_t stream);
int autovc_wino5_output_f32(int B, int T, int C, const float* Yt, const float* bias, float* y, int64_t ldy,
                            hipStream_t stream);
/* Weight gradient: dy: dy (B,T,C) rows of lddy -> dY~ (8, B*T/4, C) (the output
 * transform's transpose); with M_i = dY~_i^T X~_i (8 batched GEMMs over the tiles),
 * wgrad: M (8,Co,Ci) -> dW (Co,Ci,5) = G^T M, accumulate != 0 adds into dW. */
int autovc_wino5_dy_f32(int B, int T, int C, const float* dy, int64_t lddy, float* out, hipStream_t stream);
int autovc_wino5_wgrad_f32(int Co, int Ci, const float* Mt, float* dW, int accumulate, hipStream_t stream);

/* ---------------------------------------------------------------- BatchNorm1d + act
 * Replaces nn.BatchNorm1d (train/eval) + F.relu / torch.tanh / identity after each
 * ConvNorm (model_vc_mel.py:57,69,100,115,140,151,160,165,167).  y, z are (M=B*T, C)
 * row-major with leading dims.  act: 0 none, 1 relu, 2 tanh.  stats writes the batch
 * mean / biased var and (if given) updates running_mean / running_var (unbiased,
 * momentum) and num_batches_tracked.  fwd: z = act(gamma (y-mean)/sqrt(var+eps) + beta)
 * (+ residual).  bwd: dy from dz (z = the forward output), dgamma/dbeta (+)=.
 * workspace: autovc_bn_workspace_bytes(C) bytes.
 */
#define AUTOVC_ACT_NONE 0
#define AUTOVC_ACT_RELU 1
#define AUTOVC_ACT_TANH 2
int64_t autovc_bn_workspace_bytes(int C);
int autovc_bn_stats_f32(int64_t M, int C, const float* y, int64_t ldy, float* mean, float* var,
                        float* running_mean, float* running_var, float momentum,
                        int64_t* num_batches, void* workspace, hipStream_t stream);
int autovc_bn_act_fwd_f32(int64_t M, int C, const float* y, int64_t ldy, const float* mean,
                          const float* var, const float* gamma, const float* beta, float eps,
                          int act, const float* residual, int64_t ldr, float* z, int64_t ldz,
                          hipStream_t stream);
int autovc_bn_act_bwd_f32(int64_t M, int C, const float* dz, int64_t lddz, const float* z,
                          int64_t ldz, const float* y, int64_t ldy, const float* mean,
                          const float* var, const float* gamma, float eps, int act, float* dy,
                          int64_t lddy, float* dgamma, float* dbeta, int accumulate,
                          void* workspace, hipStream_t stream);

/* ---------------------------------------------------------------- fused Conv-BN stacks
 * The encoder / decoder / postnet stacks (ConvNorm -> BatchNorm1d -> act, x3 / x3 / x5,
 * model_vc_mel.py:49-59,68-69,92-102,113-115,132-169) with every BatchNorm pass folded
 * into the Winograd transforms around it.  Each layer's pre-BN output y is written once;
 * its BatchNorm + activation are applied by the next layer's input transform
 * (input_bn), and its statistics come from the output transform that writes y
 * (output_stats).  Backward: the input-gradient output transform also reduces the
 * previous layer's BatchNorm-backward sums (output_bnbwd), and ONE kernel turns (dz, y)
 * into every consumer of dy — the weight-gradient dY~ transform, the input-gradient input
 * transform and the conv bias sums — without storing dy (bnbwd).
 * Row-block partials: autovc_wino5_rows(B, T) rows x C (x 2) doubles.
 * coef (4 x C floats) = [alpha | shift | mean | invstd], alpha = gamma / sqrt(var + eps),
 * shift = beta - mean alpha: written by autovc_bn_finalize_f32 (train: batch statistics,
 * running stats updated as autovc_bn_stats_f32 does) or autovc_bn_coef_f32 (eval: from
 * running stats).  sums ([C][2]) from autovc_bn_bwd_finalize_f32.  B*T/4 tiles, T, C % 4 == 0. */
int64_t autovc_wino5_rows(int B, int T);
int autovc_wino5_input_bn_f32(int B, int T, int C, const float* y, int64_t ldy, const float* coef, int act,
                              float* out, hipStream_t stream);
int autovc_wino5_output_stats_f32(int B, int T, int C, const float* Yt, const float* bias, float* y,
                                  int64_t ldy, double* part, hipStream_t stream);
int autovc_wino5_output_bnbwd_f32(int B, int T, int C, const float* Yt, const float* yprev, int64_t ldy,
                                  const float* coef, int act, float* dz, int64_t lddz, double* part,
                                  hipStream_t stream);
int autovc_wino5_bnbwd_f32(int B, int T, int C, const float* dz, int64_t lddz, const float* y, int64_t ldy,
                           const float* coef, int act, const float* sums, float* Dt, float* Xt,
                           double* bias_part, hipStream_t stream);
int autovc_bn_finalize_f32(int RS, int64_t M, int C, const double* part, const float* gamma, const float* beta,
                           float eps, float* mean, float* var, float* coef, float* running_mean,
                           float* running_var, float momentum, int64_t* num_batches, hipStream_t stream);
int autovc_bn_coef_f32(int C, const float* mean, const float* var, const float* gamma, const float* beta,
                       float eps, float* coef, hipStream_t stream);
/* The BatchNorm-backward sums of a stack's LAST layer, whose dz comes from outside the
 * stack: kRowSplits-row partials (autovc_bn_partial_rows(M) rows) over dz and z. */
int autovc_bn_partial_rows(int64_t M);
int autovc_bn_bwd_partial_f32(int64_t M, int C, const float* dz, int64_t lddz, const float* z, int64_t ldz,
                              const float* y, int64_t ldy, const float* mean, int act, double* part,
                              hipStream_t stream);
int autovc_bn_bwd_finalize_f32(int RS, int C, const double* part, const float* var, float eps, float* sums,
                               float* dgamma, float* dbeta, int accumulate, hipStream_t stream);
/* autovc_bn_bwd_finalize_f32 and, in the same launch, autovc_colsum_f64_finalize_f32 of the
 * previous (deeper) layer's conv bias partials (RSb rows x Cb, fp64) into db — the Conv-BN
 * stack backward's two per-layer finalizes as one launch (model_vc_mel.py:49-59,132-169
 * backward: BatchNorm1d's and the Conv1d bias's gradients). */
int autovc_bn_bwd_finalize_bias_f32(int RS, int C, const double* part, const float* var, float eps, float* sums,
                                    float* dgamma, float* dbeta, int accumulate, int RSb, int Cb,
                                    const double* bias_part, float* db, int acc_b, hipStream_t stream);
int autovc_colsum_f64_finalize_f32(int RS, int C, const double* part, float* out, int accumulate,
                                   hipStream_t stream);

/* The same stacks under precision("bf16") (BASELINE config 3), where the convs are bf16
 * im2col GEMMs (autovc_gemm_bf16_f32's conv operand forms; Ci, Co % 4 == 0):
 *   fwd: y (B*T, Co) = conv(act(x * alpha + shift)) + bias — x is the previous layer's
 *        pre-BN output and x_coef its coef (null: x used as is, the stack's first layer);
 *        part (autovc_bnconv_stats_rows(B*T) x Co x 2 doubles) = its raw (sum y, sum y^2)
 *        partials for autovc_bn_finalize_f32;
 *   dx:  dz (B*T, Ci) = conv^T(dy); with y_prev (the previous layer's pre-BN output) also
 *        part = that layer's BatchNorm-backward sums for autovc_bn_bwd_finalize_f32;
 *   dw:  dWf (Co, 5 Ci) = dy^T im2col(act(x * alpha + shift)) (autovc_conv_unpack_grad_f32
 *        turns it into (Co, Ci, 5));
 *   autovc_bn_dy_f32: dy (M, C) of a layer from (dz, y, coef, sums) — BatchNorm and
 *        activation backward — and its conv bias partials (autovc_bn_partial_rows(M) x C
 *        doubles, for autovc_colsum_f64_finalize_f32).
 * src: bit 0 = the activation operand (x / dy), bit 1 = the other (Wf / Wd / x) is a bf16
 * copy in memory (2-byte elements; Ci, Co % 8 == 0): the producers' bf16 copies
 * (autovc_bn_apply_bf16, autovc_bn_dy_f32's dy_bf16, kind 4 / 5 weight packs) are staged as
 * they are.  A BatchNorm-on-load operand (x_coef) is fp32.  dx: src 0 or 3.
 * workspace: autovc_bnconv_workspace_floats(B, T, Ci, Co) floats (split-K slabs). */
int autovc_bnconv_stats_rows(int64_t M);
int64_t autovc_bnconv_workspace_floats(int B, int T, int Ci, int Co);
int autovc_bnconv_fwd_bf16_f32(int B, int T, int Ci, int Co, const void* x, const float* x_coef, int x_act,
                               const void* Wf, const float* bias, float* y, double* part, int src, float* workspace,
                               hipStream_t stream);
int autovc_bnconv_dx_bf16_f32(int B, int T, int Co, int Ci, const void* dy, const void* Wd, float* dz,
                              const float* y_prev, const float* coef_prev, int act_prev, double* part, int src,
                              float* workspace, hipStream_t stream);
int autovc_bnconv_dw_bf16_f32(int B, int T, int Co, int Ci, const void* dy, const void* x, const float* x_coef,
                              int x_act, float* dWf, int src, float* workspace, hipStream_t stream);
int autovc_bn_dy_f32(int64_t M, int C, const float* dz, const float* y, const float* coef, int act,
                     const float* sums, float* dy, void* dy_bf16, double* bias_part, hipStream_t stream);
/* z (M, C) bf16 = act(y * alpha + shift): the bf16 copy of a stack layer's output read by
 * the next layer's bf16-source GEMMs (C % 4 == 0). */
int autovc_bn_apply_bf16(int64_t M, int C, const float* y, const float* coef, int act, void* z,
                         hipStream_t stream);

/* ---------------------------------------------------------------- LSTM recurrences
 * Replaces the cuDNN/mkldnn recurrence of nn.LSTM (model_vc_mel.py:61,90,104).
 * gx = x W_ih^T + b_ih + b_hh precomputed (autovc_gemm_f32).  Large H (multiple of 16):
 * one launch per step; h written at h[b*h_ldb + t*h_ldt + j]; c_all (B,T,H); gates
 * (B,T,4H) post-activation [i|f|g|o] (null in inference).  Backward produces dG (B,T,4H)
 * (pre-activation gate grads) from dh_out using W_hh^T (H,4H); workspace of
 * autovc_lstm_bwd_workspace_floats floats.  Small H (=32, encoder BLSTM): whole sequence
 * in one launch, ndir directions, gx (B,T,ndir*4H), h/c (B,T,ndir*H), W_hh (4H,H) per direction.
 */
int autovc_lstm_fwd_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                        const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                        float* gates, int reverse, hipStream_t stream);
/* Two stacked large-H layers (nn.LSTM(I, H, num_layers=2), decoder lstm2,
 * model_vc_mel.py:104,118) as a wavefront: launch t runs layer 0 step t and layer 1 step
 * t-1 (T+1 launches).  gx0 = x W_ih0^T + b_ih0 + b_hh0 precomputed (strides as above);
 * layer 1's input projection h0_t W_ih1^T runs inside its step (first K segment);
 * h0/h1, c0/c1 (B,T,H) contiguous; gates0/gates1 (B,T,4H) or null.  Same arithmetic as
 * two autovc_lstm_fwd_f32 calls with the layer-1 projection GEMM in between. */
int autovc_lstm2_fwd_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                         const float* W_hh0, const float* b_ih1, const float* b_hh1, const float* W_ih1,
                         const float* W_hh1, float* h0, float* c0, float* gates0, float* h1, float* c1,
                         float* gates1, hipStream_t stream);
/* bf16 recurrences (precision "bf16", BASELINE config 3): as autovc_lstm_fwd_f32 /
 * autovc_lstm2_fwd_f32 / autovc_lstm_bwd_f32, but the recurrent products read bf16
 * (uint16_t bit patterns, RNE-rounded) copies of the weights — W_hh (4H,H), W_ih1 (4H,H),
 * W_hh^T (H,4H) — and of h / dG, which the step kernels write alongside their fp32
 * outputs (h_b (B,T,H), dG_b (B,T,4H)); cell math, c, gates, h, dG stay fp32.  h
 * contiguous (B,T,H); H a multiple of 128. */
int autovc_lstm_fwd_bf16(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                         const uint16_t* W_hh_b, float* h, uint16_t* h_b, float* c_all, float* gates,
                         int reverse, hipStream_t stream);
int autovc_lstm2_fwd_bf16(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                          const uint16_t* W_hh0_b, const float* b_ih1, const float* b_hh1,
                          const uint16_t* W_ih1_b, const uint16_t* W_hh1_b, float* h0, uint16_t* h0_b,
                          float* c0, float* gates0, float* h1, uint16_t* h1_b, float* c1, float* gates1,
                          hipStream_t stream);
int autovc_lstm_bwd_bf16(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                         const float* gates, const float* c_all, const uint16_t* W_hh_T_b, float* dG,
                         uint16_t* dG_b, int reverse, int splits, float* workspace, hipStream_t stream);
/* autovc_lstm2_bwd_f32 with the recurrent products on bf16 copies: W*T_b are RNE copies of
 * the (H, 4H) transposes; the steps also write dG1_b / dG0_b (B,T,4H) bf16 beside the fp32
 * dG1 / dG0.  H a multiple of 128, splits 2 or 4, workspace of
 * autovc_lstm2_bwd_workspace_floats floats. */
int autovc_lstm2_bwd_bf16(int B, int T, int H, const float* dh1_out, int64_t d_ldb, int64_t d_ldt,
                          const float* gates1, const float* c1, const float* gates0, const float* c0,
                          const uint16_t* W_hh1_T_b, const uint16_t* W_ih1_T_b, const uint16_t* W_hh0_T_b,
                          float* dG1, uint16_t* dG1_b, float* dG0, uint16_t* dG0_b, int splits, float* workspace,
                          hipStream_t stream);
/* autovc_lstm2_fwd_f32 with every launch timed by its own dispatch events; synchronises;
 * *avg_us (HOST pointer) = mean kernel time of launches 2..T-1 (bench.py roofline). */
int autovc_lstm2_fwd_timed_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                               const float* W_hh0, const float* b_ih1, const float* b_hh1, const float* W_ih1,
                               const float* W_hh1, float* h0, float* c0, float* gates0, float* h1, float* c1,
                               float* gates1, hipStream_t stream, float* avg_us);
/* autovc_lstm2_fwd_f32 as ONE persistent, weight-stationary launch (csrc/lstm2_persist.hip):
 * each workgroup (one per CU, 8 waves) owns all B = 64 rows x 16 gate columns (4 hidden
 * units) of both layers and keeps their W_hh0 / W_ih1 tiles in LDS and W_hh1 fragments in
 * VGPRs for the whole sequence; the T + 1 wavefront iterations are separated by an
 * XCD-hierarchical grid barrier.  Same arguments and outputs as autovc_lstm2_fwd_f32
 * (model_vc_mel.py:104,118) plus a workspace of autovc_lstm2_persist_workspace_bytes bytes
 * (barrier words + k-blocked copies of h0 / h1), 16-byte aligned, re-initialised by every
 * call.  Only where autovc_lstm2_persist_supported(B, H) (H = 1024, B = 64, H/4 workgroups
 * all resident at once); else -1.  Every spin is bounded: autovc_lstm2_persist_status(
 * workspace, stream) (synchronising) returns non-zero if the last call's barriers timed out. */
int64_t autovc_lstm2_persist_workspace_bytes(int B, int T, int H);
int autovc_lstm2_persist_supported(int B, int H);
int autovc_lstm2_fwd_persist_f32(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                 const float* W_hh0, const float* b_ih1, const float* b_hh1,
                                 const float* W_ih1, const float* W_hh1, float* h0, float* c0, float* gates0,
                                 float* h1, float* c1, float* gates1, void* workspace, hipStream_t stream);
/* autovc_lstm2_fwd_bf16 (precision "bf16") the same way: bf16 weight copies, bf16 hand-off
 * copies of h inside the workspace (autovc_lstm2_persist_workspace_bytes), fp32 outputs;
 * H = 1024, B = 64 where autovc_lstm2_persist_supported holds (the bf16 kernel needs less LDS). */
int autovc_lstm2_fwd_persist_bf16(int B, int T, int H, const float* gx0, int64_t gx_ldb, int64_t gx_ldt,
                                  const uint16_t* W_hh0_b, const float* b_ih1, const float* b_hh1,
                                  const uint16_t* W_ih1_b, const uint16_t* W_hh1_b, float* h0, float* c0,
                                  float* gates0, float* h1, float* c1, float* gates1, void* workspace,
                                  hipStream_t stream);
/* One large-H layer (decoder lstm1, model_vc_mel.py:90,111) the same way: arguments and
 * outputs of autovc_lstm_fwd_f32 (forward direction) plus a workspace of
 * autovc_lstm_persist_workspace_bytes bytes; H = 512 or 1024, B = 64
 * (autovc_lstm_persist_supported); autovc_lstm2_persist_status reads its barrier words too. */
int64_t autovc_lstm_persist_workspace_bytes(int B, int T, int H);
int autovc_lstm_persist_supported(int B, int H);
int autovc_lstm_fwd_persist_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                                const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                                float* gates, void* workspace, hipStream_t stream);
int autovc_lstm2_persist_status(const void* workspace, hipStream_t stream);
/* One large-H layer (decoder lstm1, model_vc_mel.py:90,111) as ONE persistent launch whose
 * synchronisation stays inside each XCD: XCD x owns batch rows 8x .. 8x+7 (independent
 * sequences), its 32 workgroups each hold W_hh's 4 x 16 columns for 16 units in registers,
 * and per step only those rows' h_{t-1} moves, through the XCD's L2, behind a per-XCD step
 * counter.  Arguments and outputs of autovc_lstm_fwd_f32 (forward direction) plus a
 * workspace of autovc_lstm_xcd_workspace_bytes() bytes (barrier words, re-initialised by
 * every call).  Only where autovc_lstm_xcd_supported(B, H): B = 64, H = 512 on 8 XCDs x 32
 * CUs.  A group that cannot run its 32 workgroups together times out into the fault path
 * of autovc_fault_status. */
int autovc_lstm_xcd_supported(int B, int H);
int64_t autovc_lstm_xcd_workspace_bytes(void);
int autovc_lstm_fwd_xcd_f32(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                            const float* W_hh, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                            float* gates, void* workspace, hipStream_t stream);
/* precision "bf16": the same launch on the RNE bf16 copy of W_hh and bf16-rounded h in the
 * recurrent product (autovc_lstm_fwd_bf16's numerics; fp32 accumulation, cell math and
 * outputs). */
int autovc_lstm_fwd_xcd_bf16(int B, int T, int H, const float* gx, int64_t gx_ldb, int64_t gx_ldt,
                             const uint16_t* W_hh_b, float* h, int64_t h_ldb, int64_t h_ldt, float* c_all,
                             float* gates, void* workspace, hipStream_t stream);
/* The same layer's backward (BPTT, model_vc_mel.py:90,111 under autograd) as one XCD-local
 * launch: arguments and outputs of autovc_lstm_bwd_f32 (WT = W_hh^T (H, 4H), dG (B,T,4H))
 * without its split count / workspace, plus the autovc_lstm_xcd_workspace_bytes() workspace.
 * Per step only the group's 8 rows of dG_{t+1} move, through the XCD's L2.  The bf16 form
 * is autovc_lstm_bwd_bf16's numerics (RNE bf16 W_hh^T and dG in the product, fp32 cell
 * math) and writes dGb, the bf16 copy of dG, which it also exchanges.  Same shapes and
 * fault path as the forward. */
int autovc_lstm_bwd_xcd_f32(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                            const float* gates, const float* c_all, const float* WT, float* dG,
                            void* workspace, hipStream_t stream);
int autovc_lstm_bwd_xcd_bf16(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                             const float* gates, const float* c_all, const uint16_t* WT_b, float* dG,
                             uint16_t* dGb, void* workspace, hipStream_t stream);
/* Co-residency failures reach the caller without a per-call sync: a persistent launch
 * whose grid barrier timed out writes NaN over the h / c it owns (so the loss turns NaN)
 * and sets bit 0 of a sticky per-device fault word.  autovc_fault_status (synchronises
 * `stream`) returns the word in *out and resets it when clear != 0; the Solver and
 * bench.py check it at their sync points and raise.  No reference counterpart (the
 * reference's nn.LSTM has no grid barrier). */
int autovc_fault_status(hipStream_t stream, int clear, int* out);
/* Test hook: the persistent launches' spin budget in s_memrealtime ticks (100 MHz); 0
 * restores the default of 1 s.  A tiny value forces the timeout path. */
int autovc_lstm_persist_set_timeout_ticks(int ticks);
/* autovc_lstm_fwd_f32 with every step launch timed by its own dispatch events;
 * synchronises; *avg_us (HOST pointer) = mean kernel time of steps 1..T-1 (bench.py). */
int autovc_lstm_fwd_timed_f32(int B, int T, int H, const float* gx, int64_t gx_ldb,
                              int64_t gx_ldt, const float* W_hh, float* h, int64_t h_ldb,
                              int64_t h_ldt, float* c_all, float* gates, hipStream_t stream,
                              float* avg_us);
int64_t autovc_lstm_bwd_workspace_floats(int B, int H, int splits);
/* The large-H backward steps (autovc_lstm_bwd_f32 / _bf16, autovc_lstm2_bwd_f32 / _bf16 at
 * splits 2 / 4) run ONE launch per step by default: the split-K product jobs of each
 * 32 x 32 output tile hand their partials over write-through and the last to arrive runs
 * the tile's pointwise cell backward (bit-identical to the product + pointwise launch
 * pair).  on = 0 selects the launch pair, 1 the fused step, -1 the environment's choice
 * (AVC_LSTM_BWD_FUSED=0: the pair).  A/B and test hook; no reference counterpart. */
int autovc_lstm_bwd_set_fused(int on);
int autovc_lstm_bwd_f32(int B, int T, int H, const float* dh_out, int64_t d_ldb, int64_t d_ldt,
                        const float* gates, const float* c_all, const float* W_hh_T, float* dG,
                        int reverse, int splits, float* workspace, hipStream_t stream);
/* Backward of the two stacked layers of decoder lstm2 (nn.LSTM(512, 1024, 2),
 * model_vc_mel.py:104,118 — replaces torch's BPTT of both layers plus the input-gradient
 * GEMM between them) as a one-step-lagged wavefront: 2(T+1) launches, layer 1's input
 * gradient dG1_t W_ih1 computed inside its step as layer 0's dh_t.  W_*_T are the (H, 4H)
 * transposes of W_hh1, W_ih1 (layer 1's input size is H) and W_hh0; dh1_out = dL/dh1;
 * dG1 / dG0 out (B, T, 4H); splits 2 or 4; workspace of
 * autovc_lstm2_bwd_workspace_floats floats.  fp32 only. */
int64_t autovc_lstm2_bwd_workspace_floats(int B, int H, int splits);
int autovc_lstm2_bwd_f32(int B, int T, int H, const float* dh1_out, int64_t d_ldb, int64_t d_ldt,
                         const float* gates1, const float* c1, const float* gates0, const float* c0,
                         const float* W_hh1_T, const float* W_ih1_T, const float* W_hh0_T, float* dG1,
                         float* dG0, int splits, float* workspace, hipStream_t stream);
int autovc_blstm_fwd_f32(int B, int T, int H, int ndir, const float* gx, const float* W_hh_f,
                         const float* W_hh_b, float* h, float* c_all, float* gates,
                         hipStream_t stream);
int autovc_blstm_bwd_f32(int B, int T, int H, int ndir, const float* dh_out, const float* gates,
                         const float* c_all, const float* W_hh_f, const float* W_hh_b, float* dG,
                         hipStream_t stream);

/* ---------------------------------------------------------------- bottleneck / glue
 * frame_concat: out[b,t] = [X[b, t/rep] (C1), E[b] (C2)]  — encoder input
 *   (model_vc_mel.py:64-66, rep=1) and decoder input (code up-sample ++ c_trg, :186-192,
 *   rep=freq).  code_gather: codes[b,k] = [h_fwd[b,k*freq+freq-1], h_bwd[b,k*freq]]
 *   (model_vc_mel.py:74-79; exact copies; bwd = exact inverse scatter).
 */
int autovc_frame_concat_f32(int B, int T, int C1, int C2, int rep, const float* X, int64_t ldx,
                            const float* E, float* out, hipStream_t stream);
int autovc_frame_concat_bwd_f32(int B, int T, int C1, int C2, int rep, const float* dout,
                                float* dX, int64_t ldx, float* dE, int accumulate,
                                hipStream_t stream);
int autovc_code_gather_f32(int B, int T, int D, int freq, const float* h, float* codes,
                           hipStream_t stream);
int autovc_code_gather_bwd_f32(int B, int T, int D, int freq, const float* dcodes, float* dh,
                               hipStream_t stream);

/* ---------------------------------------------------------------- losses / optimiser
 * loss kind 0 = F.mse_loss, 1 = F.l1_loss (mean), solver_encoder.py:230,233,236; the
 * scalar stays on the device.  adam: torch.optim.Adam step (solver_encoder.py:130,300)
 * over one flat fp32 buffer of every parameter.
 */
int64_t autovc_loss_workspace_bytes(void);
int autovc_loss_f32(int kind, int64_t n, const float* a, const float* b, float* out,
                    void* workspace, hipStream_t stream);
int autovc_loss_bwd_f32(int kind, int64_t n, const float* a, const float* b, const float* gout,
                        float* ga, float* gb, int acc_a, int acc_b, hipStream_t stream);
int autovc_adam_f32(int64_t n, float* p, const float* g, float* m, float* v, float lr,
                    float beta1, float beta2, float eps, float weight_decay,
                    float bias_correction1, float bias_correction2_sqrt, hipStream_t stream);

/* ---------------------------------------------------------------- layout helpers */
int autovc_conv_pack_f32(int Co, int Ci, int K, const float* W, float* Wf, float* Wd,
                         hipStream_t stream);
int autovc_conv_unpack_grad_f32(int Co, int Ci, int K, const float* dWf, float* dW,
                                int accumulate, hipStream_t stream);
int autovc_transpose_f32(int R, int C, const float* in, float* out, hipStream_t stream);
/* row-wise L2 normalisation: the D-VECTOR speaker encoder's embeds / ||embeds|| (model_bl.py:17-19) */
int autovc_l2norm_rows_f32(int M, int N, const float* x, int64_t ldx, float* out, int64_t ldo,
                           hipStream_t stream);
int64_t autovc_colsum_workspace_floats(int N);
int autovc_colsum_f32(int64_t M, int N, const float* X, int64_t ld, float* out, float* out2,
                      int accumulate, float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------- WaveNet vocoder
 * Replaces wavenet_vocoder 0.1.1 WaveNet.incremental_forward as called by
 * synthesis.py:67-69 (third-party, absent from the reference tree; restated in
 * oracle/wavenet.py, parity unpinned).
 *
 * upsample: the upsample_conv stack (n_stages x [ConvTranspose2d(1,1,(3,s),stride (1,s),
 *   pad (1,0)) + ReLU], hparams.py:110-114).  c (B, C, Tc) as wavegen builds it
 *   (synthesis.py:57), w = per-stage (3, s) kernels concatenated, bias[n_stages];
 *   out (Tc*prod(s), B, C) time-major.
 *
 * generate: runs sample steps t0 <= t < t1 of the incremental loop for B utterances.
 *   packed   weights after make_generation_fast_ (weight norm folded), floats:
 *              first_conv w[R], b[R];
 *              per layer l: gate block (G, taps*R + G/2) = [W_0 .. W_(taps-2) linearised
 *                         (o, tap, i) | sqrt(.5) W_(taps-1) W_out(l-1) (G/2) | sqrt(.5) W_(taps-1) (R)]
 *                         (layer 0: [W_0 .. W_(taps-2) | 0 | W_(taps-1)]) — the current tap folded
 *                         back one layer so each layer is one launch;
 *                         [conv1x1_out (R, G/2); conv1x1_skip (S, G/2)], their biases [R+S];
 *              last_conv_layers.1 W (S, S), b[S]; last_conv_layers.3 W (n_out, S), b[n_out]
 *            (autovc_wavenet_packed_floats gives the size; autovc_amd/wavenet.py builds it)
 *   pre      (Tch, B, n_layers*G): conditioning 1x1 + both biases of every layer (+ the folded
 *            sqrt(.5) W_(taps-1) b_out(l-1) for l >= 1); row
 *            (t % Tch) must hold step t (one autovc_gemm_f32 over the upsampled c per chunk)
 *   seed, utt_base: Philox4x32-10 key and the global index of utterance 0 (the draw of
 *            sample t of utterance u depends only on (seed, u, t))
 *   teacher  optional (B, teacher_len): the input at step t < teacher_len (test_inputs)
 *   y_out    (B, T) samples; mol_out optional (B, T, n_out) head outputs
 *   workspace autovc_wavenet_workspace_bytes; zeroed by the call with t0 == 0 and carried
 *            to the following chunks
 *   graph_steps > 0: runs of that many steps that stay inside one conditioning chunk replay
 *            a captured hipGraph, one per (ring slot, chunk row) of the run's first step
 *            (cached, at most 16): every kernel argument of a step, ring slot and
 *            conditioning row included, is static in it, so no step kernel waits on a
 *            counter read.  Keep Tch a small multiple of graph_steps and of the ring
 *            (autovc_amd/wavenet.py: Tch = lcm(ring, graph_steps)) so a few graphs serve
 *            every chunk.  The other steps, and graph_steps = 0, launch directly.
 *   autovc_wavenet_ring_frames: frames of the per-layer input rings (power of two >=
 *            (taps-1) * max dilation + 1).
 */
/* Persistent generation (B <= 8, R = 512, G = 512, S = 256, 3 taps, a 256-CU device): ONE
 * launch per autovc_wavenet_generate_f32 call, same arguments and outputs, every hand-off a
 * tagged 16-byte write-through granule (dataflow, no grid barrier); a wait that
 * times out poisons the call's samples with NaN and sets bit 2 of the autovc_wavenet_fault word.
 *   layer-pipelined (wn_pipe_kernel, 24 layers): ten CUs per layer hold its current-tap and
 *   residual rows for the whole call; utterances travel through the layers one behind another.
 *   all-CU (wn_grid_kernel, 8..24 layers): every CU holds one gate pair of every layer.
 * Mode (AVC_WN_GRID or autovc_wavenet_set_grid): 0 never (per-layer launches), 1 all-CU for
 * every eligible batch, 2 all-CU for B <= 2, 3 (the default) layer-pipelined for every eligible
 * batch (other shapes run the launches); any other AVC_WN_GRID value makes
 * autovc_wavenet_generate_f32 fail.  autovc_wavenet_grid_explicit: 1 if the mode was chosen
 * (AVC_WN_GRID set or autovc_wavenet_set_grid called), 0 for the library default — the Python
 * layer regenerates on the launches with a warning when a DEFAULT-mode persistent call times
 * out, and raises when the mode was chosen; autovc_wavenet_reset_grid restores the default (3,
 * not chosen).  autovc_wavenet_last_path: 2 if the last generate call ran the layer-pipelined
 * kernel, 1 the all-CU kernel (for both the caller must read autovc_wavenet_fault), 0 the
 * per-layer launches. */
int autovc_wavenet_set_grid(int on);
int autovc_wavenet_get_grid(void);
int autovc_wavenet_grid_explicit(void);
int autovc_wavenet_reset_grid(void);
int autovc_wavenet_last_path(void);
/* The first wait of the all-CU generation that timed out since the last clear: out5 = {kind
 * (0 none, 1 layer inputs, 2 past-tap sums, 3 LDS handshake, 4 past-tap inputs, 5 past-tap
 * consumers, 6 skip sums, 7 h1), step, phase (or job), workgroup, last tag seen (-1 if not
 * recorded)}; synchronises the device. */
int autovc_wavenet_grid_diag(int clear, int* out5);
/* The all-CU generation's spin budget per wait in s_memrealtime ticks (0 = 1 s; a tiny value
 * forces the timeout path in tests) and its sticky fault word (bit 2: a wait timed out and the
 * call's samples are NaN); autovc_wavenet_fault synchronises, clear != 0 resets it. */
int autovc_wavenet_set_timeout_ticks(int ticks);
int autovc_wavenet_fault(int clear, int* out);
int64_t autovc_wavenet_ring_frames(int n_layers, int layers_per_stack, int taps);
int64_t autovc_wavenet_packed_floats(int n_layers, int taps, int R, int G, int S, int n_out);
int64_t autovc_wavenet_workspace_bytes(int B, int T, int n_layers, int layers_per_stack, int taps,
                                       int R, int G, int S);
int autovc_wavenet_upsample_f32(int B, int Tc, int C, int n_stages, const int* scales /* host */,
                                const float* c, const float* w, const float* bias, float* out,
                                hipStream_t stream);
int autovc_wavenet_generate_f32(int B, int T, int t0, int t1, int n_layers, int layers_per_stack,
                                int taps, int R, int G, int S, int n_out, int legacy,
                                const float* packed, const float* pre, int Tch, uint64_t seed,
                                int utt_base, float log_scale_min, const float* teacher,
                                int teacher_len, float* y_out, float* mol_out, void* workspace,
                                int graph_steps, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* AUTOVC_HIP_H_ */
