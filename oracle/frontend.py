"""ORACLE (test infrastructure only) — CPU restatement of the AutoVC mel front end.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (autovc_amd/) never does.

Restates, in numpy float64 exactly as the reference computes it:
  make_spect.py:30-34  Spect.butter_highpass  (scipy.signal.butter order 5, 30 Hz HP)
  make_spect.py:36-48  Spect.pySTFT           (reflect pad, as_strided frames, Hann, |rfft|)
  make_spect.py:51     librosa.filters.mel(16000, 1024, fmin=90, fmax=7600, n_mels=80)
                       (librosa==0.9.1, requirements.txt:1 — absent here; its published
                       Slaney algorithm is restated in `librosa_mel` below)
  make_spect.py:52,68-83,92-94  min_level, per-speaker RandomState dither, mel/log/clip
  librosa.load(sr=16000) on 16 kHz PCM16 = int16 / 32768 as float32 (no resampling)

Pinned: tests/test_oracle_frontend.py checks this restatement against the reference's
own bundled pairs wavs/<spk>/<f>.wav -> spmel/<spk>/<f>.npy (copied under tests/golden/),
bit-exact (max abs diff 0.0).
"""
from __future__ import annotations

import numpy as np
from scipy import signal
from scipy.io import wavfile

FS = 16000
CUTOFF = 30
ORDER = 5
FFT_LENGTH = 1024
HOP_LENGTH = 256
MIN_LEVEL = np.exp(-100 / 20 * np.log(10))


# ---- librosa 0.9.1 (Slaney) mel filterbank, restated -------------------------------
def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        log_t = f >= min_log_hz
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = m >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (m[log_t] - min_log_mel))
    return freqs


def librosa_mel(sr=FS, n_fft=FFT_LENGTH, n_mels=80, fmin=90.0, fmax=7600.0):
    """librosa.filters.mel(..., htk=False, norm='slaney', dtype=float32): (n_mels, 1+n_fft//2)."""
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.linspace(0, float(sr) / 2, 1 + n_fft // 2, endpoint=True)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


# ---- make_spect.py -----------------------------------------------------------------
def butter_highpass():
    nyq = 0.5 * FS
    return signal.butter(ORDER, CUTOFF / nyq, btype="high", analog=False)


def hann_periodic(n=FFT_LENGTH):
    """scipy.signal.get_window('hann', n, fftbins=True) (make_spect.py:46)."""
    return signal.get_window("hann", n, fftbins=True)


def py_stft(x):
    """make_spect.py:36-48 -> (513, n_frames) float64 magnitudes."""
    x = np.pad(x, FFT_LENGTH // 2, mode="reflect")
    noverlap = FFT_LENGTH - HOP_LENGTH
    n_frames = (x.shape[-1] - noverlap) // HOP_LENGTH
    idx = np.arange(n_frames)[:, None] * HOP_LENGTH + np.arange(FFT_LENGTH)[None, :]
    frames = x[idx]
    return np.abs(np.fft.rfft(hann_periodic() * frames, n=FFT_LENGTH).T)


def load_wav(path):
    """librosa.load(path, sr=16000) for 16 kHz PCM16 files: int16 / 32768 -> float32."""
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", wavfile.WavFileWarning)
        sr, data = wavfile.read(path)
    if sr != FS:
        raise ValueError(f"{path}: sample rate {sr} != {FS} (resampling not restated)")
    if data.dtype == np.int16:
        return data.astype(np.float32) / 32768.0
    return data.astype(np.float32)


def preprocess(x, prng):
    """make_spect.py:74-76: filtfilt high-pass, then dither (consumes prng)."""
    b, a = butter_highpass()
    y = signal.filtfilt(b, a, x)
    return y * 0.96 + (prng.rand(y.shape[0]) - 0.5) * 1e-06


# ---- operation-order restatements of the two preprocessing steps --------------------
# The GPU kernel (autovc_amd/csrc/preprocess.hip) follows these loops exactly; they are
# pinned against scipy / numpy themselves (tests/test_oracle_frontend.py), which shows
# that a bit-exact GPU result is attainable (no reassociation anywhere).

def lfilter_df2t(b, a, x, z):
    """scipy.signal.lfilter inner loop (direct form II transposed, a[0] == 1), scalar
    float64 in scipy's operation order: y = z0 + b0 x; z_i = (z_{i+1} + x b_{i+1}) - y a_{i+1};
    z_last = x b_last - y a_last."""
    z = [float(v) for v in z]
    y = np.empty(len(x))
    n = len(b)
    for k, xn in enumerate(np.asarray(x, dtype=np.float64)):
        yn = z[0] + b[0] * xn
        for i in range(n - 2):
            z[i] = z[i + 1] + xn * b[i + 1] - yn * a[i + 1]
        z[n - 2] = xn * b[n - 1] - yn * a[n - 1]
        y[k] = yn
    return y


def filtfilt_restated(x, b=None, a=None):
    """scipy.signal.filtfilt(b, a, x) defaults (make_spect.py:74): odd extension of
    padlen = 3*max(len(a), len(b)) samples computed in x's own dtype, lfilter_zi states
    scaled by each pass's first sample, forward then backward pass."""
    if b is None:
        b, a = butter_highpass()
    x = np.asarray(x)
    n = 3 * max(len(a), len(b))
    ext = np.concatenate((2 * x[0:1] - x[n:0:-1], x, 2 * x[-1:] - x[-2:-(n + 2):-1]))
    zi = signal.lfilter_zi(b, a)
    y = lfilter_df2t(b, a, ext, zi * ext[0:1])
    y = lfilter_df2t(b, a, y[::-1], zi * y[-1:])
    return y[::-1][n:-n]


def mt19937_rand(seed, n):
    """numpy RandomState(seed).rand(n): init_genrand seeding, the 624-word twist,
    tempering, and random_sample's 53-bit doubles (a >> 5, b >> 6)."""
    mt = [seed & 0xFFFFFFFF]
    for i in range(1, 624):
        mt.append((1812433253 * (mt[-1] ^ (mt[-1] >> 30)) + i) & 0xFFFFFFFF)
    words = []
    while len(words) < 2 * n:
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        for v in mt:
            v ^= v >> 11
            v ^= (v << 7) & 0x9D2C5680
            v ^= (v << 15) & 0xEFC60000
            v ^= v >> 18
            words.append(v & 0xFFFFFFFF)
    w = np.asarray(words[: 2 * n], dtype=np.uint64)
    return ((w[0::2] >> 5).astype(np.float64) * 67108864.0 + (w[1::2] >> 6)) / 9007199254740992.0


def spmel_from_wav(wav, mel_basis=None):
    """make_spect.py:78-83 on an already preprocessed wav -> (T, 80) float32."""
    if mel_basis is None:
        mel_basis = librosa_mel().T
    D = py_stft(wav)
    D_mel = np.dot(D.T, mel_basis)
    D_db = 20 * np.log10(np.maximum(MIN_LEVEL, D_mel)) - 16
    return np.clip((D_db + 100) / 100, 0, 1).astype(np.float32)


def stft_from_wav(wav):
    """make_spect.py:84-86 -> (513, T) float32 (reference on-disk layout, NOT transposed)."""
    D = py_stft(wav)
    D_db = 20 * np.log10(np.maximum(MIN_LEVEL, D)) - 16
    return np.clip((D_db + 100) / 100, 0, 1).astype(np.float32)


def speaker_spmels(wav_paths, speaker, mode="spmel"):
    """Whole-speaker restatement of make_spect.py:63-94 for one speaker directory.

    `wav_paths` are that speaker's files; they are processed in sorted order with one
    RandomState(int(speaker[1:])) whose stream every file consumes (also files whose
    output is not kept).  Returns {basename: array}.
    """
    prng = np.random.RandomState(int(speaker[1:]))
    out = {}
    mel_basis = librosa_mel().T
    for p in sorted(wav_paths):
        name = p.replace("\\", "/").rsplit("/", 1)[-1]
        if "mic1" in name:
            continue
        wav = preprocess(load_wav(p), prng)
        key = name[:name.rfind(".")]
        out[key] = spmel_from_wav(wav, mel_basis) if mode == "spmel" else stft_from_wav(wav)
    return out
