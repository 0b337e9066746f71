"""Host-side DSP constants and the GPU front-end entry (STFT + mel + log/clip).

Host part (constants only): make_spect.py:30-34 butter_highpass coefficients (+ scipy's
  lfilter_zi initial state), make_spect.py:51 the Slaney mel basis (librosa 0.9.1
  `filters.mel`, restated).  `preprocess` is the reference's host filtfilt + dither, kept
  for callers that hold a RandomState object.
GPU part (HIP, libautovc_hip.so):
  make_spect.py:74-76  filtfilt + MT19937 dither, bit-exact (`autovc_preprocess_f64`)
  make_spect.py:36-48  pySTFT + :79-86 mel projection, dB, clip (`autovc_stft_mel_f32`)
"""
from __future__ import annotations

import functools

import numpy as np

from . import _lib

FS = 16000
CUTOFF = 30
ORDER = 5
FFT_LENGTH = 1024
HOP_LENGTH = 256
N_BINS = FFT_LENGTH // 2 + 1
MIN_LEVEL = np.exp(-100 / 20 * np.log(10))


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz,
                    min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)),
                    f_sp * m)


@functools.lru_cache(maxsize=8)
def mel_basis(sr=FS, n_fft=FFT_LENGTH, n_mels=80, fmin=90.0, fmax=7600.0) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) (Slaney, float32): (n_mels, 1+n_fft//2)."""
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.linspace(0, float(sr) / 2, 1 + n_fft // 2, endpoint=True)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, np.newaxis]
    w.setflags(write=False)
    return w


def sparse_mel(basis: np.ndarray):
    """(lo, len, woff, weights) of each mel row's contiguous non-zero bin range."""
    lo, ln, off, ws = [], [], [], []
    o = 0
    for row in basis:
        nz = np.nonzero(row)[0]
        a, b = (int(nz[0]), int(nz[-1]) + 1) if len(nz) else (0, 0)
        lo.append(a)
        ln.append(b - a)
        off.append(o)
        ws.append(row[a:b])
        o += b - a
    return (np.asarray(lo, np.int32), np.asarray(ln, np.int32), np.asarray(off, np.int32),
            np.concatenate(ws).astype(np.float32))


def butter_highpass():
    from scipy import signal
    return signal.butter(ORDER, CUTOFF / (0.5 * FS), btype="high", analog=False)


def preprocess(x: np.ndarray, prng: np.random.RandomState) -> np.ndarray:
    """make_spect.py:74-76 (host): filtfilt high-pass + dither; float64 out."""
    from scipy import signal
    b, a = butter_highpass()
    y = signal.filtfilt(b, a, x)
    return y * 0.96 + (prng.rand(y.shape[0]) - 0.5) * 1e-06


@functools.lru_cache(maxsize=None)
def _filter_consts():
    """(b, a, zi) of make_spect.py:30-34 as contiguous float64 host arrays; zi is
    scipy.signal.lfilter_zi(b, a), the state filtfilt scales by each pass's first sample."""
    from scipy import signal
    b, a = butter_highpass()
    zi = signal.lfilter_zi(b, a)
    return tuple(np.ascontiguousarray(v, dtype=np.float64) for v in (b, a, zi))


PADLEN = 3 * (ORDER + 1)   # scipy filtfilt's default padlen for this filter


def preprocess_gpu(wavs, seeds=None, groups=None, device="cuda"):
    """make_spect.py:74-76 on the GPU for a batch of utterances, bit-exact with scipy/numpy.

    wavs   : list of 1-D raw utterances (float32 as load_wav returns them, or float64;
             one dtype per batch, because numpy computes the odd extension in the input's
             precision).  Each must be longer than 18 samples (scipy's ValueError).
    seeds  : dither RandomState seeds, one per group; None = filtfilt only (no 0.96
             scale, no dither).
    groups : utterances per seed, consecutive in `wavs` (a speaker's sorted files share
             one stream, make_spect.py:68-70); default one utterance per seed.
    Returns (wav, lens): one float64 CUDA tensor with the utterances back to back, and
    their lengths — the input of `stft_mel_packed`.
    """
    import torch
    lens = [int(np.shape(w)[0]) for w in wavs]
    if not lens:
        return torch.empty(0, dtype=torch.float64, device=device), []
    short = [n for n in lens if n <= PADLEN]
    if short:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {PADLEN}.")
    f32 = [(w.dtype == torch.float32) if torch.is_tensor(w) else (np.asarray(w).dtype == np.float32)
           for w in wavs]
    if any(f32) and not all(f32):
        raise ValueError("preprocess_gpu: mix of float32 and float64 utterances in one batch")
    dt = torch.float32 if f32[0] else torch.float64
    parts = [w.to(device=device, dtype=dt).reshape(-1) if torch.is_tensor(w)
             else torch.as_tensor(np.asarray(w, dtype=np.float32 if f32[0] else np.float64)).reshape(-1)
             for w in wavs]
    x = torch.cat([p.to(device, non_blocking=True) for p in parts])
    off_h = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    woff = torch.from_numpy(off_h).to(device)
    out = torch.empty(int(off_h[-1]), dtype=torch.float64, device=x.device)
    b, a, zi = _filter_consts()
    n_streams, soff, sd = 0, None, None
    if seeds is not None:
        groups = [1] * len(seeds) if groups is None else [int(g) for g in groups]
        if len(groups) != len(seeds) or sum(groups) != len(lens) or min(groups) < 0:
            raise ValueError("preprocess_gpu: groups must give one utterance count per seed, summing to len(wavs)")
        gidx = np.concatenate([[0], np.cumsum(groups)]).astype(np.int64)
        soff = torch.from_numpy(off_h[gidx]).to(device)
        sd_h = np.asarray(seeds, dtype=np.int64)
        if (sd_h < 0).any() or (sd_h > 0xFFFFFFFF).any():
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        sd = torch.from_numpy(sd_h.astype(np.uint32).view(np.int32)).to(device)
        n_streams = len(seeds)
    _lib.call("autovc_preprocess_f64", _lib.ptr(x), 0 if f32[0] else 1, _lib.ptr(woff), len(lens),
              b.ctypes.data, a.ctypes.data, zi.ctypes.data, ORDER, _lib.ptr(soff), _lib.ptr(sd), n_streams,
              _lib.ptr(out), _lib.stream_ptr(out.device))
    return out, lens


def n_frames(n_samples: int) -> int:
    """Frames of pySTFT for a signal of n_samples (make_spect.py:41)."""
    return (n_samples + FFT_LENGTH - (FFT_LENGTH - HOP_LENGTH)) // HOP_LENGTH


class _DeviceMel:
    """Per-device cache of the sparse mel basis."""
    _cache: dict = {}

    @classmethod
    def get(cls, device, n_mels=80):
        import torch
        key = (str(device), n_mels)
        if key not in cls._cache:
            lo, ln, off, w = sparse_mel(mel_basis(n_mels=n_mels))
            cls._cache[key] = tuple(torch.from_numpy(a).to(device) for a in (lo, ln, off, w))
        return cls._cache[key]


def stft_mel(wavs, mode: str = "spmel", device="cuda", n_mels: int = 80):
    """GPU STFT (+ mel) of a batch of preprocessed utterances.

    wavs: list of 1-D arrays / tensors (float, already filtfilt+dithered).
    Returns a list of float32 CUDA tensors, (T_u, 80) for 'spmel' and (T_u, 513)
    (frame-major) for 'stft'.  One kernel launch for the whole batch.
    """
    import torch
    if mode not in ("spmel", "stft"):
        raise ValueError(f"unknown front-end mode {mode!r}")
    if len(wavs) == 0:
        return []
    lens = [int(w.shape[0]) for w in wavs]
    parts = [torch.as_tensor(np.asarray(w, dtype=np.float64)) if not torch.is_tensor(w)
             else w.to(torch.float64) for w in wavs]
    wav = torch.cat([p.reshape(-1).to(device, non_blocking=True) for p in parts])
    return stft_mel_packed(wav, lens, mode, n_mels)


def stft_mel_packed(wav, lens, mode: str = "spmel", n_mels: int = 80):
    """`stft_mel` of utterances already back to back in one float64 CUDA tensor (the
    output of `preprocess_gpu`): no host round trip between the two front-end stages."""
    import torch
    if mode not in ("spmel", "stft"):
        raise ValueError(f"unknown front-end mode {mode!r}")
    if len(lens) == 0:
        return []
    if wav.dtype != torch.float64 or not wav.is_cuda or wav.numel() != sum(lens):
        raise ValueError("stft_mel_packed: wav must be a float64 CUDA tensor of sum(lens) samples")
    device = wav.device
    frames = [n_frames(n) for n in lens]
    woff = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int64, device=device)
    foff_h = np.concatenate([[0], np.cumsum(frames)])
    foff = torch.tensor(foff_h, dtype=torch.int64, device=device)
    total = int(foff_h[-1])
    width = n_mels if mode == "spmel" else N_BINS
    out = torch.empty((total, width), dtype=torch.float32, device=device)
    if mode == "spmel":
        lo, ln, off, w = _DeviceMel.get(out.device, n_mels)
        m = 0
    else:
        lo = ln = off = w = None
        m = 1
    _lib.call("autovc_stft_mel_f32", _lib.ptr(wav), _lib.ptr(woff), _lib.ptr(foff), len(lens),
              total, _lib.ptr(lo), _lib.ptr(ln), _lib.ptr(off), _lib.ptr(w),
              n_mels if mode == "spmel" else 0, m, _lib.ptr(out), _lib.stream_ptr(out.device))
    return list(torch.split(out, frames, dim=0))
