"""Host-side DSP constants and the GPU front-end entry (STFT + mel + log/clip).

Host part (numpy/scipy, as in the reference):
  make_spect.py:30-34  butter_highpass, make_spect.py:74-76 filtfilt + dither
  make_spect.py:51     the Slaney mel basis (librosa 0.9.1 `filters.mel`, restated)
GPU part (HIP, libautovc_hip.so `autovc_stft_mel_f32`):
  make_spect.py:36-48 pySTFT + :79-86 mel projection, dB, clip
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
    frames = [n_frames(n) for n in lens]
    parts = [torch.as_tensor(np.asarray(w, dtype=np.float64)) if not torch.is_tensor(w)
             else w.to(torch.float64) for w in wavs]
    wav = torch.cat([p.reshape(-1).to(device, non_blocking=True) for p in parts])
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
    _lib.call("autovc_stft_mel_f32", _lib.ptr(wav), _lib.ptr(woff), _lib.ptr(foff), len(wavs),
              total, _lib.ptr(lo), _lib.ptr(ln), _lib.ptr(off), _lib.ptr(w),
              n_mels if mode == "spmel" else 0, m, _lib.ptr(out), _lib.stream_ptr(out.device))
    return list(torch.split(out, frames, dim=0))
