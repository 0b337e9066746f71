"""End-to-end voice conversion on the GPU — BASELINE config 5 / SURVEY §8d C5:
wav -> STFT+mel (make_spect.py) -> Generator conversion (conversion.py) -> WaveNet
synthesis (vocoder.py / synthesis.wavegen).

Stages and where they run:
  spectrograms  filtfilt + dither (make_spect.py:74-76, RandomState per utterance) in one
                launch pair (autovc_preprocess_f64), then one fused STFT+mel launch for all
                utterances on the same device buffer (autovc_stft_mel_f32)
  convert       conversion.py:40-44,90-102: pad to a multiple of `freq`, eval forward with
                (emb_org, emb_trg), drop the padding.  Utterances with the same padded length
                run as one batch (eval BatchNorm and the LSTMs are per-row, so a batch equals
                B=1 calls).  513-bin models are projected to 80 mels with the mel basis
                (conversion.py:102) by one GEMM.
  vocode        synthesis.wavegen_batch: all utterances in one batched WaveNet run, Philox
                draws keyed by (seed, global utterance index, sample)
Sharding (8 GPUs): give each rank its slice and its global utterance offset; no collective.
"""
from __future__ import annotations

import numpy as np
import torch

from . import dsp
from . import functional as AF
from .synthesis import wavegen_batch


def pad_seq(x, base=32):
    """conversion.py:14-17."""
    len_out = int(base * np.ceil(float(x.shape[0]) / base))
    len_pad = len_out - x.shape[0]
    assert len_pad >= 0
    return np.pad(x, ((0, len_pad), (0, 0)), "constant"), len_pad


def spectrograms(wavs, mode="spmel", device="cuda", seeds=None):
    """wavs: list of float arrays at 16 kHz -> list of (T, 80|513) device tensors."""
    seeds = seeds if seeds is not None else list(range(len(wavs)))
    wav, lens = dsp.preprocess_gpu([np.asarray(w, np.float64) for w in wavs], seeds=list(seeds), device=device)
    return dsp.stft_mel_packed(wav, lens, mode)


def _mel_project(y):
    """(T, 513) -> (T, 80) = y @ mel_basis (conversion.py:102), on the GEMM; K padded to 516."""
    basis = torch.from_numpy(np.ascontiguousarray(dsp.mel_basis().T)).to(y.device)   # (513, 80)
    Kp = 516
    yp = torch.zeros(y.shape[0], Kp, device=y.device, dtype=torch.float32)
    yp[:, : y.shape[1]] = y
    bT = torch.zeros(80, Kp, device=y.device, dtype=torch.float32)                     # B[n*ldb + k]
    bT[:, : basis.shape[0]] = basis.t()
    out = torch.empty(y.shape[0], 80, device=y.device, dtype=torch.float32)
    AF.gemm(y.shape[0], 80, Kp, yp, Kp, 0, bT, Kp, 0, out, 80)
    return out


@torch.no_grad()
def convert(G, specs, emb_org, emb_trg, freq=32, batch=True):
    """specs: list of (T_i, F) device tensors; emb_org / emb_trg: (N, 256) device tensors.
    Returns the converted (T_i, 80) mels (x_identic_psnt without padding)."""
    G.eval()
    dev = emb_org.device
    padded, pads = [], []
    for s in specs:
        p, lp = pad_seq(s.detach().cpu().numpy(), freq)
        padded.append(p)
        pads.append(lp)
    groups = {}
    for i, p in enumerate(padded):
        groups.setdefault(p.shape[0] if batch else (p.shape[0], i), []).append(i)
    out = [None] * len(specs)
    for idx in groups.values():
        x = torch.from_numpy(np.stack([padded[i] for i in idx])).to(dev)
        sel = torch.tensor(idx, device=dev)
        _, x_psnt, _ = G(x, emb_org.index_select(0, sel), emb_trg.index_select(0, sel))
        for r, i in enumerate(idx):
            T = specs[i].shape[0]
            y = x_psnt[r, 0, :T, :]
            out[i] = _mel_project(y) if y.shape[1] == 513 else y.contiguous()
    return out


def convert_and_vocode(wavs, G, vocoder, emb_org, emb_trg, mode="spmel", seed=0, utt_offset=0, device="cuda"):
    """The whole C5 chain for a list of utterances; returns (converted mels, waveforms)."""
    specs = spectrograms(wavs, mode, device=device, seeds=[utt_offset + i for i in range(len(wavs))])
    mels = convert(G, specs, emb_org, emb_trg)
    waves = wavegen_batch(vocoder, [m.cpu().numpy() for m in mels], seed=seed, utt_offset=utt_offset)
    return mels, waves
