"""Waveform synthesis — reference synthesis.py:19-73 API (build_model, wavegen) on the
HIP WaveNet generator, plus a batched / sharded extension (wavegen_batch).

Differences from the reference, all deliberate:
  * the model must live on the GPU (the reference falls back to CPU when CUDA is absent,
    synthesis.py:15-16; there is no CPU path here);
  * sampling uniforms come from the Philox stream of autovc_amd.wavenet (seeded from
    torch's default generator), not torch's global RNG — a stochastic sampler either way;
  * `torch.set_num_threads(4)` (synthesis.py:14) is not applied: no CPU compute remains.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .hparams import hparams
from .wavenet import WaveNet


def _identity(x):
    return x


def wavenet(out_channels=256, layers=20, stacks=2, residual_channels=512, gate_channels=512,
            skip_out_channels=512, cin_channels=-1, gin_channels=-1, weight_normalization=True,
            dropout=1 - 0.95, kernel_size=3, n_speakers=None, upsample_conditional_features=False,
            upsample_scales=(16, 16), freq_axis_kernel_size=3, scalar_input=False,
            use_speaker_embedding=True, legacy=True):
    """wavenet_vocoder.builder.wavenet (the builder synthesis.py:21 resolves by name)."""
    return WaveNet(out_channels=out_channels, layers=layers, stacks=stacks, residual_channels=residual_channels,
                   gate_channels=gate_channels, skip_out_channels=skip_out_channels, kernel_size=kernel_size,
                   dropout=dropout, cin_channels=cin_channels, gin_channels=gin_channels, n_speakers=n_speakers,
                   weight_normalization=weight_normalization,
                   upsample_conditional_features=upsample_conditional_features,
                   upsample_scales=upsample_scales, freq_axis_kernel_size=freq_axis_kernel_size,
                   scalar_input=scalar_input, use_speaker_embedding=use_speaker_embedding, legacy=legacy)


_BUILDERS = {"wavenet": wavenet}


def build_model():
    """synthesis.py:19-40."""
    return _BUILDERS[hparams.builder](
        out_channels=hparams.out_channels,
        layers=hparams.layers,
        stacks=hparams.stacks,
        residual_channels=hparams.residual_channels,
        gate_channels=hparams.gate_channels,
        skip_out_channels=hparams.skip_out_channels,
        cin_channels=hparams.cin_channels,
        gin_channels=hparams.gin_channels,
        weight_normalization=hparams.weight_normalization,
        n_speakers=hparams.n_speakers,
        dropout=hparams.dropout,
        kernel_size=hparams.kernel_size,
        upsample_conditional_features=hparams.upsample_conditional_features,
        upsample_scales=hparams.upsample_scales,
        freq_axis_kernel_size=hparams.freq_axis_kernel_size,
        scalar_input=True,
        legacy=hparams.legacy,
    )


def _device_of(model):
    return next(model.parameters()).device


def wavegen(model, c=None, tqdm=_identity):
    """synthesis.py:44-73: c (Tc, 80) numpy mel -> (Tc * hop_size,) float32 numpy waveform."""
    model.eval()
    model.make_generation_fast_()
    Tc = c.shape[0]
    length = Tc * hparams.hop_size
    dev = _device_of(model)
    cc = torch.as_tensor(np.ascontiguousarray(np.asarray(c, dtype=np.float32).T)).unsqueeze(0).to(dev)
    initial_input = torch.zeros(1, 1, 1, device=dev)
    with torch.no_grad():
        y_hat = model.incremental_forward(initial_input, c=cc, g=None, T=length, tqdm=tqdm, softmax=True,
                                          quantize=True, log_scale_min=hparams.log_scale_min)
    return y_hat.view(-1).cpu().numpy()


def wavegen_batch(model, cs, seed=None, utt_offset=0, graph_steps=32):
    """Batched synthesis (new API): cs = list of (Tc_i, 80) mels -> list of (Tc_i * hop,)
    waveforms.  Utterances are padded to the longest; the Philox draws depend only on
    (seed, utt_offset + i, sample), so a rank of a sharded job passing its global offset
    produces exactly what one large batch would."""
    model.eval()
    model.make_generation_fast_()
    dev = _device_of(model)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    hop = int(math.prod(model.upsample_scales)) if model.upsample_conv is not None else 1
    Tmax = max(int(c.shape[0]) for c in cs)
    cin = model.cin_channels
    batch = np.zeros((len(cs), cin, Tmax), dtype=np.float32)
    for i, c in enumerate(cs):
        batch[i, :, : c.shape[0]] = np.asarray(c, dtype=np.float32).T
    with torch.no_grad():
        y = model.generate(torch.from_numpy(batch).to(dev), T=Tmax * hop, seed=seed, utt_base=utt_offset,
                           log_scale_min=hparams.log_scale_min, graph_steps=graph_steps)
    y = y.cpu().numpy()
    return [y[i, : int(c.shape[0]) * hop].copy() for i, c in enumerate(cs)]
