"""GeneratorSTFT — the 513-bin variant of model_vc_stft.py:7-53 on the HIP kernels.

Same construction as the reference (a Generator whose encoder conv0, decoder projection
and postnet end layers are swapped for 513-bin ones, model_vc_stft.py:16-29), hence the
same `model.`-prefixed state_dict keys.  Deliberate difference: the reference forward
calls self.decoder / self.postnet, which do not exist, and raises AttributeError (F10);
here forward delegates to self.model, the arithmetic the reference intended.
Channel counts 513 / 769 are zero-padded to multiples of 4 inside the conv ops.
"""
from __future__ import annotations

import torch.nn as nn

from .model_vc_mel import ConvNorm, Generator, LinearNorm


class GeneratorSTFT(nn.Module):
    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.model = Generator(dim_neck, dim_emb, dim_pre, freq)
        self.model.encoder.convolutions[0][0] = ConvNorm(513 + dim_emb, 512, kernel_size=5, stride=1, padding=2)
        self.model.decoder.linear_projection = LinearNorm(in_dim=1024, out_dim=513)
        self.model.postnet.convolutions[0][0] = ConvNorm(513, 512, kernel_size=5, stride=1, padding=2, dilation=1,
                                                         w_init_gain="tanh")
        self.model.postnet.convolutions[4] = nn.Sequential(
            ConvNorm(512, 513, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="linear"),
            nn.BatchNorm1d(513))

    def forward(self, x, c_org, c_trg):
        return self.model(x, c_org, c_trg)
