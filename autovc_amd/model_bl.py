"""D-VECTOR speaker encoder — reference model_bl.py:5-20, inference on the GPU.

3-layer LSTM (dim_input -> dim_cell) on the HIP step kernels (autovc_amd.model_vc_mel.LSTM,
same `lstm.weight_ih_l{k}` ... names), the embedding Linear applied to the last frame only
(one GEMM reading the last frame in place), and the row-wise L2 normalisation kernel.
make_metadata.py:41-80 runs it as `D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256)` in
eval mode to average 10 crops per speaker into the train.pkl speaker embedding.
Inference only, as in the reference (it is never trained there).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from . import functional as AF
from .model_vc_mel import LSTM


class D_VECTOR(nn.Module):
    """d vector speaker embedding."""

    def __init__(self, num_layers=3, dim_input=40, dim_cell=256, dim_emb=64):
        super().__init__()
        self.lstm = LSTM(input_size=dim_input, hidden_size=dim_cell, num_layers=num_layers, batch_first=True)
        self.embedding = nn.Linear(dim_cell, dim_emb)

    def forward(self, x):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            with torch.no_grad():
                return self._forward(x)
        return self._forward(x)

    def _forward(self, x):
        self.lstm.flatten_parameters()
        if x.device.type != "cuda":
            raise RuntimeError("D_VECTOR runs on the MI355X: move the model and inputs to cuda")
        lstm_out, _ = self.lstm(x.contiguous())                      # (B, T, H)
        B, T, H = lstm_out.shape
        E = self.embedding.out_features
        emb = torch.empty(B, E, device=x.device, dtype=torch.float32)
        # embeds = Linear(lstm_out[:, -1, :]): the last frame read in place (lda = T*H)
        AF.gemm(B, E, H, lstm_out, T * H, 0, self.embedding.weight.detach(), H, 0, emb, E,
                bias1=self.embedding.bias.detach(), a_off=(T - 1) * H)
        out = torch.empty_like(emb)
        _lib.call("autovc_l2norm_rows_f32", B, E, emb.data_ptr(), E, out.data_ptr(), E, _lib.stream_ptr(x.device))
        return out
