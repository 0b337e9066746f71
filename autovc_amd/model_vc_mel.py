"""AutoVC Generator on MI355X — same classes, constructor signatures, module tree and
state_dict keys as the reference model_vc_mel.py, so reference checkpoints load and
solver/conversion callers run unchanged.  Every forward/backward runs through the HIP
kernels of libautovc_hip.so (autovc_amd.functional); parameters stay ordinary
nn.Parameters (Conv1d / BatchNorm1d / Linear / LSTM-named tensors).

Reference: model_vc_mel.py:7-17 LinearNorm, :20-38 ConvNorm, :41-81 Encoder,
:84-122 Decoder, :125-169 Postnet, :172-203 Generator.
Internal layout is NTC (B, T, C); the reference's (B, C, T) conv views are never built.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import functional as AF


class LinearNorm(nn.Module):
    """model_vc_mel.py:7-17 (xavier_uniform with the named gain)."""

    def __init__(self, in_dim, out_dim, bias=True, w_init_gain="linear"):
        super().__init__()
        self.linear_layer = nn.Linear(in_dim, out_dim, bias=bias)
        nn.init.xavier_uniform_(self.linear_layer.weight, gain=nn.init.calculate_gain(w_init_gain))

    def forward(self, x):
        return AF.linear(x, self.linear_layer.weight, self.linear_layer.bias)


class ConvNorm(nn.Module):
    """model_vc_mel.py:20-38.  forward() keeps the reference's (B, C, T) signature; the
    Generator uses the fused NTC conv+BN+act path instead (functional.conv_bn_act)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=None, dilation=1,
                 bias=True, w_init_gain="linear"):
        super().__init__()
        if padding is None:
            assert kernel_size % 2 == 1
            padding = int(dilation * (kernel_size - 1) / 2)
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              padding=padding, dilation=dilation, bias=bias)
        nn.init.xavier_uniform_(self.conv.weight, gain=nn.init.calculate_gain(w_init_gain))

    def forward(self, signal):
        c = self.conv
        if c.kernel_size[0] != AF.KS or c.padding[0] != AF.PAD or c.stride[0] != 1 or c.dilation[0] != 1:
            raise NotImplementedError("autovc_amd ConvNorm supports kernel 5 / pad 2 / stride 1 (the AutoVC layers)")
        y = AF.conv_only(signal.transpose(1, 2), c.weight, c.bias)
        return y.transpose(1, 2)


def _is_k5(conv):
    return conv.kernel_size[0] == AF.KS and conv.padding[0] == AF.PAD and conv.stride[0] == 1


class LSTM(nn.Module):
    """nn.LSTM(input_size, hidden_size, num_layers, batch_first=True[, bidirectional]) with the
    same parameter names / init (weight_ih_l{k}[_reverse], ...), run on the HIP kernels.
    forward returns (output, None): the reference discards the final states
    (model_vc_mel.py:73,111,118)."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True, bidirectional=False):
        super().__init__()
        if not batch_first:
            raise NotImplementedError("autovc_amd LSTM is batch_first (as every AutoVC LSTM)")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional = bidirectional
        self.batch_first = True
        dirs = 2 if bidirectional else 1
        H = hidden_size
        for layer in range(num_layers):
            isz = input_size if layer == 0 else H * dirs
            for sfx in ([""] + (["_reverse"] if bidirectional else [])):
                self.register_parameter(f"weight_ih_l{layer}{sfx}", nn.Parameter(torch.empty(4 * H, isz)))
                self.register_parameter(f"weight_hh_l{layer}{sfx}", nn.Parameter(torch.empty(4 * H, H)))
                self.register_parameter(f"bias_ih_l{layer}{sfx}", nn.Parameter(torch.empty(4 * H)))
                self.register_parameter(f"bias_hh_l{layer}{sfx}", nn.Parameter(torch.empty(4 * H)))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for w in self.parameters():
            nn.init.uniform_(w, -stdv, stdv)

    def flatten_parameters(self):  # cuDNN-only concept; kept for API compatibility
        return None

    def forward(self, x, hx=None):
        if hx is not None:
            raise NotImplementedError("initial states are zero in AutoVC")
        save = torch.is_grad_enabled()
        if (not self.bidirectional and self.num_layers == 2 and self.hidden_size % 64 == 0
                and self.hidden_size >= 256):
            # stacked pair as one wavefront (decoder lstm2, model_vc_mel.py:104)
            return AF.LSTM2StackFn.apply(x, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0,
                                         self.weight_ih_l1, self.weight_hh_l1, self.bias_ih_l1, self.bias_hh_l1,
                                         save), None
        out = x
        for layer in range(self.num_layers):
            g = lambda n, s="": getattr(self, f"{n}_l{layer}{s}")  # noqa: E731
            if self.bidirectional:
                out = AF.BLSTMLayerFn.apply(out, g("weight_ih"), g("weight_hh"), g("bias_ih"), g("bias_hh"),
                                            g("weight_ih", "_reverse"), g("weight_hh", "_reverse"),
                                            g("bias_ih", "_reverse"), g("bias_hh", "_reverse"), save)
            else:
                out = AF.LSTMLayerFn.apply(out, g("weight_ih"), g("weight_hh"), g("bias_ih"), g("bias_hh"), save)
        return out, None


class Encoder(nn.Module):
    """model_vc_mel.py:41-81."""

    def __init__(self, dim_neck, dim_emb, freq):
        super().__init__()
        self.dim_neck = dim_neck
        self.freq = freq
        convolutions = []
        for i in range(3):
            convolutions.append(nn.Sequential(
                ConvNorm(80 + dim_emb if i == 0 else 512, 512, kernel_size=5, stride=1, padding=2, dilation=1,
                         w_init_gain="relu"),
                nn.BatchNorm1d(512)))
        self.convolutions = nn.ModuleList(convolutions)
        self.lstm = LSTM(512, dim_neck, 2, batch_first=True, bidirectional=True)

    def encode(self, x, c_org):
        """x (B,T,F) or (B,1,T,F), c_org (B,E) -> code_real (B, T/freq * 2*dim_neck)."""
        if x.dim() == 4:
            x = x.squeeze(1)
        B, T, F_in = x.shape
        h = AF.FrameConcatFn.apply(x, c_org, T, 1)            # :64-66
        h = AF.conv_bn_chain(h, [(conv[0].conv, conv[1], "relu") for conv in self.convolutions])   # :68-69
        out, _ = self.lstm(h)                                  # :72-73
        return AF.CodeGatherFn.apply(out, self.freq)           # :74-79

    def forward(self, x, c_org):
        codes = self.encode(x, c_org)
        n = codes.shape[1] // (2 * self.dim_neck)
        return list(codes.view(codes.shape[0], n, 2 * self.dim_neck).unbind(1))


class Decoder(nn.Module):
    """model_vc_mel.py:84-122."""

    def __init__(self, dim_neck, dim_emb, dim_pre):
        super().__init__()
        self.lstm1 = LSTM(dim_neck * 2 + dim_emb, dim_pre, 1, batch_first=True)
        convolutions = []
        for i in range(3):
            convolutions.append(nn.Sequential(
                ConvNorm(dim_pre, dim_pre, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="relu"),
                nn.BatchNorm1d(dim_pre)))
        self.convolutions = nn.ModuleList(convolutions)
        self.lstm2 = LSTM(dim_pre, 1024, 2, batch_first=True)
        self.linear_projection = LinearNorm(1024, 80)

    def forward(self, x):
        x, _ = self.lstm1(x)
        x = AF.conv_bn_chain(x, [(conv[0].conv, conv[1], "relu") for conv in self.convolutions])
        outputs, _ = self.lstm2(x)
        return self.linear_projection(outputs)


class Postnet(nn.Module):
    """model_vc_mel.py:125-169.  forward keeps the reference (B, C, T) signature."""

    def __init__(self):
        super().__init__()
        self.convolutions = nn.ModuleList()
        self.convolutions.append(nn.Sequential(
            ConvNorm(80, 512, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="tanh"),
            nn.BatchNorm1d(512)))
        for _ in range(1, 5 - 1):
            self.convolutions.append(nn.Sequential(
                ConvNorm(512, 512, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="tanh"),
                nn.BatchNorm1d(512)))
        self.convolutions.append(nn.Sequential(
            ConvNorm(512, 80, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="linear"),
            nn.BatchNorm1d(80)))

    def forward_ntc(self, x, residual=None):
        """x (B,T,C) -> postnet(x) (+ residual), NTC; the residual add of
        model_vc_mel.py:197 is fused into the last BN pass."""
        n = len(self.convolutions)
        return AF.conv_bn_chain(x, [(c[0].conv, c[1], "tanh" if i < n - 1 else "none")
                                    for i, c in enumerate(self.convolutions)], residual=residual)

    def forward(self, x):
        return self.forward_ntc(x.transpose(1, 2)).transpose(1, 2)


class Generator(nn.Module):
    """model_vc_mel.py:172-203."""

    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, dim_emb, freq)
        self.decoder = Decoder(dim_neck, dim_emb, dim_pre)
        self.postnet = Postnet()

    def conv_layers(self):
        """Every ConvNorm's nn.Conv1d (encoder, decoder, postnet)."""
        return ([c[0].conv for c in self.encoder.convolutions] + [c[0].conv for c in self.decoder.convolutions]
                + [c[0].conv for c in self.postnet.convolutions])

    def forward(self, x, c_org, c_trg):
        if x.is_cuda:   # inside the Solver's weight scope: all weight transforms in one launch
            full = c_trg is not None
            AF.prepare_weights(self.conv_layers() if full else [c[0].conv for c in self.encoder.convolutions],
                               [self.decoder.lstm1, self.decoder.lstm2] if full else [], x.shape[-2], self.training,
                               B=x.shape[0])
        with AF.blstm_last_pass(c_trg is not None):   # the full pass's encoder is differentiated last
            code_real = self.encoder.encode(x, c_org)                   # :182
        if c_trg is None:
            return code_real                                            # :183-184
        T = x.shape[-2]
        n = code_real.shape[1] // (2 * self.encoder.dim_neck)
        dec_in = AF.FrameConcatFn.apply(code_real.view(code_real.shape[0], n, -1), c_trg, T,
                                        int(T / n))                    # :186-192
        x_identic = self.decoder(dec_in)                                # :194
        x_identic_psnt = self.postnet.forward_ntc(x_identic, residual=x_identic)  # :196-197
        return x_identic.unsqueeze(1), x_identic_psnt.unsqueeze(1), code_real   # :199-203
