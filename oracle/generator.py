"""ORACLE (test infrastructure only) — CPU restatement of the AutoVC Generator and of one
Solver training step, in plain PyTorch CPU ops on a flat {state_dict key: tensor} map.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (autovc_amd/) never does.

Restates:
  model_vc_mel.py:41-81   Encoder  (cat emb, 3x conv5+BN+ReLU, 2-layer BLSTM(32), codes)
  model_vc_mel.py:84-122  Decoder  (LSTM(320->512), 3x conv5+BN+ReLU, LSTM(512->1024) x2,
                                    Linear(1024->80))
  model_vc_mel.py:125-169 Postnet  (4x conv5+BN+tanh, conv5+BN)
  model_vc_mel.py:172-203 Generator.forward
  model_vc_stft.py:7-29   the 513-bin variant (same arithmetic, other widths, `model.` keys)
  solver_encoder.py:228-243,293-300  loss composition + backward + Adam step
BatchNorm in train mode updates the running statistics in the map exactly like
nn.BatchNorm1d (momentum 0.1, unbiased running_var, num_batches_tracked += 1).

Pinned against tests/golden/generator_*.npz, produced by tests/golden/make_generator_golden.py
from the reference's own model_vc_mel.Generator and solver_encoder.Solver.train (imported
from /root/reference in the build container).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------- deterministic weights
def deterministic_state_dict(template: dict) -> dict:
    """The fixture weight scheme: for key k at index i of the state_dict,
    RandomState(1000+i).uniform(-s, s) with s = 1/sqrt(fan_in) for >=2-D tensors,
    BN weight = 1 + U(-0.1, 0.1), biases U(-0.1, 0.1), running_mean 0, running_var 1,
    num_batches_tracked 0.  `template` maps key -> tensor (shapes/dtypes)."""
    out = {}
    for i, (k, v) in enumerate(template.items()):
        rs = np.random.RandomState(1000 + i)
        shape = tuple(v.shape)
        if k.endswith("num_batches_tracked"):
            out[k] = torch.zeros((), dtype=torch.long)
        elif k.endswith("running_mean"):
            out[k] = torch.zeros(shape, dtype=torch.float32)
        elif k.endswith("running_var"):
            out[k] = torch.ones(shape, dtype=torch.float32)
        elif len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            s = 1.0 / np.sqrt(fan_in)
            out[k] = torch.from_numpy(rs.uniform(-s, s, shape).astype(np.float32))
        elif k.endswith("weight"):
            out[k] = torch.from_numpy((1.0 + rs.uniform(-0.1, 0.1, shape)).astype(np.float32))
        else:
            out[k] = torch.from_numpy(rs.uniform(-0.1, 0.1, shape).astype(np.float32))
    return out


def generator_keys(dim_neck=32, dim_emb=256, dim_pre=512, n_in=80, n_out=80, prefix=""):
    """Ordered (key, shape) list of the reference Generator state_dict (model_vc_mel.py)."""
    keys = []

    def conv_bn(p, ci, co):
        keys.extend([(f"{p}.0.conv.weight", (co, ci, 5)), (f"{p}.0.conv.bias", (co,)),
                     (f"{p}.1.weight", (co,)), (f"{p}.1.bias", (co,)), (f"{p}.1.running_mean", (co,)),
                     (f"{p}.1.running_var", (co,)), (f"{p}.1.num_batches_tracked", ())])

    def lstm(p, isz, H, layers, bidir):
        for l in range(layers):
            i = isz if l == 0 else H * (2 if bidir else 1)
            for sfx in [""] + (["_reverse"] if bidir else []):
                keys.extend([(f"{p}.weight_ih_l{l}{sfx}", (4 * H, i)), (f"{p}.weight_hh_l{l}{sfx}", (4 * H, H)),
                             (f"{p}.bias_ih_l{l}{sfx}", (4 * H,)), (f"{p}.bias_hh_l{l}{sfx}", (4 * H,))])

    for i in range(3):
        conv_bn(f"encoder.convolutions.{i}", n_in + dim_emb if i == 0 else 512, 512)
    lstm("encoder.lstm", 512, dim_neck, 2, True)
    lstm("decoder.lstm1", 2 * dim_neck + dim_emb, dim_pre, 1, False)
    for i in range(3):
        conv_bn(f"decoder.convolutions.{i}", dim_pre, dim_pre)
    lstm("decoder.lstm2", dim_pre, 1024, 2, False)
    keys.extend([("decoder.linear_projection.linear_layer.weight", (n_out, 1024)),
                 ("decoder.linear_projection.linear_layer.bias", (n_out,))])
    conv_bn("postnet.convolutions.0", n_out, 512)
    for i in range(1, 4):
        conv_bn(f"postnet.convolutions.{i}", 512, 512)
    conv_bn("postnet.convolutions.4", 512, n_out)
    return [(prefix + k, s) for k, s in keys]


def make_weights(prefix="", **kw) -> dict:
    tmpl = {k: torch.empty(s) for k, s in generator_keys(prefix=prefix, **kw)}
    return deterministic_state_dict(tmpl)


# ---------------------------------------------------------------- restatement
class OracleGenerator:
    """Functional Generator over a parameter map P (key -> tensor).  Tensors that need
    gradients are leaves the caller created with requires_grad."""

    def __init__(self, P: dict, dim_neck=32, freq=32, prefix="", training=True, fused_lstm=False):
        """fused_lstm=True runs the LSTMs through torch's own fused CPU kernel (the op the
        reference's nn.LSTM calls) instead of the explicit per-step restatement: same
        semantics, reference-speed — used for the CPU-baseline timing."""
        self.P, self.dim_neck, self.freq, self.pre, self.training = P, dim_neck, freq, prefix, training
        self.fused_lstm = fused_lstm

    def _g(self, k):
        return self.P[self.pre + k]

    def _conv_bn(self, x_nct, p, act):
        y = F.conv1d(x_nct, self._g(f"{p}.0.conv.weight"), self._g(f"{p}.0.conv.bias"), padding=2)
        rm, rv = self._g(f"{p}.1.running_mean"), self._g(f"{p}.1.running_var")
        if self.training:
            n = y.shape[0] * y.shape[2]
            mean = y.mean(dim=(0, 2))
            var_b = y.var(dim=(0, 2), unbiased=False)
            with torch.no_grad():
                rm.mul_(0.9).add_(0.1 * mean.detach())
                rv.mul_(0.9).add_(0.1 * var_b.detach() * n / (n - 1))
                self.P[self.pre + f"{p}.1.num_batches_tracked"] += 1
            yh = (y - mean[None, :, None]) / torch.sqrt(var_b[None, :, None] + 1e-5)
        else:
            yh = (y - rm[None, :, None]) / torch.sqrt(rv[None, :, None] + 1e-5)
        z = yh * self._g(f"{p}.1.weight")[None, :, None] + self._g(f"{p}.1.bias")[None, :, None]
        return {"relu": F.relu, "tanh": torch.tanh, "none": lambda v: v}[act](z)

    @staticmethod
    def _lstm_dir(x, Wih, Whh, bih, bhh, reverse):
        B, T, _ = x.shape
        H = Whh.shape[1]
        gx = x @ Wih.t() + bih + bhh
        h = x.new_zeros(B, H)
        c = x.new_zeros(B, H)
        outs = [None] * T
        order = range(T - 1, -1, -1) if reverse else range(T)
        for t in order:
            g = gx[:, t] + h @ Whh.t()
            i, f, gg, o = g.chunk(4, dim=1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            outs[t] = h
        return torch.stack(outs, dim=1)

    def _lstm(self, x, p, layers, bidir):
        if self.fused_lstm:
            ws = []
            for l in range(layers):
                for sfx in [""] + (["_reverse"] if bidir else []):
                    ws += [self._g(f"{p}.{n}_l{l}{sfx}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            H = ws[1].shape[1]
            h0 = x.new_zeros(layers * (2 if bidir else 1), x.shape[0], H)
            return torch._VF.lstm(x, (h0, h0), ws, True, layers, 0.0, self.training, bidir, True)[0]
        for l in range(layers):
            a = [self._g(f"{p}.{n}_l{l}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            fw = self._lstm_dir(x, *a, reverse=False)
            if bidir:
                b = [self._g(f"{p}.{n}_l{l}_reverse") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
                x = torch.cat([fw, self._lstm_dir(x, *b, reverse=True)], dim=-1)
            else:
                x = fw
        return x

    def encode(self, x, c_org):
        if x.dim() == 4:
            x = x.squeeze(1)
        x = x.transpose(2, 1)
        x = torch.cat((x, c_org.unsqueeze(-1).expand(-1, -1, x.size(-1))), dim=1)
        for i in range(3):
            x = self._conv_bn(x, f"encoder.convolutions.{i}", "relu")
        out = self._lstm(x.transpose(1, 2), "encoder.lstm", 2, True)
        d, fq = self.dim_neck, self.freq
        T = out.shape[1]
        if T % fq != 0:
            raise IndexError("T must be a multiple of freq")
        codes = [torch.cat((out[:, i + fq - 1, :d], out[:, i, d:]), dim=-1) for i in range(0, T, fq)]
        return torch.cat(codes, dim=-1)

    def forward(self, x, c_org, c_trg):
        code_real = self.encode(x, c_org)
        if c_trg is None:
            return code_real
        T = x.shape[-2]
        n = code_real.shape[1] // (2 * self.dim_neck)
        codes = code_real.view(code_real.shape[0], n, -1)
        code_exp = codes.repeat_interleave(T // n, dim=1)
        dec_in = torch.cat((code_exp, c_trg.unsqueeze(1).expand(-1, T, -1)), dim=-1)
        h = self._lstm(dec_in, "decoder.lstm1", 1, False).transpose(1, 2)
        for i in range(3):
            h = self._conv_bn(h, f"decoder.convolutions.{i}", "relu")
        h = self._lstm(h.transpose(1, 2), "decoder.lstm2", 2, False)
        x_id = h @ self._g("decoder.linear_projection.linear_layer.weight").t() + \
            self._g("decoder.linear_projection.linear_layer.bias")
        p = x_id.transpose(2, 1)
        for i in range(4):
            p = self._conv_bn(p, f"postnet.convolutions.{i}", "tanh")
        p = self._conv_bn(p, "postnet.convolutions.4", "none")
        x_psnt = x_id + p.transpose(2, 1)
        return x_id.unsqueeze(1), x_psnt.unsqueeze(1), code_real


def solver_losses(G, x_real, emb, lambda_cd=1.0):
    """solver_encoder.py:228-243 for the spmel/stft branch -> (g_loss, id, id_psnt, cd)."""
    x_id, x_psnt, code_real = G.forward(x_real, emb, emb)
    l_id = F.mse_loss(x_real.squeeze(), x_id.squeeze())
    l_psnt = F.mse_loss(x_real, x_psnt.squeeze())
    code_rec = G.forward(x_psnt, emb, None)
    l_cd = F.l1_loss(code_real, code_rec)
    return l_id + l_psnt + lambda_cd * l_cd, l_id, l_psnt, l_cd


def train_steps(P, batches, lr=1e-4, n_steps=1, dim_neck=32, freq=32, prefix=""):
    """Run n_steps Solver iterations (losses, backward, torch Adam) on the map P (modified in
    place).  Returns ([(id, id_psnt, cd) per step], grads of the first step)."""
    params = [v for k, v in P.items() if v.dtype == torch.float32 and "running_" not in k]
    for v in params:
        v.requires_grad_(True)
    opt = torch.optim.Adam(params, lr)
    G = OracleGenerator(P, dim_neck, freq, prefix, training=True)
    hist, first_grads = [], None
    for s in range(n_steps):
        x, e = batches[s % len(batches)]
        g_loss, a, b, c = solver_losses(G, x, e)
        opt.zero_grad()
        g_loss.backward()
        if first_grads is None:
            first_grads = {k: v.grad.detach().clone() for k, v in P.items() if getattr(v, "grad", None) is not None}
        opt.step()
        hist.append((a.item(), b.item(), c.item()))
    for v in params:
        v.requires_grad_(False)
    return hist, first_grads
