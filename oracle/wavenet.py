"""ORACLE (test infrastructure only) — CPU restatement of the WaveNet vocoder inference
path that synthesis.wavegen drives, in plain numpy/PyTorch CPU ops on a flat
{state_dict key: tensor} map.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (autovc_amd/) never does.

PARITY UNPINNED.  The arithmetic lives in the third-party package wavenet_vocoder==0.1.1
(reference requirements.txt:7), which is neither vendored in the reference nor installed
in this image, and the reference holds no test, golden vector or checkpoint for it
(results/*.wav depend on an absent checkpoint and on stochastic sampling; they pin only
the output length 256*Tc).  This module restates the package's published algorithm:
  builder.wavenet / WaveNet.__init__  (24 layers, 4 stacks -> dilation 2**(l % 6),
      scalar input, legacy skip accumulation, upsample 4x ConvTranspose2d(1,1,(3,4),
      stride (1,4), pad (1,0)) + ReLU)                  call site synthesis.py:19-40
  WaveNet.incremental_forward  (first_conv 1x1, 24 x ResidualConv1dGLU, skips
      (s + h) * sqrt(.5), ReLU -> 1x1 -> ReLU -> 1x1, sampling, feedback)
                                                        call site synthesis.py:67-69
  conv.Conv1d.incremental_forward  (input buffer of k + (k-1)(d-1) frames, shifted one
      frame per step, every d-th row, F.linear with the (out, k, in) linearized weight)
  ResidualConv1dGLU._forward  (split a|b, + conditioning 1x1, tanh(a)*sigmoid(b),
      skip 1x1, out 1x1, (out + residual) * sqrt(.5))
  mixture.sample_from_discretized_mix_logistic  (Gumbel-max over 10 logits with
      u ~ U(1e-5, 1-1e-5), clamp(log_scale, log_scale_min), mu + e^s (log u - log(1-u)),
      clamp [-1, 1])
  make_generation_fast_  (remove weight norm: W = g * v / ||v||, norm over all dims but 0)
The uniforms are injected (`philox_uniforms`, the same counter-based stream the HIP
sampler draws) instead of torch's global RNG, so sampling is deterministic and the GPU
path can be compared sample by sample.  Self-consistency checks in
tests/test_oracle_wavenet.py pin the incremental restatement against an independent
full-sequence (non-incremental) formulation built on torch's own conv ops.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# hparams.py:59-114 (the reference's WaveNet configuration)
HPARAMS = dict(out_channels=30, layers=24, stacks=4, residual_channels=512, gate_channels=512,
               skip_out_channels=256, kernel_size=3, cin_channels=80, upsample_scales=(4, 4, 4, 4),
               freq_axis_kernel_size=3, log_scale_min=float(-32.23619130191664), hop_size=256)

SQRT_HALF = math.sqrt(0.5)
N_UNIFORMS = 11          # 10 Gumbel-max uniforms + 1 logistic uniform per sample


# ---------------------------------------------------------------- weights
def wavenet_keys(hp=HPARAMS, weight_norm=False):
    """Ordered (key, shape) list of the r9y9 WaveNet state_dict (after make_generation_fast_
    when weight_norm=False; with weight_g / weight_v pairs otherwise)."""
    R, G, S, C, K = (hp["residual_channels"], hp["gate_channels"], hp["skip_out_channels"],
                     hp["cin_channels"], hp["kernel_size"])
    keys = []

    def conv(name, co, ci, k, kind="1d"):
        shape = (co, ci, k) if kind == "1d" else (1, 1, hp["freq_axis_kernel_size"], k)
        if weight_norm:
            gshape = (co, 1, 1) if kind == "1d" else (1, 1, 1, 1)
            keys.append((f"{name}.bias", (co,) if kind == "1d" else (1,)))
            keys.append((f"{name}.weight_g", gshape))
            keys.append((f"{name}.weight_v", shape))
        else:
            keys.append((f"{name}.weight", shape))
            keys.append((f"{name}.bias", (co,) if kind == "1d" else (1,)))

    conv("first_conv", R, 1, 1)
    for l in range(hp["layers"]):
        p = f"conv_layers.{l}"
        conv(f"{p}.conv", G, R, K)
        conv(f"{p}.conv1x1c", G, C, 1)
        conv(f"{p}.conv1x1_out", R, G // 2, 1)
        conv(f"{p}.conv1x1_skip", S, G // 2, 1)
    conv("last_conv_layers.1", S, S, 1)
    conv("last_conv_layers.3", hp["out_channels"], S, 1)
    for i, s in enumerate(hp["upsample_scales"]):
        conv(f"upsample_conv.{2 * i}", 1, 1, s, kind="2d")
    return keys


def make_weights(hp=HPARAMS, seed=4322):
    """Deterministic folded (weight-norm removed) weights.  Key i draws from
    RandomState(seed + i): conv weights N(0, sqrt(1 / (k * in))) (r9y9 Conv1d init with
    std_mul 1), biases U(-0.05, 0.05) (r9y9 zeroes them; non-zero here so the bias paths
    are exercised), upsample kernels 1/3 + U(-0.05, 0.05) (r9y9 fills 1/3)."""
    out = {}
    for i, (k, shape) in enumerate(wavenet_keys(hp)):
        rs = np.random.RandomState(seed + i)
        if k.startswith("upsample_conv") and k.endswith("weight"):
            w = 1.0 / 3.0 + rs.uniform(-0.05, 0.05, shape)
        elif k.endswith("weight"):
            fan_in = int(np.prod(shape[1:]))
            w = rs.normal(0.0, math.sqrt(1.0 / fan_in), shape)
        else:
            w = rs.uniform(-0.05, 0.05, shape)
        out[k] = torch.from_numpy(np.asarray(w, dtype=np.float32))
    return out


def fold_weight_norm(sd):
    """make_generation_fast_ / torch remove_weight_norm: weight = g * v / ||v|| with the
    norm over every dim but 0 (weight_norm's default dim=0)."""
    out = {}
    for k, v in sd.items():
        if k.endswith("weight_g"):
            base = k[: -len("_g")]
            vv = sd[base + "_v"].double()
            norm = vv.reshape(vv.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (vv.dim() - 1))
            out[base] = (sd[k].double() * vv / norm).float()
        elif k.endswith("weight_v"):
            continue
        else:
            out[k] = v
    return out


# ---------------------------------------------------------------- counter-based uniforms
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al., SC'11) on uint64 numpy arrays holding 32-bit lanes."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & _MASK for x in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & _MASK)
    k1 = np.uint64(k1 & _MASK)
    for _ in range(10):
        p0 = np.uint64(_M0) * c0
        p1 = np.uint64(_M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(_MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(_MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(_W0)) & np.uint64(_MASK)
        k1 = (k1 + np.uint64(_W1)) & np.uint64(_MASK)
    return c0, c1, c2, c3


def philox_uniforms(seed, utt_ids, t0, t1):
    """(len(utt_ids), t1 - t0, 11) float32 uniforms in [1e-5, 1 - 1e-5] for output samples
    t0..t1-1.  Sample t of utterance u draws Philox(key = seed, counter = (t, u, j, 0)),
    j = 0..2, giving 12 words; word w -> v = (w >> 9) + 0.5 scaled by 2**-23 (exact in
    fp32) -> 1e-5 + (1 - 2e-5) * v in float64 -> rounded to float32.  Uniform i < 10 feeds
    the Gumbel-max mixture choice, uniform 10 the logistic sample (the two torch
    uniform_(1e-5, 1 - 1e-5) draws of sample_from_discretized_mix_logistic)."""
    utt = np.asarray(utt_ids, dtype=np.uint64)[:, None]
    t = np.arange(t0, t1, dtype=np.uint64)[None, :]
    utt, t = np.broadcast_arrays(utt, t)
    words = []
    for j in range(3):
        words.extend(philox4x32(t, utt, np.full_like(t, j), np.zeros_like(t), seed & _MASK, (seed >> 32) & _MASK))
    w = np.stack(words[:N_UNIFORMS], axis=-1)
    v = ((w >> np.uint64(9)).astype(np.float64) + 0.5) * (2.0 ** -23)
    return (1e-5 + (1.0 - 2e-5) * v).astype(np.float32)


# ---------------------------------------------------------------- model
class OracleWaveNet:
    """r9y9 WaveNet inference on CPU.  `W` = folded state dict (weights as in make_weights)."""

    def __init__(self, W, hp=HPARAMS, dtype=torch.float64):
        self.hp = hp
        self.dtype = dtype
        self.W = {k: v.to(dtype) for k, v in W.items()}
        self.lps = hp["layers"] // hp["stacks"]

    # --- upsample network (WaveNet.__init__ upsample_conv; applied in incremental_forward)
    def upsample(self, c):
        """c (B, 80, Tc) -> (B, 80, Tc * prod(scales)) with torch's conv_transpose2d + ReLU."""
        x = c.to(self.dtype).unsqueeze(1)
        for i, s in enumerate(self.hp["upsample_scales"]):
            w = self.W[f"upsample_conv.{2 * i}.weight"]
            b = self.W[f"upsample_conv.{2 * i}.bias"]
            pad = (self.hp["freq_axis_kernel_size"] - 1) // 2
            x = F.relu(F.conv_transpose2d(x, w, b, stride=(1, s), padding=(pad, 0)))
        return x.squeeze(1)

    def upsample_loops(self, c):
        """Same as upsample() written out: out[f, s*t + j] = relu(b + sum_k w[k, j] *
        in[f + 1 - k, t]) per stage (transposed conv, kernel == stride on time)."""
        x = c.to(self.dtype).numpy() if torch.is_tensor(c) else np.asarray(c, np.float64)
        for i, s in enumerate(self.hp["upsample_scales"]):
            w = self.W[f"upsample_conv.{2 * i}.weight"].numpy()[0, 0]
            b = float(self.W[f"upsample_conv.{2 * i}.bias"].numpy()[0])
            B, Fq, T = x.shape
            y = np.full((B, Fq, T, s), b)
            kf = w.shape[0]
            pad = (kf - 1) // 2
            for k in range(kf):
                for f in range(Fq):
                    src = f + pad - k
                    if 0 <= src < Fq:
                        y[:, f, :, :] += w[k][None, None, :] * x[:, src, :, None]
            x = np.maximum(y.reshape(B, Fq, T * s), 0.0)
        return torch.from_numpy(x)

    # --- head + sampling
    def _head(self, skips):
        W = self.W
        x = F.relu(skips)
        x = F.linear(x, W["last_conv_layers.1.weight"][:, :, 0], W["last_conv_layers.1.bias"])
        x = F.relu(x)
        return F.linear(x, W["last_conv_layers.3.weight"][:, :, 0], W["last_conv_layers.3.bias"])

    def sample(self, y, u):
        """sample_from_discretized_mix_logistic with injected uniforms u (B, 11)."""
        nr = y.shape[1] // 3
        logit = y[:, :nr]
        temp = logit - torch.log(-torch.log(u[:, :nr].to(y.dtype)))
        idx = temp.argmax(dim=1)
        one_hot = F.one_hot(idx, nr).to(y.dtype)
        means = (y[:, nr:2 * nr] * one_hot).sum(1)
        log_scales = torch.clamp((y[:, 2 * nr:3 * nr] * one_hot).sum(1), min=self.hp["log_scale_min"])
        uu = u[:, nr].to(y.dtype)
        x = means + torch.exp(log_scales) * (torch.log(uu) - torch.log(1.0 - uu))
        return torch.clamp(torch.clamp(x, min=-1.0), max=1.0)

    # --- incremental generation (WaveNet.incremental_forward)
    @torch.no_grad()
    def incremental(self, c_up, T, uniforms=None, teacher=None, return_mol=False):
        """c_up (B, 80, T) upsampled conditioning.  uniforms (B, T, 11) drive sampling;
        teacher (B, Tt): the input at step t < Tt is teacher[:, t] (test_inputs).  Returns
        y (B, T) [and the MoL parameters (B, T, 30) of every step]."""
        hp, W, dt = self.hp, self.W, self.dtype
        B = c_up.shape[0]
        R, G = hp["residual_channels"], hp["gate_channels"]
        K = hp["kernel_size"]
        c = c_up.to(dt).transpose(1, 2)                                  # (B, T, 80)
        bufs = []
        lin = []
        for l in range(hp["layers"]):
            d = 2 ** (l % self.lps)
            bufs.append(torch.zeros(B, K + (K - 1) * (d - 1), R, dtype=dt))
            w = W[f"conv_layers.{l}.conv.weight"]                       # (G, R, K)
            lin.append(w.transpose(1, 2).contiguous().view(G, -1))      # (G, K*R)
        x_in = torch.zeros(B, dtype=dt)
        ys, mols = [], []
        for t in range(T):
            if teacher is not None and t < teacher.shape[1]:
                x_in = teacher[:, t].to(dt)
            elif t > 0:
                x_in = ys[-1]
            x = x_in[:, None] * W["first_conv.weight"][:, 0, 0][None, :] + W["first_conv.bias"][None, :]
            ct = c[:, t, :]
            skips = None
            for l in range(hp["layers"]):
                p = f"conv_layers.{l}"
                d = 2 ** (l % self.lps)
                residual = x
                buf = bufs[l]
                buf[:, :-1, :] = buf[:, 1:, :].clone()
                buf[:, -1, :] = x
                inp = buf[:, 0::d, :] if d > 1 else buf
                h = F.linear(inp.reshape(B, -1), lin[l], W[f"{p}.conv.bias"])
                a, b = h.split(G // 2, dim=1)
                cc = F.linear(ct, W[f"{p}.conv1x1c.weight"][:, :, 0], W[f"{p}.conv1x1c.bias"])
                ca, cb = cc.split(G // 2, dim=1)
                a, b = a + ca, b + cb
                g = torch.tanh(a) * torch.sigmoid(b)
                s = F.linear(g, W[f"{p}.conv1x1_skip.weight"][:, :, 0], W[f"{p}.conv1x1_skip.bias"])
                o = F.linear(g, W[f"{p}.conv1x1_out.weight"][:, :, 0], W[f"{p}.conv1x1_out.bias"])
                x = (o + residual) * SQRT_HALF
                skips = s if skips is None else (skips + s) * SQRT_HALF
            y = self._head(skips)
            if return_mol:
                mols.append(y)
            if uniforms is not None:
                ys.append(self.sample(y, torch.as_tensor(uniforms[:, t, :])))
            else:
                ys.append(torch.zeros(B, dtype=dt))
        out = torch.stack(ys, dim=1)
        if return_mol:
            return out, torch.stack(mols, dim=1)
        return out

    # --- independent full-sequence formulation (self-consistency check of incremental())
    @torch.no_grad()
    def teacher_forced_full(self, c_up, inputs):
        """MoL parameters (B, T, 30) for the given step inputs (B, T) computed over the whole
        sequence at once with causal dilated conv1d (WaveNet.forward semantics)."""
        hp, W, dt = self.hp, self.W, self.dtype
        G, K = hp["gate_channels"], hp["kernel_size"]
        T = inputs.shape[1]
        c = c_up.to(dt)
        x = F.conv1d(inputs.to(dt)[:, None, :], W["first_conv.weight"], W["first_conv.bias"])
        skips = None
        for l in range(hp["layers"]):
            p = f"conv_layers.{l}"
            d = 2 ** (l % self.lps)
            residual = x
            h = F.conv1d(x, W[f"{p}.conv.weight"], W[f"{p}.conv.bias"], padding=(K - 1) * d, dilation=d)[:, :, :T]
            a, b = h.split(G // 2, dim=1)
            cc = F.conv1d(c, W[f"{p}.conv1x1c.weight"], W[f"{p}.conv1x1c.bias"])
            ca, cb = cc.split(G // 2, dim=1)
            g = torch.tanh(a + ca) * torch.sigmoid(b + cb)
            s = F.conv1d(g, W[f"{p}.conv1x1_skip.weight"], W[f"{p}.conv1x1_skip.bias"])
            o = F.conv1d(g, W[f"{p}.conv1x1_out.weight"], W[f"{p}.conv1x1_out.bias"])
            x = (o + residual) * SQRT_HALF
            skips = s if skips is None else (skips + s) * SQRT_HALF
        y = F.relu(skips)
        y = F.relu(F.conv1d(y, W["last_conv_layers.1.weight"], W["last_conv_layers.1.bias"]))
        y = F.conv1d(y, W["last_conv_layers.3.weight"], W["last_conv_layers.3.bias"])
        return y.transpose(1, 2)


def small_hparams(layers=6, stacks=2):
    """A reduced configuration for fast oracle self-checks (same channel widths)."""
    hp = dict(HPARAMS)
    hp.update(layers=layers, stacks=stacks)
    return hp
