"""WaveNet vocoder with the r9y9 wavenet_vocoder 0.1.1 module API, generating on the GPU.

The reference builds this model with `builder.wavenet(...)` (synthesis.py:19-40, hparams
hparams.py:59-119), loads a checkpoint with `load_state_dict` (vocoder.py:14-15) and calls
`make_generation_fast_()` + `incremental_forward(...)` (synthesis.py:50-69).  This module
keeps the parameter tree and state_dict keys of that package (first_conv, conv_layers.{l}.
{conv, conv1x1c, conv1x1_out, conv1x1_skip}, last_conv_layers.{1,3}, upsample_conv.{0,2,4,6},
each with weight_g / weight_v under weight normalisation), so its checkpoints load as-is.

incremental_forward runs entirely in libautovc_hip.so:
  upsample   autovc_wavenet_upsample_f32 (conditioning frames -> samples, time-major)
  pre        autovc_gemm_f32: every layer's conditioning 1x1 conv + both biases for a
             chunk of samples in one MFMA GEMM (sample-independent work off the chain)
  generate   autovc_wavenet_generate_f32: the sample loop (one kernel per layer — each
             layer's current conv tap folded back onto the previous layer's gate output —
             + skip tail + head, sampling fused into the first layer's kernel), replayed as a
             hipGraph
Sampling draws its uniforms from a counter-based Philox stream keyed by (seed, utterance,
sample), so batched, sharded and chunked runs produce the same waveform per utterance.
The seed comes from torch's default generator (torch.manual_seed reproduces a run).

Supported configuration: the one the reference uses — scalar (raw) input with a
discretized mixture-of-logistics output, local conditioning, no global conditioning.
Training-mode forward is not part of the path (the reference only synthesises).
"""
from __future__ import annotations

import ctypes
import math
import warnings

import torch
import torch.nn as nn

from . import _lib
from . import functional as Fh


def _weight_norm(m, enabled):
    if not enabled:
        return m
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        return nn.utils.weight_norm(m)


def _conv1d(in_ch, out_ch, kernel_size, weight_normalization=True, std_mul=4.0, dropout=0.0, **kw):
    """wavenet_vocoder/modules.py Conv1d: normal init std = sqrt(std_mul (1 - dropout) / (k in)),
    zero bias, weight norm."""
    m = nn.Conv1d(in_ch, out_ch, kernel_size, **kw)
    std = math.sqrt((std_mul * (1.0 - dropout)) / (m.kernel_size[0] * in_ch))
    nn.init.normal_(m.weight, 0.0, std)
    nn.init.zeros_(m.bias)
    return _weight_norm(m, weight_normalization)


def _conv1x1(in_ch, out_ch, weight_normalization=True):
    return _conv1d(in_ch, out_ch, 1, weight_normalization, std_mul=1.0)


def _conv_transpose2d(kernel_size, weight_normalization=True, **kw):
    """wavenet_vocoder/modules.py ConvTranspose2d: weights 1/freq_kernel, zero bias."""
    m = nn.ConvTranspose2d(1, 1, kernel_size, **kw)
    nn.init.constant_(m.weight, 1.0 / kernel_size[0])
    nn.init.zeros_(m.bias)
    return _weight_norm(m, weight_normalization)


def _effective_weight(m):
    """The weight incremental_forward uses: weight-norm folded if still attached."""
    if hasattr(m, "weight_g"):
        return torch._weight_norm(m.weight_v, m.weight_g, 0)
    return m.weight


class ResidualConv1dGLU(nn.Module):
    """wavenet_vocoder/modules.py ResidualConv1dGLU (parameters only; the arithmetic is in
    the HIP generator)."""

    def __init__(self, residual_channels, gate_channels, kernel_size, skip_out_channels=None,
                 cin_channels=-1, gin_channels=-1, dropout=1 - 0.95, dilation=1, causal=True,
                 bias=True, weight_normalization=True):
        super().__init__()
        if skip_out_channels is None:
            skip_out_channels = residual_channels
        padding = (kernel_size - 1) * dilation if causal else (kernel_size - 1) // 2 * dilation
        self.dropout = dropout
        self.causal = causal
        self.dilation = dilation
        self.conv = _conv1d(residual_channels, gate_channels, kernel_size, weight_normalization,
                            std_mul=1.0, dropout=dropout, padding=padding, dilation=dilation, bias=bias)
        self.conv1x1c = _conv1x1(cin_channels, gate_channels, weight_normalization) if cin_channels > 0 else None
        if gin_channels > 0:
            raise NotImplementedError("global conditioning (gin_channels > 0) is not on the AutoVC path")
        self.conv1x1_out = _conv1x1(gate_channels // 2, residual_channels, weight_normalization)
        self.conv1x1_skip = _conv1x1(gate_channels // 2, skip_out_channels, weight_normalization)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        # wavenet_vocoder 0.1.1 (the reference's pin) gives the conditioning 1x1 a bias (its
        # weight-normalised Conv1d1x1 asserts bias=True); later releases build it with
        # bias=False.  A checkpoint of either kind loads: a missing
        # conv1x1c.bias is a zero bias, the same arithmetic.
        key = prefix + "conv1x1c.bias"
        if self.conv1x1c is not None and key not in state_dict and any(k.startswith(prefix + "conv1x1c.")
                                                                       for k in state_dict):
            state_dict[key] = torch.zeros_like(self.conv1x1c.bias)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)


def receptive_field_size(total_layers, num_cycles, kernel_size, dilation=lambda x: 2 ** x):
    layers_per_cycle = total_layers // num_cycles
    dilations = [dilation(i % layers_per_cycle) for i in range(total_layers)]
    return (kernel_size - 1) * sum(dilations) + 1


class WaveNet(nn.Module):
    """r9y9 WaveNet (wavenet_vocoder/wavenet.py) with a HIP incremental_forward."""

    def __init__(self, out_channels=256, layers=20, stacks=2, residual_channels=512, gate_channels=512,
                 skip_out_channels=512, kernel_size=3, dropout=1 - 0.95, cin_channels=-1, gin_channels=-1,
                 n_speakers=None, weight_normalization=True, upsample_conditional_features=False,
                 upsample_scales=None, freq_axis_kernel_size=3, scalar_input=False,
                 use_speaker_embedding=True, legacy=True):
        super().__init__()
        if not scalar_input:
            raise NotImplementedError("one-hot (mu-law quantize) input is not on the AutoVC path "
                                      "(hparams.input_type = 'raw' => scalar_input=True)")
        if gin_channels > 0:
            raise NotImplementedError("global conditioning is not on the AutoVC path (gin_channels = -1)")
        if cin_channels <= 0:
            raise NotImplementedError("the AutoVC vocoder is locally conditioned on mels (cin_channels > 0)")
        if freq_axis_kernel_size != 3 and upsample_conditional_features:
            raise NotImplementedError("upsample network supports freq_axis_kernel_size = 3 (hparams.py:114)")
        assert layers % stacks == 0
        self.scalar_input = scalar_input
        self.out_channels = out_channels
        self.cin_channels = cin_channels
        self.legacy = legacy
        self.layers = layers
        self.stacks = stacks
        self.layers_per_stack = layers // stacks
        self.kernel_size = kernel_size
        self.residual_channels = residual_channels
        self.gate_channels = gate_channels
        self.skip_out_channels = skip_out_channels
        self.first_conv = _conv1x1(1, residual_channels, weight_normalization)
        self.conv_layers = nn.ModuleList([
            ResidualConv1dGLU(residual_channels, gate_channels, kernel_size, skip_out_channels=skip_out_channels,
                              bias=True, dilation=2 ** (l % self.layers_per_stack), dropout=dropout,
                              cin_channels=cin_channels, gin_channels=gin_channels,
                              weight_normalization=weight_normalization)
            for l in range(layers)])
        self.last_conv_layers = nn.ModuleList([
            nn.ReLU(inplace=True),
            _conv1x1(skip_out_channels, skip_out_channels, weight_normalization),
            nn.ReLU(inplace=True),
            _conv1x1(skip_out_channels, out_channels, weight_normalization),
        ])
        self.embed_speakers = None
        if upsample_conditional_features:
            self.upsample_scales = list(upsample_scales)
            self.upsample_conv = nn.ModuleList()
            for s in self.upsample_scales:
                pad = (freq_axis_kernel_size - 1) // 2
                self.upsample_conv.append(_conv_transpose2d((freq_axis_kernel_size, s), weight_normalization,
                                                            padding=(pad, 0), dilation=1, stride=(1, s)))
                self.upsample_conv.append(nn.ReLU(inplace=True))
        else:
            self.upsample_scales = []
            self.upsample_conv = None
        self.receptive_field = receptive_field_size(layers, stacks, kernel_size)

    # ---------------------------------------------------------------- reference API
    def has_speaker_embedding(self):
        return self.embed_speakers is not None

    def local_conditioning_enabled(self):
        return self.cin_channels > 0

    def make_generation_fast_(self):
        """Remove weight normalisation everywhere (wavenet.py make_generation_fast_)."""
        def remove(m):
            try:
                nn.utils.remove_weight_norm(m)
            except ValueError:
                return
        self.apply(remove)

    def clear_buffer(self):
        """The HIP generator keeps no state between calls (rings live in a per-call workspace)."""

    def forward(self, x, c=None, g=None, softmax=False):
        raise NotImplementedError("WaveNet training forward is not on the AutoVC hot path; use incremental_forward")

    # ---------------------------------------------------------------- HIP generation
    def _packed(self, dev):
        """Weights in the layout of autovc_wavenet_packed_floats (include/autovc_hip.h).  Layer
        l >= 1 carries its current conv tap folded back one layer (see csrc/wavenet.hip):
        [W_0 .. W_(K-2) | sqrt(.5) W_(K-1) W_out(l-1) | sqrt(.5) W_(K-1)], the products on the
        GEMM, and sqrt(.5) W_(K-1) b_out(l-1) joins the layer's conditioning bias."""
        R, G, S, K = self.residual_channels, self.gate_channels, self.skip_out_channels, self.kernel_size
        H = G // 2
        sq = math.sqrt(0.5)
        f32 = dict(device=dev, dtype=torch.float32)

        def w2(m):
            return _effective_weight(m).detach().to(**f32)

        parts = [w2(self.first_conv).reshape(R), self.first_conv.bias.detach().to(**f32).reshape(R)]
        wc, bconv, bcond = [], [], []
        prev_w = prev_b = None
        for l, layer in enumerate(self.conv_layers):
            W = w2(layer.conv)                                            # (G, R, K)
            taps = W[:, :, : K - 1].permute(0, 2, 1).reshape(G, (K - 1) * R)
            cur = W[:, :, K - 1].contiguous()                             # (G, R)
            bc = layer.conv.bias.detach().to(**f32).reshape(G).clone()
            if l == 0:
                mblk = torch.zeros(G, H, **f32)
                curblk = cur
            else:
                mblk = torch.empty(G, H, **f32)
                Fh.gemm(G, H, R, cur, R, 0, prev_w, H, 1, mblk, H)         # W_(K-1) W_out(l-1)
                mblk.mul_(sq)
                curblk = cur * sq
                cb = torch.empty(1, G, **f32)
                Fh.gemm(1, G, R, prev_b.reshape(1, R), R, 0, cur, R, 0, cb, G)
                bc = bc + sq * cb.reshape(G)
            wout = w2(layer.conv1x1_out).reshape(R, H)
            wskip = w2(layer.conv1x1_skip).reshape(S, H)
            bout = layer.conv1x1_out.bias.detach().to(**f32).reshape(R)
            parts += [torch.cat([taps, mblk, curblk], dim=1), wout, wskip, bout,
                      layer.conv1x1_skip.bias.detach().to(**f32).reshape(S)]
            prev_w, prev_b = wout.contiguous(), bout
            wc.append(w2(layer.conv1x1c).reshape(G, self.cin_channels))
            bconv.append(bc)
            bcond.append(layer.conv1x1c.bias.detach().to(**f32).reshape(G))
        l1, l3 = self.last_conv_layers[1], self.last_conv_layers[3]
        parts += [w2(l1).reshape(-1), l1.bias.detach().to(**f32).reshape(-1),
                  w2(l3).reshape(-1), l3.bias.detach().to(**f32).reshape(-1)]
        packed = torch.cat([p.reshape(-1) for p in parts]).contiguous()
        n = _lib.load().autovc_wavenet_packed_floats(self.layers, self.kernel_size, R, G, S, self.out_channels)
        if packed.numel() != n:
            raise RuntimeError(f"WaveNet packing: {packed.numel()} floats, library expects {n}")
        out = dict(packed=packed, wc=torch.cat(wc).contiguous(), bconv=torch.cat(bconv).contiguous(),
                   bcond=torch.cat(bcond).contiguous())
        if self.upsample_conv is not None:
            convs = [m for m in self.upsample_conv if isinstance(m, nn.ConvTranspose2d)]
            out["up_w"] = torch.cat([_effective_weight(m).detach().reshape(-1) for m in convs]).to(**f32)
            out["up_b"] = torch.cat([m.bias.detach().reshape(-1) for m in convs]).to(**f32)
        return out

    def upsample(self, c, P=None):
        """c (B, cin, Tc) -> time-major (Tc * prod(scales), B, cin) conditioning on the GPU."""
        P = P or self._packed(c.device)
        B, C, Tc = c.shape
        scales = self.upsample_scales
        T = Tc * int(math.prod(scales))
        out = torch.empty(T, B, C, device=c.device, dtype=torch.float32)
        arr = (_lib.c_int * len(scales))(*scales)
        _lib.call("autovc_wavenet_upsample_f32", B, Tc, C, len(scales), arr, c.contiguous().data_ptr(),
                  P["up_w"].data_ptr(), P["up_b"].data_ptr(), out.data_ptr(), _lib.stream_ptr(c.device))
        return out

    @torch.no_grad()
    def generate(self, c, T=None, seed=0, utt_base=0, teacher=None, return_mol=False,
                 log_scale_min=-7.0, chunk=None, graph_steps=32):
        """Batched incremental generation on the GPU.

        c        (B, cin, Tc) conditioning frames (upsampled here) — or (B, cin, T) already at
                 sample rate when the model has no upsample network
        teacher  optional (B, Tt) inputs of steps 0..Tt-1 (test_inputs)
        Returns y (B, T) [, mol (B, T, out_channels)] as device tensors."""
        if self.training:
            raise RuntimeError("incremental_forward only supports eval mode")
        dev = c.device
        if dev.type != "cuda":
            raise RuntimeError("WaveNet generation runs on the MI355X: move the model and inputs to cuda")
        c = c.to(torch.float32).contiguous()
        B = c.shape[0]
        P = self._packed(dev)
        if self.upsample_conv is not None:
            c_up = self.upsample(c, P)
        else:
            c_up = c.permute(2, 0, 1).contiguous()
        T_c = c_up.shape[0]
        if T is None:
            T = T_c
        if T != T_c:
            raise ValueError(f"conditioning covers {T_c} samples, T={T} requested "
                             "(incremental_forward asserts c.size(-1) == T)")
        R, G, S = self.residual_channels, self.gate_channels, self.skip_out_channels
        nG = self.layers * G
        lib = _lib.load()
        ring = int(lib.autovc_wavenet_ring_frames(self.layers, self.layers_per_stack, self.kernel_size))
        # the conditioning chunk is lcm(ring, graph_steps) samples: every captured graph then
        # starts at one of chunk / graph_steps (ring slot, chunk row) pairs, so a few cached
        # graphs, whose step kernels get both as static arguments, serve the whole sequence
        graph_steps = int(graph_steps or 0)
        cap = max(1, (1 << 30) // (B * nG * 4))          # <= 1 GiB of conditioning per chunk
        if graph_steps:
            # a multiple of lcm(ring, graph_steps): a graph-step count sharing few factors
            # with the ring makes that lcm large, so it is capped (graphs then recapture
            # at the chunk seams instead of holding a multi-GiB chunk)
            unit = math.lcm(ring, graph_steps)
            want = unit if chunk is None else max(unit, (int(chunk) + unit - 1) // unit * unit)
            if want > cap:
                want = max(graph_steps, cap // graph_steps * graph_steps)
            chunk = want
        elif chunk is None:
            chunk = cap
        chunk = min(chunk, T)
        pre = torch.empty(chunk, B, nG, device=dev, dtype=torch.float32)
        y = torch.empty(B, T, device=dev, dtype=torch.float32)
        mol = torch.empty(B, T, self.out_channels, device=dev, dtype=torch.float32) if return_mol else None
        tch = None
        if teacher is not None:
            tch = teacher.to(dev, torch.float32).reshape(B, -1).contiguous()
        ws_bytes = lib.autovc_wavenet_workspace_bytes(B, T, self.layers, self.layers_per_stack,
                                                              self.kernel_size, R, G, S)
        ws = torch.empty((ws_bytes + 3) // 4, device=dev, dtype=torch.float32)
        stream = _lib.stream_ptr(dev)
        for t0 in range(0, T, chunk):
            t1 = min(T, t0 + chunk)
            Fh.gemm((t1 - t0) * B, nG, self.cin_channels, c_up, self.cin_channels, 0,
                    P["wc"], self.cin_channels, 0, pre, nG, bias1=P["bconv"], bias2=P["bcond"],
                    a_off=t0 * B * self.cin_channels)
            _lib.call("autovc_wavenet_generate_f32", B, T, t0, t1, self.layers, self.layers_per_stack,
                      self.kernel_size, R, G, S, self.out_channels, int(self.legacy), P["packed"].data_ptr(),
                      pre.data_ptr(), chunk, int(seed) & ((1 << 64) - 1), int(utt_base), float(log_scale_min),
                      _lib.ptr(tch), 0 if tch is None else tch.shape[1], y.data_ptr(), _lib.ptr(mol),
                      ws.data_ptr(), int(graph_steps), stream)
        # the all-CU generation poisons its outputs and sets a fault word if a hand-off wait
        # timed out (its 256 workgroups were not all resident): read it whenever that kernel
        # ran (reading synchronises the device, so the per-layer launches do not pay for it)
        # and raise — never silently regenerate on another path
        path = lib.autovc_wavenet_last_path()
        if path in (1, 2):
            fault = ctypes.c_int(0)
            _lib.call("autovc_wavenet_fault", 1, ctypes.addressof(fault))
            if fault.value:
                diag = (ctypes.c_int * 5)()
                _lib.call("autovc_wavenet_grid_diag", 1, ctypes.addressof(diag))
                name = ("wn_grid_kernel (all-CU WaveNet generation)" if path == 1 else
                        "wn_pipe_kernel (layer-pipelined WaveNet generation)")
                msg = (f"{name}: a hand-off wait timed out "
                       f"(kind, step, phase, workgroup, tag seen = {tuple(diag)}) — its 256 workgroups were not all "
                       "resident (another process on this GPU?)")
                if lib.autovc_wavenet_grid_explicit():
                    # the persistent path was asked for (AVC_WN_GRID / autovc_wavenet_set_grid): fail loudly
                    raise Fh.DeviceFault(
                        msg + "; outputs are NaN.  Run one generation process per GPU (INTEGRATION.md, "
                        "Co-residency) or set AVC_WN_GRID=0 for the per-layer launches.")
                # the library's default choice: warn and regenerate this call on the per-layer launches
                warnings.warn(msg + "; regenerating this call on the per-layer launches (INTEGRATION.md, "
                              "Co-residency).", RuntimeWarning, stacklevel=2)
                _lib.call("autovc_wavenet_set_grid", 0)
                try:
                    return self.generate(c, T=T, seed=seed, utt_base=utt_base, teacher=teacher,
                                         return_mol=return_mol, log_scale_min=log_scale_min, chunk=chunk,
                                         graph_steps=graph_steps)
                finally:
                    _lib.call("autovc_wavenet_reset_grid")
        return (y, mol) if return_mol else y

    def incremental_forward(self, initial_input=None, c=None, g=None, T=100, test_inputs=None,
                            tqdm=lambda x: x, softmax=True, quantize=True, log_scale_min=-7.0, seed=None):
        """wavenet.py incremental_forward: returns (B, 1, T) samples (scalar input / MoL)."""
        if g is not None:
            raise NotImplementedError("global conditioning is not on the AutoVC path")
        if c is None:
            raise NotImplementedError("the AutoVC vocoder is locally conditioned (c is required)")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        B = c.shape[0]
        teacher = None
        if test_inputs is not None:
            teacher = test_inputs.reshape(test_inputs.shape[0], -1)
        elif initial_input is not None and bool((initial_input != 0).any()):
            teacher = initial_input.reshape(-1)[:1].expand(B).reshape(B, 1)
        y = self.generate(c, T=T, seed=seed, teacher=teacher, log_scale_min=log_scale_min)
        return y.unsqueeze(1)
