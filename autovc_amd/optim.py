"""Fused Adam over one flat parameter buffer (libautovc_hip.so `autovc_adam_f32`).

Replaces torch.optim.Adam as built at solver_encoder.py:130 (betas (0.9, 0.999), eps 1e-8,
no weight decay, torch 1.8.1 update order) and stepped at :300.  On construction every
parameter of each group is re-pointed into one contiguous fp32 buffer (16-byte aligned
slots), and its .grad into a second one, so that:
  * the optimizer step is ONE HBM-bound kernel over 28.4 M parameters (28 B/param),
  * data-parallel training all-reduces ONE contiguous gradient buffer (autovc_amd.ddp),
  * zero_grad is one memset and keeps the views (autograd accumulates into them in place).
state_dict()/load_state_dict() keep torch.optim.Adam's layout ('step', 'exp_avg',
'exp_avg_sq' per parameter), so reference checkpoints' optimizer entries load.
"""
from __future__ import annotations

import math

import torch

from . import _lib


def _ceil4(n):
    return (n + 3) // 4 * 4


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by AutoVC")
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self._flat = []
        for group in self.param_groups:
            self._flat.append(self._flatten(group["params"]))

    @staticmethod
    def _flatten(params):
        if not params:
            return None
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedAdam runs on the GPU: move the model to cuda before building it")
        offs, total = [], 0
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise TypeError("FusedAdam: all parameters must be float32 on one device")
            offs.append(total)
            total += _ceil4(p.numel())
        flat_p = torch.zeros(total, dtype=torch.float32, device=dev)
        flat_g = torch.zeros(total, dtype=torch.float32, device=dev)
        flat_m = torch.zeros(total, dtype=torch.float32, device=dev)
        flat_v = torch.zeros(total, dtype=torch.float32, device=dev)
        for p, o in zip(params, offs):
            n = p.numel()
            flat_p[o:o + n].copy_(p.detach().reshape(-1))
            p.data = flat_p[o:o + n].view_as(p)
            p.grad = flat_g[o:o + n].view_as(p)
            p._avc_flat = True  # autovc_amd.functional accumulates this gradient in place
        return dict(p=flat_p, g=flat_g, m=flat_m, v=flat_v, offs=offs, step=0, params=list(params))

    # -- flat buffers (used by autovc_amd.ddp)
    def flat_grads(self):
        return [f["g"] for f in self._flat if f is not None]

    def flat_params(self):
        return [f["p"] for f in self._flat if f is not None]

    def zero_grad(self, set_to_none: bool = False):
        for f in self._flat:
            if f is None:
                continue
            f["g"].zero_()
            for p, o in zip(f["params"], f["offs"]):
                if p.grad is None or p.grad.data_ptr() != f["g"].data_ptr() + 4 * o:
                    p.grad = f["g"][o:o + p.numel()].view_as(p)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.begin_step()
        for gi, f in enumerate(self._flat):
            if f is not None:
                self.update_range(gi, 0, f["p"].numel())
        return loss

    # -- split step (autovc_amd.ddp overlaps the gradient all-reduce of one bucket with the
    #    update of the previous one): begin_step() once, then update_range() per slice
    @torch.no_grad()
    def begin_step(self):
        from .functional import join_grad_stream   # weight gradients may still be in flight
        join_grad_stream()
        for f in self._flat:
            if f is None:
                continue
            self._reattach_grads(f)
            f["step"] += 1

    @torch.no_grad()
    def update_range(self, group_index, start, count):
        """Adam on flat elements [start, start + count) of one group (start a multiple of 4,
        so every slice stays 16-byte aligned); the step count was advanced by begin_step."""
        group, f = self.param_groups[group_index], self._flat[group_index]
        if start % 4 or start < 0 or count <= 0 or start + count > f["p"].numel():
            raise ValueError(f"FusedAdam.update_range: bad slice [{start}, {start + count})")
        b1, b2 = group["betas"]
        bc1 = 1.0 - b1 ** f["step"]
        bc2_sqrt = math.sqrt(1.0 - b2 ** f["step"])
        o = 4 * start
        _lib.call("autovc_adam_f32", count, f["p"].data_ptr() + o, f["g"].data_ptr() + o,
                  f["m"].data_ptr() + o, f["v"].data_ptr() + o, float(group["lr"]), float(b1), float(b2),
                  float(group["eps"]), float(group["weight_decay"]), float(bc1), float(bc2_sqrt),
                  _lib.stream_ptr(f["p"].device))

    def _reattach_grads(self, f):
        """If autograd replaced a .grad (e.g. zero_grad(set_to_none) by a caller), copy it
        back into the flat buffer so the fused step sees it."""
        base = f["g"].data_ptr()
        for p, o in zip(f["params"], f["offs"]):
            if p.grad is None:
                continue
            if p.grad.data_ptr() != base + 4 * o:
                f["g"][o:o + p.numel()].copy_(p.grad.reshape(-1))
                p.grad = f["g"][o:o + p.numel()].view_as(p)

    # -- torch.optim.Adam-compatible state
    def state_dict(self):
        for f in self._flat:
            if f is None:
                continue
            for p, o in zip(f["params"], f["offs"]):
                n = p.numel()
                self.state[p] = {"step": f["step"], "exp_avg": f["m"][o:o + n].view_as(p),
                                 "exp_avg_sq": f["v"][o:o + n].view_as(p)}
        return super().state_dict()

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        saved = state_dict["state"]
        if len(groups) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        for group, sg, f in zip(self.param_groups, groups, self._flat):
            for k in ("lr", "betas", "eps", "weight_decay"):
                if k in sg:
                    group[k] = sg[k]
            if f is None:
                continue
            if len(sg["params"]) != len(f["params"]):
                raise ValueError("loaded state dict contains a group that doesn't match the size of the optimizer's group")
            step = 0
            for pid, p, o in zip(sg["params"], f["params"], f["offs"]):
                st = saved.get(pid)
                if not st:
                    continue
                n = p.numel()
                f["m"][o:o + n].copy_(st["exp_avg"].reshape(-1).to(f["m"]))
                f["v"][o:o + n].copy_(st["exp_avg_sq"].reshape(-1).to(f["v"]))
                s = st["step"]
                step = int(s.item() if torch.is_tensor(s) else s)
            f["step"] = step
