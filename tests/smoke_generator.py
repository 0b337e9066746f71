"""Smoke checks used by __graft_entry__.smoke(): one small Generator training step and a
short WaveNet synthesis on cuda:0, each checked against the CPU oracle."""
from __future__ import annotations

import numpy as np
import torch

from oracle import generator as og
from oracle import wavenet as ow


def _rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def generator_step(dev, B=2, T=64):
    """Solver step losses + gradients (B=2, T=64) vs the oracle (SURVEY §8d bars)."""
    from autovc_amd import functional as AF
    from autovc_amd.model_vc_mel import Generator
    g = torch.Generator().manual_seed(5)
    x = torch.clamp(torch.randn(B, T, 80, generator=g) * 0.18 + 0.43, 0, 1)
    e = torch.randn(B, 256, generator=g)
    e = e / e.norm(dim=1, keepdim=True) * 0.8
    P = og.make_weights()
    params = {k: v for k, v in P.items() if v.dtype == torch.float32 and "running_" not in k}
    for v in params.values():
        v.requires_grad_(True)
    ref = og.solver_losses(og.OracleGenerator(P), x, e)
    ref[0].backward()
    G = Generator(32, 256, 512, 32)
    G.load_state_dict(og.make_weights())
    G = G.to(dev)
    xd, ed = x.to(dev), e.to(dev)
    x_id, x_psnt, code = G(xd, ed, ed)
    la = AF.mse_loss(xd, x_id.squeeze())
    lb = AF.mse_loss(xd, x_psnt.squeeze())
    lc = AF.l1_loss(code, G(x_psnt, ed, None))
    (la + lb + lc).backward()
    err = _rel(torch.stack([la, lb, lc]), torch.stack(list(ref[1:])))
    assert err < 1e-4, f"generator losses rel err {err}"
    w = "decoder.lstm2.weight_hh_l0"
    gerr = float((dict(G.named_parameters())[w].grad.cpu() - params[w].grad).norm() / params[w].grad.norm())
    assert gerr < 1e-2, f"{w} grad rel err {gerr}"
    print(f"smoke: generator step ok (loss rel err {err:.1e}, lstm2 dW_hh rel err {gerr:.1e})")


def wavenet_steps(dev, B=2, T=256):
    """Teacher-forced MoL outputs of a 6-layer WaveNet vs the oracle (<= 1e-4 rel)."""
    from autovc_amd.wavenet import WaveNet
    hp = ow.small_hparams(layers=6, stacks=2)
    m = WaveNet(out_channels=30, layers=6, stacks=2, residual_channels=512, gate_channels=512,
                skip_out_channels=256, cin_channels=80, upsample_conditional_features=True,
                upsample_scales=[4, 4, 4, 4], scalar_input=True)
    m.make_generation_fast_()
    W = ow.make_weights(hp)
    m.load_state_dict(W)
    m = m.to(dev).eval()
    rs = np.random.RandomState(1)
    c = torch.from_numpy(rs.rand(B, 80, T // 256).astype(np.float32))
    teacher = torch.from_numpy(rs.uniform(-0.9, 0.9, (B, T)).astype(np.float32))
    _, mol = m.generate(c.to(dev), seed=3, teacher=teacher.to(dev), return_mol=True,
                        log_scale_min=hp["log_scale_min"])
    o = ow.OracleWaveNet(W, hp)
    _, mol_ref = o.incremental(o.upsample(c), T, teacher=teacher.double(), return_mol=True)
    err = _rel(mol, mol_ref)
    assert err < 1e-4, f"wavenet MoL rel err {err}"
    print(f"smoke: wavenet ok (MoL rel err {err:.1e})")


def run(dev):
    generator_step(dev)
    wavenet_steps(dev)
