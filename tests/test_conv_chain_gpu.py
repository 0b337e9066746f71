"""The fused Conv-BN stacks (functional.ConvBNChainFn: BatchNorm statistics in the Winograd
output transform, BatchNorm + activation applied by the next layer's input transform, the
BatchNorm backward and the conv bias sums folded into the gradient transforms) against the
per-layer path (ConvBNActFn: conv, then separate BatchNorm kernels), which the Generator
goldens pin to the reference.  Same modules, same inputs: outputs, input gradient,
every parameter gradient and the running statistics agree to fp32 summation-order noise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _stack(chans, acts, seed):
    g = torch.Generator().manual_seed(seed)
    layers = []
    for ci, co, act in zip(chans[:-1], chans[1:], acts):
        conv = torch.nn.Conv1d(ci, co, 5, padding=2)
        bn = torch.nn.BatchNorm1d(co)
        with torch.no_grad():
            conv.weight.copy_((torch.rand(co, ci, 5, generator=g) * 2 - 1) / (5 * ci) ** 0.5)
            conv.bias.copy_(torch.rand(co, generator=g) * 0.2 - 0.1)
            bn.weight.copy_(torch.rand(co, generator=g) * 0.5 + 0.75)
            bn.bias.copy_(torch.rand(co, generator=g) * 0.2 - 0.1)
        layers.append((conv, bn, act))
    return layers


def _run(layers, x, dz, residual, chain, training=True):
    from autovc_amd import functional as AF
    dev = x.device
    mods = [(c.to(dev), b.to(dev).train(training), a) for c, b, a in layers]
    for c, b, _ in mods:
        for p in list(c.parameters()) + list(b.parameters()):
            p.grad = None
    prev = AF._CHAIN_ON
    AF._CHAIN_ON = chain
    try:
        xr = x.clone().requires_grad_(training)
        res = residual.clone().requires_grad_(training) if residual is not None else None
        out = AF.conv_bn_chain(xr, mods, residual=res)
        grads = {}
        if training:
            out.backward(dz)
            grads["x"] = xr.grad
            if res is not None:
                grads["res"] = res.grad
            for i, (c, b, _) in enumerate(mods):
                for n, p in (("W", c.weight), ("b", c.bias), ("g", b.weight), ("be", b.bias)):
                    grads[f"{n}{i}"] = p.grad.clone()
        stats = [(b.running_mean.clone(), b.running_var.clone(), int(b.num_batches_tracked)) for _, b, _ in mods]
    finally:
        AF._CHAIN_ON = prev
    torch.cuda.synchronize()
    return out.detach(), grads, stats


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("name,chans,acts,res", [
    ("encoder", [336, 512, 512, 512], ["relu"] * 3, False),
    ("decoder", [320, 512, 512, 512], ["relu"] * 3, False),
    ("postnet", [80, 512, 512, 512, 512, 80], ["tanh"] * 4 + ["none"], True),
])
@pytest.mark.parametrize("B,T", [(2, 64), (8, 128)])
def test_chain_matches_per_layer_path(cuda, name, chans, acts, res, B, T):
    import copy
    g = torch.Generator().manual_seed(1)
    x = torch.clamp(torch.randn(B, T, chans[0], generator=g) * 0.18 + 0.43, 0, 1).to(cuda)
    dz = (torch.randn(B, T, chans[-1], generator=g) * 1e-3).to(cuda)
    residual = torch.randn(B, T, chans[-1], generator=g).to(cuda) if res else None
    layers = _stack(chans, acts, seed=3)
    o1, g1, s1 = _run(copy.deepcopy(layers), x, dz, residual, chain=True)
    o0, g0, s0 = _run(copy.deepcopy(layers), x, dz, residual, chain=False)
    assert _rel(o1, o0) < 1e-5
    for k in g0:
        if k.startswith("b") and not k.startswith("be"):
            # a conv bias feeding a BatchNorm has zero true gradient: both are rounding noise
            assert g1[k].abs().max().item() < 1e-6 and g0[k].abs().max().item() < 1e-6, k
            continue
        assert _rel(g1[k], g0[k]) < 2e-4, (k, _rel(g1[k], g0[k]))
    for (m1, v1, n1), (m0, v0, n0) in zip(s1, s0):
        assert n1 == n0 == 1
        assert _rel(m1, m0) < 1e-5 and _rel(v1, v0) < 1e-5


def test_chain_eval_mode_matches_per_layer_path(cuda):
    import copy
    g = torch.Generator().manual_seed(2)
    layers = _stack([80, 512, 512, 80], ["tanh", "tanh", "none"], seed=4)
    for _, bn, _ in layers:   # non-trivial running statistics
        bn.running_mean.uniform_(-0.2, 0.2, generator=g)
        bn.running_var.uniform_(0.5, 1.5, generator=g)
    x = torch.randn(4, 64, 80, generator=g).to(cuda)
    with torch.no_grad():
        o1, _, _ = _run(copy.deepcopy(layers), x, None, x, chain=True, training=False)
        o0, _, _ = _run(copy.deepcopy(layers), x, None, x, chain=False, training=False)
    assert _rel(o1, o0) < 1e-6


def _run_prec(layers, x, dz, residual, precision, chain_bf16, training=True):
    """chain_bf16: 0 = per-layer bf16 path, 1 / 2 = ConvBNChainBf16Fn mode 1 / 2."""
    from autovc_amd import functional as AF
    prev = AF._CHAIN_BF16_ON, AF._CHAIN_BF16_MODE
    AF._CHAIN_BF16_ON, AF._CHAIN_BF16_MODE = bool(chain_bf16), int(chain_bf16)
    try:
        with AF.precision(precision):
            return _run(layers, x, dz, residual, chain=True, training=training)
    finally:
        AF._CHAIN_BF16_ON, AF._CHAIN_BF16_MODE = prev


@pytest.mark.parametrize("name,chans,acts,res", [
    ("encoder", [336, 512, 512, 512], ["relu"] * 3, False),
    ("postnet", [80, 512, 512, 512, 512, 80], ["tanh"] * 4 + ["none"], True),
])
@pytest.mark.parametrize("B,T", [(2, 64), (8, 128), (64, 128)])
@pytest.mark.parametrize("mode", [1, 2])
def test_bf16_chain_as_accurate_as_per_layer_bf16(cuda, name, chans, acts, res, B, T, mode):
    """ConvBNChainBf16Fn (BatchNorm + activation applied while the bf16 conv GEMM stages its
    operand, statistics from the split-K reduce, BN backward sums from the input-gradient
    GEMM's reduce) against the fp32 per-layer path: its error is that of the per-layer bf16
    path (conv GEMMs on bf16 operands, separate BatchNorm kernels) — outputs, every gradient
    and the running statistics — and the forward is bit-identical from run to run."""
    import copy
    g = torch.Generator().manual_seed(1)
    x = torch.clamp(torch.randn(B, T, chans[0], generator=g) * 0.18 + 0.43, 0, 1).to(cuda)
    dz = (torch.randn(B, T, chans[-1], generator=g) * 1e-3).to(cuda)
    residual = torch.randn(B, T, chans[-1], generator=g).to(cuda) if res else None
    layers = _stack(chans, acts, seed=3)
    ref, gref, sref = _run(copy.deepcopy(layers), x, dz, residual, chain=False)        # fp32 per layer
    o1, g1, s1 = _run_prec(copy.deepcopy(layers), x, dz, residual, "bf16", mode)       # bf16 chain
    o0, g0, s0 = _run_prec(copy.deepcopy(layers), x, dz, residual, "bf16", 0)          # bf16 per layer
    o2, _, _ = _run_prec(copy.deepcopy(layers), x, dz, residual, "bf16", mode)
    assert torch.equal(o1, o2)
    e1, e0 = _rel(o1, ref), _rel(o0, ref)
    assert e1 < 1e-2 and e1 < 1.5 * e0 + 1e-4, (e1, e0)
    for k in gref:
        if k.startswith("b") and not k.startswith("be"):
            assert g1[k].abs().max().item() < 1e-5, k   # conv bias before a BatchNorm: zero true gradient
            continue
        e1, e0 = _rel(g1[k], gref[k]), _rel(g0[k], gref[k])
        # (the stack's input gradient carries ~10 % bf16 error on both paths: BatchNorm
        # backward cancellation of the zero-mean part)
        assert e1 < 0.3 and e1 < 1.5 * e0 + 1e-3, (k, e1, e0)
    for (m1, v1, n1), (m0, v0, n0), (mr, vr, nr) in zip(s1, s0, sref):
        assert n1 == n0 == nr == 1
        assert _rel(m1, mr) < 1.5 * _rel(m0, mr) + 1e-4 and _rel(v1, vr) < 1.5 * _rel(v0, vr) + 1e-4


@pytest.mark.parametrize("mode", [1, 2])
def test_bf16_chain_eval_mode(cuda, mode):
    import copy
    g = torch.Generator().manual_seed(2)
    layers = _stack([80, 512, 512, 80], ["tanh", "tanh", "none"], seed=4)
    for _, bn, _ in layers:
        bn.running_mean.uniform_(-0.2, 0.2, generator=g)
        bn.running_var.uniform_(0.5, 1.5, generator=g)
    x = torch.randn(4, 64, 80, generator=g).to(cuda)
    with torch.no_grad():
        ref, _, _ = _run(copy.deepcopy(layers), x, None, x, chain=False, training=False)
        o1, _, _ = _run_prec(copy.deepcopy(layers), x, None, x, "bf16", mode, training=False)
        o0, _, _ = _run_prec(copy.deepcopy(layers), x, None, x, "bf16", 0, training=False)
    assert _rel(o1, ref) < 1.5 * _rel(o0, ref) + 1e-4
