"""The fused backward step of the large-H LSTM layers (one launch per step: split-K product
jobs hand their partials over write-through and each tile's last arriver runs the pointwise
cell backward, csrc/lstm.hip) against the product + pointwise launch pair it replaces:
every gradient bit-identical (same products, same partial values, same summation order,
same pointwise arithmetic).  The pair itself is pinned to the oracle and the reference
goldens by test_generator_gpu.py / test_bf16_gpu.py, which run the fused default."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(cuda, stacked, B, T, I, H, prec, fused, seed):
    from autovc_amd import _lib
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(seed)
    s = 1 / H ** 0.5
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,)]
    if stacked:
        shapes += [(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    ps = [((torch.rand(*sh, generator=g) * 2 - 1) * s).to(cuda).requires_grad_() for sh in shapes]
    x = torch.randn(B, T, I, generator=g).to(cuda).requires_grad_()
    gh = torch.randn(B, T, H, generator=g).to(cuda)
    _lib.call("autovc_lstm_bwd_set_fused", int(fused))
    try:
        with AF.precision(prec):
            fn = AF.LSTM2StackFn if stacked else AF.LSTMLayerFn
            fn.apply(x, *ps, True).backward(gh)
            AF.join_grad_stream()
        torch.cuda.synchronize()
    finally:
        _lib.call("autovc_lstm_bwd_set_fused", -1)
    return [x.grad] + [p.grad for p in ps]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,I,H", [(64, 16, 320, 512), (9, 12, 512, 1024), (40, 5, 64, 256), (3, 1, 64, 128),
                                     (33, 3, 96, 128)])
def test_single_layer_fused_bit_identical(cuda, prec, B, T, I, H):
    a = _run(cuda, False, B, T, I, H, prec, True, 11)
    b = _run(cuda, False, B, T, I, H, prec, False, 11)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("splits", ["4", "2"])
@pytest.mark.parametrize("B,T,I,H", [(64, 12, 512, 1024), (9, 7, 256, 512), (3, 2, 64, 128), (40, 1, 128, 256)])
def test_stacked_fused_bit_identical(cuda, monkeypatch, prec, splits, B, T, I, H):
    monkeypatch.setenv("AVC_LSTM2_SPLITS", splits)
    a = _run(cuda, True, B, T, I, H, prec, True, 12)
    b = _run(cuda, True, B, T, I, H, prec, False, 12)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_fused_repeatable_across_calls(cuda):
    """the per-tile counters return to zero after every step (a second call, reusing the
    workspace, gives the same gradients)"""
    a = _run(cuda, True, 64, 20, 512, 1024, "fp32", True, 13)
    b = _run(cuda, True, 64, 20, 512, 1024, "fp32", True, 13)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
