"""Retired with the time-chunked LSTM weight gradients (round 6; DESIGN.md section 4, round 5:
measured slower).  Runs against the library of commit 35d60fe only."""
import pytest
import torch


def _stack_grads_flat(cuda, prec, chunks, B=64, T=32, I=512, H=1024, seed=14):
    """decoder lstm2's gradients with the parameters in FusedAdam's flat buffer (the Solver's
    setting, where the time-chunked weight gradients apply)"""
    from autovc_amd import functional as AF
    from autovc_amd.optim import FusedAdam
    g = torch.Generator().manual_seed(seed)
    s = 1 / H ** 0.5
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,), (4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    ps = [torch.nn.Parameter(((torch.rand(*sh, generator=g) * 2 - 1) * s).to(cuda)) for sh in shapes]
    opt = FusedAdam(ps)
    opt.zero_grad()
    x = torch.randn(B, T, I, generator=g).to(cuda).requires_grad_()
    gh = torch.randn(B, T, H, generator=g).to(cuda)
    old = AF._DW_CHUNKS
    AF._DW_CHUNKS = chunks
    try:
        with AF.precision(prec):
            AF.LSTM2StackFn.apply(x, *ps, True).backward(gh)
            AF.join_grad_stream()
        torch.cuda.synchronize()
    finally:
        AF._DW_CHUNKS = old
    return [x.grad.clone()] + [p.grad.clone() for p in ps]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("chunks", [2, 4])
def test_time_chunked_weight_gradients(cuda, prec, chunks):
    """the four dW GEMMs of the stacked backward issued per time chunk (autovc_gemm_tchunk_*,
    accumulated in chunk order) against one whole-sequence GEMM each: equal up to fp32 (bf16:
    operand-rounding-order) summation differences; dx and the biases are not chunked and are
    bit-identical"""
    whole = _stack_grads_flat(cuda, prec, 0)
    chunked = _stack_grads_flat(cuda, prec, chunks)
    tol = 1e-5 if prec == "fp32" else 1e-4
    for k, (a, b) in enumerate(zip(chunked, whole)):
        if k in (0, 3, 4, 7, 8):           # dx and the four bias gradients
            assert torch.equal(a, b), k
        else:
            err = float((a - b).abs().max() / b.abs().max())
            assert err < tol, (k, err)


@pytest.mark.parametrize("tap0", [0, -1])
@pytest.mark.parametrize("t0,Tc", [(0, 4), (4, 4), (8, 4), (1, 11), (0, 12)])
def test_gemm_tchunk_matches_reference(cuda, tap0, t0, Tc):
    """autovc_gemm_tchunk_f32: C += sum over steps [t0, t0 + Tc) of every sequence of
    A[b, t]^T Bm[b, t + tap0] (zero before the first step), against float64 torch"""
    from autovc_amd import _lib
    g = torch.Generator().manual_seed(15)
    B, T, M, N = 5, 12, 256, 132
    A = torch.randn(B, T, M, generator=g)
    X = torch.randn(B, T, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    Xs = torch.zeros_like(X)
    if tap0 == -1:
        Xs[:, 1:] = X[:, :-1]
    else:
        Xs = X
    ref = C0.double() + torch.einsum("btm,btn->mn", A[:, t0:t0 + Tc].double(), Xs[:, t0:t0 + Tc].double())
    Ad, Xd, C = A.to(cuda), X.to(cuda), C0.to(cuda)
    _lib.call("autovc_gemm_tchunk_f32", M, N, B, T, t0, Tc, Ad.data_ptr(), M, Xd.data_ptr(), N, tap0, C.data_ptr(), N,
              1, 1, 0, _lib.stream_ptr(cuda))
    torch.cuda.synchronize()
    err = float((C.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-6, err
