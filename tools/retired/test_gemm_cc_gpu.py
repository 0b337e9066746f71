"""The LDS-DMA weight-gradient GEMM (gemm_cc_kernel, autovc_gemm_set_cc(1..4)): C (+)= A^T B with
both operands K-strided — the LSTM dW shapes (B the one-frame-shifted h: conv view tap0 = -1),
the Conv1d dW shape (B = the 5-tap im2col view), ragged widths and split-K — against a float64
torch reference, and against the register-staged kernel it replaces (fp32 summation-order
noise apart).  Reference semantics: the weight gradients of model_vc_mel.py:61,104,118 and
its ConvNorm layers (torch autograd's dW = dY^T X)."""
import pytest
import torch

from autovc_amd import _lib
from autovc_amd import functional as AF

pytestmark = pytest.mark.gpu


def _ref(A, Bv, M, N, K, b_conv):
    """float64 C = A^T B(view): A (K, M); B (K-frames, C) with the conv view of autovc_gemm."""
    A64 = A.double()
    if b_conv is None:
        Bm = Bv.double()[:, :N]
    else:
        T, Cc, tap0 = b_conv
        X = Bv.double()
        Bm = torch.zeros(K, N, dtype=torch.float64, device=A.device)
        f = torch.arange(K, device=A.device)
        for q0 in range(0, N, Cc):
            tap = q0 // Cc
            src = f + tap0 + tap        # frame of this tap (the view walks ld == C into the next frames)
            ok = ((f % T) + tap + tap0 >= 0) & ((f % T) + tap + tap0 < T)
            rows = X[src.clamp(0, K - 1)]
            Bm[:, q0:q0 + Cc] = torch.where(ok[:, None], rows, torch.zeros_like(rows))
    return A64.t() @ Bm


@pytest.mark.parametrize("M,N,K,bc,splits,acc", [
    (4096, 1024, 8192, None, 1, True),          # lstm2 dW_ih1 (x = h0)
    (4096, 1024, 8192, "shift", 1, True),       # lstm2 dW_hh (h_{t-1})
    (2048, 320, 8192, None, 1, False),          # lstm1 dW_ih: N = 320 (not a tile multiple)
    (512, 2560, 8192, "conv5", 2, True),        # Conv1d dW, 5-tap im2col view, split-K 2
    (300, 200, 1000, None, 1, False),           # ragged everything, K not a stage multiple
    (128, 132, 64, "shift", 3, True),           # split-K 3 over a short K
])
def test_cc_kernel_matches_reference(cuda, M, N, K, bc, splits, acc):
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(K, M, device=cuda, generator=g)
    if bc == "conv5":
        Cc = N // 5
        X = torch.randn(K, Cc, device=cuda, generator=g)
        b_conv = (128, Cc, -2)
        ldb = Cc
    else:
        X = torch.randn(K, N, device=cuda, generator=g)
        b_conv = (128 if K % 128 == 0 else K, N, -1) if bc == "shift" else None
        ldb = N
    C0 = torch.randn(M, N, device=cuda, generator=g)
    ref = _ref(A, X, M, N, K, b_conv) + (C0.double() if acc else 0)
    out = {}
    try:
        for cc in (0, 1, 2, 3, 4):     # register-staged; LDS-DMA 3 x 32, 2 x 32, 4 x 16, 3 x 16 k
            _lib.call("autovc_gemm_set_cc", cc)
            C = C0.clone()
            AF.gemm(M, N, K, A, M, 1, X, ldb, 1, C, N, b_conv=b_conv, splits=splits, accumulate=acc)
            torch.cuda.synchronize()
            out[cc] = C
    finally:
        _lib.call("autovc_gemm_set_cc", 0)
    scale = ref.abs().max().item()
    for cc in out:
        err = (out[cc].double() - ref).abs().max().item() / scale
        assert err < 2e-5, (cc, err)
        # the kernels sum each k-stage in a different order: fp32 noise apart, no more
        assert (out[cc].double() - out[0].double()).abs().max().item() / scale < 2e-5, cc


def test_cc_kernel_repeatable(cuda):
    """Deterministic: the same call twice gives the same bits."""
    g = torch.Generator(device=cuda).manual_seed(5)
    A = torch.randn(8192, 4096, device=cuda, generator=g)
    X = torch.randn(8192, 1024, device=cuda, generator=g)
    try:
        _lib.call("autovc_gemm_set_cc", 1)
        outs = []
        for _ in range(2):
            C = torch.zeros(4096, 1024, device=cuda)
            AF.gemm(4096, 1024, 8192, A, 4096, 1, X, 1024, 1, C, 1024, b_conv=(128, 1024, -1))
            outs.append(C)
        torch.cuda.synchronize()
    finally:
        _lib.call("autovc_gemm_set_cc", 0)
    assert torch.equal(outs[0], outs[1])
