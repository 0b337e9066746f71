"""precision "fp32" GEMMs on bf16 MFMA (gemm_bf16_kernel X6: each fp32 operand staged as three
exact bf16 planes, six products in two accumulators) against the fp64 product and against the
fp32-MFMA kernel on the same operands: the error stays that of an fp32 GEMM (max and mean,
relative to the output's max), for every operand layout, the three tile configurations,
masked edges, split-K with accumulate and bias, implicit-im2col operands and the batched
(Winograd) form."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mode(on):
    from autovc_amd import _lib
    return _lib.load().autovc_gemm_set_fp32_x6(int(on))


@pytest.fixture
def x6_off_after():
    from autovc_amd import _lib
    prev = _lib.load().autovc_gemm_set_fp32_x6(0)
    yield
    _lib.load().autovc_gemm_set_fp32_x6(prev)


def _errs(C, ref):
    d = (C.double() - ref).abs()
    s = ref.abs().max().item()
    return d.max().item() / s, d.mean().item() / s


def _run(M, N, K, A, lda, at, B, ldb, bt, C0=None, bias=None, splits=1, a_conv=(0, 0, 0), b_conv=(0, 0, 0)):
    from autovc_amd import _lib
    dev = A.device
    out = {}
    for on in (0, 1):
        _mode(on)
        C = C0.clone() if C0 is not None else torch.full((M, N), float("nan"), device=dev)
        ws = torch.empty(4 * max(1, _lib.load().autovc_gemm_workspace_floats(M, N, splits)), dtype=torch.uint8,
                         device=dev)
        _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), lda, at, *a_conv, B.data_ptr(), ldb, bt, *b_conv,
                  C.data_ptr(), N, bias.data_ptr() if bias is not None else 0, 0, int(C0 is not None), splits,
                  ws.data_ptr(), _lib.stream_ptr(dev))
        torch.cuda.synchronize()
        out[on] = C
    return out[0], out[1]


def _check(c32, cx6, ref):
    m32, a32 = _errs(c32, ref)
    mx, ax = _errs(cx6, ref)
    assert bool(torch.isfinite(cx6).all())
    assert mx <= 1.5 * m32 + 1e-7, (mx, m32)
    assert ax <= 1.5 * a32 + 1e-9, (ax, a32)
    assert mx < 5e-6, mx


@pytest.mark.parametrize("M,N,K", [(4096, 1024, 8192), (8192, 512, 2048), (1024, 512, 1536), (300, 200, 36),
                                   (100, 260, 520), (64, 80, 1024)])
@pytest.mark.parametrize("at,bt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_x6_matches_fp32_accuracy(cuda, x6_off_after, M, N, K, at, bt):
    g = torch.Generator(device=cuda).manual_seed(M * 7 + N + K + 3 * at + bt)
    # rows of widely different magnitude: the split must hold for every exponent
    A = torch.randn(M, K, generator=g, device=cuda) * torch.logspace(-6, 6, M, device=cuda)[:, None]
    B = torch.randn(K, N, generator=g, device=cuda)
    Ad = (A.t() if at else A).contiguous()
    Bd = (B if bt else B.t()).contiguous()
    ref = A.double() @ B.double()
    rowscale = ref.abs().amax(dim=1, keepdim=True)
    c32, cx6 = _run(M, N, K, Ad, M if at else K, at, Bd, N if bt else K, bt)
    # per-row relative error (the rows span 12 decades)
    _check(c32 / rowscale, cx6 / rowscale, ref / rowscale)


def test_x6_splitk_accumulate_bias(cuda, x6_off_after):
    g = torch.Generator(device=cuda).manual_seed(5)
    M, N, K = 4096, 512, 8192
    A = torch.randn(K, M, generator=g, device=cuda)      # [K][M] (a_trans)
    B = torch.randn(K, N, generator=g, device=cuda)      # [K][N] (b_trans)
    C0 = torch.randn(M, N, generator=g, device=cuda) * 30
    bias = torch.randn(N, generator=g, device=cuda)
    ref = C0.double() + A.double().t() @ B.double() + bias.double()
    for splits in (2, 4):
        c32, cx6 = _run(M, N, K, A, M, 1, B, N, 1, C0=C0, bias=bias, splits=splits)
        _check(c32, cx6, ref)


def test_x6_conv_operand(cuda, x6_off_after):
    """A as the implicit im2col view of an NTC activation (k = 5, pad 2): the conv forward."""
    g = torch.Generator(device=cuda).manual_seed(9)
    Bn, T, Ci, Co = 4, 128, 512, 512
    x = torch.randn(Bn, T, Ci, generator=g, device=cuda)
    W = torch.randn(Co, Ci, 5, generator=g, device=cuda) / 50
    Wf = W.permute(0, 2, 1).contiguous()                   # (Co, 5, Ci): B[n][k], k = tap * Ci + c
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), W.double(), padding=2).transpose(1, 2)
    ref = ref.reshape(Bn * T, Co)
    c32, cx6 = _run(Bn * T, Co, 5 * Ci, x, Ci, 0, Wf, 5 * Ci, 0, a_conv=(T, Ci, -2))
    _check(c32, cx6, ref)


def test_x6_batched_winograd_conv(cuda, x6_off_after):
    """The Winograd conv path (8 batched GEMMs per call) end to end under both modes."""
    from autovc_amd import functional as AF
    g = torch.Generator(device=cuda).manual_seed(11)
    Bn, T, Ci, Co = 2, 128, 512, 512
    x = torch.randn(Bn, T, Ci, generator=g, device=cuda)
    W = torch.randn(Co, Ci, 5, generator=g, device=cuda) / 50
    b = torch.randn(Co, generator=g, device=cuda)
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), W.double(), b.double(), padding=2).transpose(1, 2)
    outs = []
    for on in (0, 1):
        _mode(on)
        outs.append(AF.conv_only(x, W, b))
        torch.cuda.synchronize()
    _check(outs[0], outs[1], ref)


def test_x6_mode_switch_returns_previous(cuda, x6_off_after):
    assert _mode(1) == 0
    assert _mode(0) == 1
