"""bf16 compute mode (BASELINE config 3: bf16 matmul operands, fp32 accumulation, fp32
master weights / optimizer / BatchNorm / losses).  The GEMM is checked exactly against
fp64 products of the RNE-rounded operands (a bf16 x bf16 product is exact in fp32, so only
the fp32 accumulation order differs); the training loss curve against fp32 (SURVEY §8d:
within 5 % at matched steps over >= 100 steps)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def r16(t):
    return t.bfloat16().double()


@pytest.mark.parametrize("M,N,K,at,bt", [(256, 128, 64, 0, 0), (300, 200, 36, 0, 1), (100, 260, 520, 1, 0),
                                         (64, 80, 1024, 1, 1), (8192, 512, 2560, 0, 0), (512, 2560, 8192, 1, 1),
                                         # the library-planned 256-row tiles: LSTM dW (256x256, 4
                                         # splits), dX (256x256, 2), input projection (256x128,
                                         # unsplit), and ragged edges on 256x128 with 4 splits
                                         (4096, 1024, 8192, 1, 1), (8192, 1024, 4096, 0, 1),
                                         (8192, 4096, 1024, 0, 0), (1000, 700, 3000, 1, 0),
                                         (777, 1028, 2048, 0, 1)])
def test_gemm_bf16_layouts(cuda, M, N, K, at, bt):
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    Ad = (A.t() if at else A).contiguous().to(cuda)
    Bd = (B if bt else B.t()).contiguous().to(cuda)
    C = torch.empty(M, N, device=cuda)
    with AF.precision("bf16"):
        AF.gemm(M, N, K, Ad, M if at else K, at, Bd, N if bt else K, bt, C, N, bias1=bias.to(cuda))
    ref = r16(A) @ r16(B) + bias.double()
    assert rel(C, ref) < 2e-5
    # and it is really bf16: the fp32-operand product differs by far more than that
    assert rel(C, A.double() @ B.double() + bias.double()) > 1e-4


def test_gemm_bf16_splitk_accumulate(cuda):
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(1)
    A = torch.randn(4096, 96, generator=g)
    B = torch.randn(4096, 160, generator=g)
    C0 = torch.randn(96, 160, generator=g)
    C = C0.clone().to(cuda)
    with AF.precision("bf16"):
        AF.gemm(96, 160, 4096, A.to(cuda), 96, 1, B.to(cuda), 160, 1, C, 160, accumulate=True, splits=8)
    assert rel(C, C0.double() + r16(A).t() @ r16(B)) < 2e-5


def test_conv_bf16_fwd_bwd(cuda):
    """Implicit-im2col conv under bf16: y from rounded (x, W), dX from rounded (dy, W),
    dW from rounded (dy, x) — each checked against fp64 on exactly those operands."""
    from autovc_amd import functional as AF
    F = torch.nn.functional
    torch.manual_seed(0)
    Bn, T, Ci, Co = 3, 40, 36, 52
    x = torch.randn(Bn, T, Ci)
    W = torch.randn(Co, Ci, 5)
    b = torch.randn(Co)
    gy = torch.randn(Bn, T, Co)
    xd, Wd, bd = (t.clone().to(cuda).requires_grad_() for t in (x, W, b))
    with AF.precision("bf16"):
        yd = AF.conv_only(xd, Wd, bd)
        yd.backward(gy.to(cuda))

    def conv(xx, ww):
        return F.conv1d(xx.transpose(1, 2), ww, b.double(), padding=2).transpose(1, 2)
    assert rel(yd, conv(r16(x), r16(W))) < 2e-5
    xr = r16(x).requires_grad_()
    conv(xr, r16(W)).backward(r16(gy))
    assert rel(xd.grad, xr.grad) < 2e-5
    Wr = r16(W).requires_grad_()
    conv(r16(x), Wr).backward(r16(gy))
    assert rel(Wd.grad, Wr.grad) < 2e-5


@pytest.mark.parametrize("B", [16, 64])
def test_bf16_training_loss_tracks_fp32(cuda, B):
    """100 Solver steps from the same weights and batch in fp32 and in bf16: the loss
    curves agree within 5 % at every step.  B=64 is config 3's
    per-GPU batch, where the bf16 persistent lstm2 forward and the bf16 stacked backward
    are the product path (the graph-replayed step, as bench.py runs it)."""
    import bench
    from autovc_amd import functional as AF
    if B == 64:
        assert AF.lstm2_persistent(64, 1024), "the B=64 step should run the persistent lstm2 forward"
    curves = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        solver = bench.make_solver(cuda, B)
        solver.precision = prec
        solver.hip_graph = True
        solver.G.train()
        x, e = bench.synthetic_batch(B, 128, cuda, 1234)
        losses = []
        for _ in range(100):
            losses.append(solver.train_step(x, e)[0].detach().reshape(()).clone())   # graph outputs are reused
        curves[prec] = torch.stack(losses).cpu().double()
        AF.check_device_faults(cuda)
    r = (curves["bf16"] - curves["fp32"]).abs() / curves["fp32"]
    assert float(r.max()) < 0.05, f"max rel loss gap {float(r.max()):.3f} at step {int(r.argmax())}"
    assert float(curves["bf16"][-1]) < float(curves["bf16"][0])   # it trains


@pytest.mark.parametrize("B,T,I,H,stacked", [(64, 16, 320, 512, False), (9, 12, 512, 1024, False), (9, 12, 256, 512, True),
                                               (9, 12, 512, 1024, True), (5, 1, 64, 128, False), (3, 2, 64, 128, True)])
def test_lstm_bf16_recurrence(cuda, B, T, I, H, stacked):
    """bf16 recurrences (bf16 copies of h / W / dG in the recurrent products, fp32 cell
    math): within bf16 rounding of the fp32 oracle, and genuinely different from fp32."""
    from autovc_amd import functional as AF
    from oracle import generator as og
    torch.manual_seed(7)
    s = 1 / H ** 0.5
    nl = 2 if stacked else 1
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,)] + ([(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)] if stacked else [])
    ps = [(torch.rand(*sh) * 2 - 1).mul_(s).requires_grad_() for sh in shapes]
    x = torch.randn(B, T, I, requires_grad=True)
    h = x
    for l in range(nl):
        h = og.OracleGenerator._lstm_dir(h, *ps[4 * l:4 * l + 4], reverse=False)
    gh = torch.randn_like(h)
    h.backward(gh)
    outs = {}
    for prec in ("fp32", "bf16"):
        xd = x.detach().to(cuda).requires_grad_()
        pd = [p.detach().to(cuda).requires_grad_() for p in ps]
        with AF.precision(prec):
            hd = AF.LSTM2StackFn.apply(xd, *pd, True) if stacked else AF.LSTMLayerFn.apply(xd, *pd, True)
            hd.backward(gh.to(cuda))
        outs[prec] = (hd, xd.grad, [p.grad for p in pd])
    hd, dx, dps = outs["bf16"]
    assert rel(hd, h) < 3e-2, (rel(hd, h), rel(outs["fp32"][0], h))
    assert rel(dx, x.grad) < 5e-2
    for a, b in zip(dps, ps):
        assert rel(a, b.grad) < 5e-2
    assert rel(outs["bf16"][0], outs["fp32"][0]) > 1e-5


@pytest.mark.parametrize("B,H", [(64, 1024), (9, 512)])
def test_lstm2_bf16_stacked_backward_wide_tiles(cuda, monkeypatch, B, H):
    """bf16 stacked backward: the wide-tile products (split-K 8, 64 x 64 per workgroup)
    against the 32 x 32 tiles (split-K 4) — the same bf16 operands, so the gradients differ
    only by the fp32 summation order of the partials."""
    from autovc_amd import functional as AF
    torch.manual_seed(8)
    T, I = 10, 512
    s = 1 / H ** 0.5
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,), (4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    ps = [((torch.rand(*sh) * 2 - 1) * s).to(cuda) for sh in shapes]
    x = torch.randn(B, T, I, device=cuda)
    gh = torch.randn(B, T, H, device=cuda)
    grads = {}
    for splits in ("4", "8"):
        monkeypatch.setenv("AVC_LSTM2_SPLITS", splits)
        xd = x.clone().requires_grad_()
        pd = [p.clone().requires_grad_() for p in ps]
        with AF.precision("bf16"):
            AF.LSTM2StackFn.apply(xd, *pd, True).backward(gh)
            AF.join_grad_stream()
        grads[splits] = [xd.grad] + [p.grad for p in pd]
    for a, b in zip(grads["8"], grads["4"]):
        assert rel(a, b) < 5e-3   # a partial sum order flips a few bf16 roundings of dG


@pytest.mark.parametrize("M,N,K,at,bt,bconv,acc", [
    (4096, 1024, 8192, 1, 1, None, 1),          # LSTM dW_ih (planned 256x256, 2 splits), accumulate
    (2048, 512, 64 * 128, 1, 1, (128, 512, -1), 0),   # dW_hh: B = h one step back (conv form)
    (8192, 1024, 4096, 0, 1, None, 0),          # dx = dG W_ih (256x256, split)
    (8192, 320, 2048, 0, 1, None, 0),           # decoder lstm1 dx (320 inputs)
    (1000, 520, 520, 0, 0, None, 1),            # ragged, 64-tile fallback, accumulate
])
def test_gemm_bf16src_equals_fp32_source(cuda, M, N, K, at, bt, bconv, acc):
    """autovc_gemm_bf16src_f32 reading a bf16 copy RNE(A) gives autovc_gemm_bf16_f32's result
    on the fp32 A bit for bit (the staging rounds A the same way)."""
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(M + N + K)
    A = (torch.randn(K, M, generator=g) if at else torch.randn(M, K, generator=g)).to(cuda)
    Bm = (torch.randn(K, N, generator=g) if bt else torch.randn(N, K, generator=g)).to(cuda)
    C0 = torch.randn(M, N, generator=g).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    kw = dict(b_conv=bconv, accumulate=bool(acc), bias1=None if at else bias)
    with AF.precision("bf16"):
        C1 = C0.clone()
        AF.gemm(M, N, K, A, A.shape[1], at, Bm, Bm.shape[1], bt, C1, N, **kw)
        srcs = [{"a_bf16": A.bfloat16()}]
        if bconv is None:   # a bf16 B (the per-step weight copies) alone and with a bf16 A
            srcs += [{"b_bf16": Bm.bfloat16()}, {"a_bf16": A.bfloat16(), "b_bf16": Bm.bfloat16()}]
        outs = []
        for src in srcs:
            C2 = C0.clone()
            AF.gemm(M, N, K, A, A.shape[1], at, Bm, Bm.shape[1], bt, C2, N, **src, **kw)
            outs.append(C2)
    torch.cuda.synchronize()
    for C2 in outs:
        assert torch.equal(C1, C2)


def test_gemm_bf16src_rejects_unaligned_lead(cuda):
    from autovc_amd import _lib
    A = torch.zeros(64, 68, device=cuda, dtype=torch.bfloat16)
    B = torch.zeros(68, 64, device=cuda)
    C = torch.zeros(64, 64, device=cuda)
    with pytest.raises(ValueError, match="multiples of 8"):   # lda 68
        _lib.call("autovc_gemm_bf16src_f32", 64, 64, 68, A.data_ptr(), 68, 0, B.data_ptr(), 64, 1, 0, 0, 0,
                  C.data_ptr(), 64, 0, 0, 0, 1, 0, 1, 0)
