"""GPU parity of the Generator path (libautovc_hip.so kernels) against the oracle and the
reference goldens.  Tolerances as tests/test_oracle_generator.py."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import generator as og
from parity_tol import check_grad_slices

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(GOLDEN, "generator_golden.npz"))
FWD_TOL = 1e-4


def rel(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def build(dev, prefix=""):
    from autovc_amd.model_vc_mel import Generator
    g = Generator(32, 256, 512, 32)
    g.load_state_dict(og.make_weights())
    return g.to(dev)


# ------------------------------------------------------------------ GEMM unit tests
@pytest.mark.parametrize("M,N,K,at,bt", [(256, 128, 64, 0, 0), (300, 200, 36, 0, 1), (100, 260, 520, 1, 0),
                                         (64, 80, 1024, 1, 1), (8192, 512, 2560, 0, 0)])
def test_gemm_layouts(cuda, M, N, K, at, bt):
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    Ad = (A.t() if at else A).contiguous().to(cuda)
    Bd = (B if bt else B.t()).contiguous().to(cuda)
    C = torch.empty(M, N, device=cuda)
    AF.gemm(M, N, K, Ad, M if at else K, at, Bd, N if bt else K, bt, C, N, bias1=bias.to(cuda))
    ref = A.double() @ B.double() + bias.double()
    assert rel(C, ref) < 1e-5


def test_gemm_splitk_accumulate(cuda):
    from autovc_amd import functional as AF
    g = torch.Generator().manual_seed(1)
    A = torch.randn(4096, 96, generator=g)   # stored [K][M] (a_trans)
    B = torch.randn(4096, 160, generator=g)  # stored [K][N] (b_trans)
    C0 = torch.randn(96, 160, generator=g)
    C = C0.clone().to(cuda)
    AF.gemm(96, 160, 4096, A.to(cuda), 96, 1, B.to(cuda), 160, 1, C, 160, accumulate=True, splits=8)
    assert rel(C, C0.double() + A.double().t() @ B.double()) < 1e-5


def test_conv_implicit_im2col_fwd_bwd(cuda):
    from autovc_amd import functional as AF
    torch.manual_seed(0)
    B, T, Ci, Co = 3, 40, 36, 52
    x = torch.randn(B, T, Ci, requires_grad=True)
    W = torch.randn(Co, Ci, 5, requires_grad=True)
    b = torch.randn(Co, requires_grad=True)
    y = torch.nn.functional.conv1d(x.transpose(1, 2), W, b, padding=2).transpose(1, 2)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd, Wd, bd = (t.detach().to(cuda).requires_grad_() for t in (x, W, b))
    yd = AF.conv_only(xd, Wd, bd)
    yd.backward(gy.to(cuda))
    assert rel(yd, y) < 1e-5
    assert rel(xd.grad, x.grad) < 1e-5 and rel(Wd.grad, W.grad) < 1e-5 and rel(bd.grad, b.grad) < 1e-5


@pytest.mark.parametrize("wino", [True, False])
@pytest.mark.parametrize("B,T,Ci,Co", [(2, 4, 8, 12), (3, 8, 80, 512), (2, 128, 512, 512), (4, 42, 64, 32)])
def test_conv_winograd_and_im2col(cuda, monkeypatch, wino, B, T, Ci, Co):
    """ConvNorm fwd + input gradient through Winograd F(4,5) (T % 4 == 0) and through the
    im2col GEMM (AVC_WINOGRAD=0, or T = 42), both against the fp64 conv: 1e-5 relative."""
    from autovc_amd import functional as AF
    monkeypatch.setattr(AF, "_WINOGRAD", wino)
    g = torch.Generator().manual_seed(B * T + Ci)
    x = torch.randn(B, T, Ci, generator=g, dtype=torch.float64, requires_grad=True)
    W = (torch.randn(Co, Ci, 5, generator=g, dtype=torch.float64) / (5 * Ci) ** 0.5).requires_grad_()
    b = torch.randn(Co, generator=g, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv1d(x.transpose(1, 2), W, b, padding=2).transpose(1, 2)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    xd, Wd, bd = (t.detach().float().to(cuda).requires_grad_() for t in (x, W, b))
    yd = AF.conv_only(xd, Wd, bd)
    yd.backward(gy.float().to(cuda))
    assert rel(yd, y) < 1e-5 and rel(xd.grad, x.grad) < 1e-5
    assert rel(Wd.grad, W.grad) < 1e-5 and rel(bd.grad, b.grad) < 1e-5


def test_conv_padded_channels_513(cuda):
    """Channel counts % 4 != 0 (the 513/769-bin STFT generator) go through zero padding."""
    from autovc_amd import functional as AF
    torch.manual_seed(1)
    x = torch.randn(2, 32, 513, requires_grad=True)
    W = torch.randn(7, 513, 5, requires_grad=True)
    b = torch.randn(7, requires_grad=True)
    y = torch.nn.functional.conv1d(x.transpose(1, 2), W, b, padding=2).transpose(1, 2)
    y.sum().backward()
    xd, Wd, bd = (t.detach().to(cuda).requires_grad_() for t in (x, W, b))
    yd = AF.conv_only(xd, Wd, bd)
    yd.sum().backward()
    assert rel(yd, y) < 1e-5 and rel(xd.grad, x.grad) < 1e-5 and rel(Wd.grad, W.grad) < 1e-5


@pytest.mark.parametrize("act", ["relu", "tanh", "none"])
def test_conv_bn_act_train_fwd_bwd(cuda, act):
    from autovc_amd import functional as AF
    torch.manual_seed(2)
    conv = torch.nn.Conv1d(64, 96, 5, padding=2)
    bn = torch.nn.BatchNorm1d(96)
    x = torch.randn(4, 64, 48).transpose(1, 2).contiguous().requires_grad_()
    f = {"relu": torch.relu, "tanh": torch.tanh, "none": lambda v: v}[act]
    z = f(bn(conv(x.transpose(1, 2)))).transpose(1, 2)
    gz = torch.randn_like(z)
    z.backward(gz)
    conv_d, bn_d = torch.nn.Conv1d(64, 96, 5, padding=2).to(cuda), torch.nn.BatchNorm1d(96).to(cuda)
    conv_d.load_state_dict(conv.state_dict())
    with torch.no_grad():
        bn_d.running_mean.zero_()
        bn_d.running_var.fill_(1)
        bn_d.num_batches_tracked.zero_()
    xd = x.detach().to(cuda).requires_grad_()
    zd = AF.conv_bn_act(xd, conv_d, bn_d, act)
    zd.backward(gz.to(cuda))
    assert rel(zd, z) < FWD_TOL
    assert rel(xd.grad, x.grad) < 1e-4
    assert rel(conv_d.weight.grad, conv.weight.grad) < 1e-4
    assert rel(bn_d.weight.grad, bn.weight.grad) < 1e-4 and rel(bn_d.bias.grad, bn.bias.grad) < 1e-4
    assert rel(bn_d.running_mean, bn.running_mean) < 1e-5 and rel(bn_d.running_var, bn.running_var) < 1e-5
    assert int(bn_d.num_batches_tracked) == 1


def test_wino_weight_grad_reuses_forward_transform_bit_exact(cuda, monkeypatch):
    """The conv weight gradient fed with the forward's Winograd input transform (default)
    equals the one that transforms x again (_WINO_KEEP_XT False) bit for bit."""
    from autovc_amd import functional as AF
    torch.manual_seed(5)
    x = torch.randn(4, 64, 512).to(cuda)
    gz = torch.randn(4, 64, 512).to(cuda)
    grads = []
    for keep in (True, False):
        monkeypatch.setattr(AF, "_WINO_KEEP_XT", keep)
        torch.manual_seed(6)
        conv, bn = torch.nn.Conv1d(512, 512, 5, padding=2).to(cuda), torch.nn.BatchNorm1d(512).to(cuda)
        xd = x.clone().requires_grad_()
        AF.conv_bn_act(xd, conv, bn, "relu").backward(gz)
        grads.append((conv.weight.grad.clone(), xd.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


# ------------------------------------------------------------------ LSTM unit tests
@pytest.mark.parametrize("B,T,I,H", [(64, 16, 512, 1024), (3, 9, 320, 512), (17, 5, 64, 64)])
def test_lstm_layer_fwd_bwd(cuda, B, T, I, H):
    from autovc_amd import functional as AF
    torch.manual_seed(3)
    s = 1 / H ** 0.5
    x = torch.randn(B, T, I, requires_grad=True)
    ps = [(torch.rand(*sh) * 2 - 1).mul_(s).requires_grad_() for sh in ((4 * H, I), (4 * H, H), (4 * H,), (4 * H,))]
    h = og.OracleGenerator._lstm_dir(x, *ps, reverse=False)
    gh = torch.randn_like(h)
    h.backward(gh)
    xd = x.detach().to(cuda).requires_grad_()
    pd = [p.detach().to(cuda).requires_grad_() for p in ps]
    hd = AF.LSTMLayerFn.apply(xd, *pd, True)
    hd.backward(gh.to(cuda))
    assert rel(hd, h) < FWD_TOL
    assert rel(xd.grad, x.grad) < 1e-4
    for a, b in zip(pd, ps):
        assert rel(a.grad, b.grad) < 1e-4


@pytest.mark.parametrize("B,T,I,H", [(64, 16, 512, 1024), (3, 9, 320, 512), (2, 1, 64, 128), (33, 3, 64, 256)])
def test_lstm2_stack_fwd_bwd(cuda, B, T, I, H):
    """Two stacked layers as one wavefront (autovc_lstm2_fwd_f32) vs two oracle layers."""
    from autovc_amd import functional as AF
    torch.manual_seed(5)
    s = 1 / H ** 0.5
    x = torch.randn(B, T, I, requires_grad=True)
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,), (4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    ps = [(torch.rand(*sh) * 2 - 1).mul_(s).requires_grad_() for sh in shapes]
    h0 = og.OracleGenerator._lstm_dir(x, *ps[:4], reverse=False)
    h1 = og.OracleGenerator._lstm_dir(h0, *ps[4:], reverse=False)
    gh = torch.randn_like(h1)
    h1.backward(gh)
    xd = x.detach().to(cuda).requires_grad_()
    pd = [p.detach().to(cuda).requires_grad_() for p in ps]
    hd = AF.LSTM2StackFn.apply(xd, *pd, True)
    hd.backward(gh.to(cuda))
    assert rel(hd, h1) < FWD_TOL
    assert rel(xd.grad, x.grad) < 1e-4
    for a, b in zip(pd, ps):
        assert rel(a.grad, b.grad) < 1e-4


@pytest.mark.parametrize("splits", ["2", "4", "8"])
def test_lstm2_stacked_backward_matches_layerwise(cuda, monkeypatch, splits):
    """The backward wavefront (autovc_lstm2_bwd_f32) against the layer-by-layer backward
    (two autovc_lstm_bwd_f32 recurrences + the input-gradient GEMM) at decoder lstm2's
    size: the same sums up to the order of layer 0's dh partials (splits 8: the wide-tile
    product kernel, 64 x 64 per workgroup)."""
    from autovc_amd import functional as AF
    torch.manual_seed(6)
    B, T, I, H = 64, 12, 512, 1024
    s = 1 / H ** 0.5
    x = torch.randn(B, T, I, device=cuda)
    shapes = [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,), (4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    ps = [((torch.rand(*sh) * 2 - 1) * s).to(cuda) for sh in shapes]
    gh = torch.randn(B, T, H, device=cuda)
    grads = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("AVC_LSTM2_BWD", mode)
        monkeypatch.setenv("AVC_LSTM2_SPLITS", splits)
        xd = x.clone().requires_grad_()
        pd = [p.clone().requires_grad_() for p in ps]
        AF.LSTM2StackFn.apply(xd, *pd, True).backward(gh)
        AF.join_grad_stream()
        grads[mode] = [xd.grad] + [p.grad for p in pd]
    for a, b in zip(grads["1"], grads["0"]):
        assert rel(a, b) < 1e-5


@pytest.mark.parametrize("B,T,I", [(64, 128, 512), (5, 7, 64), (9, 21, 64)])
def test_blstm_layer_fwd_bwd(cuda, B, T, I):
    from autovc_amd import functional as AF
    torch.manual_seed(4)
    H = 32
    s = 1 / H ** 0.5
    x = torch.randn(B, T, I, requires_grad=True)
    shapes = ((4 * H, I), (4 * H, H), (4 * H,), (4 * H,))
    pf = [(torch.rand(*sh) * 2 - 1).mul_(s).requires_grad_() for sh in shapes]
    pb = [(torch.rand(*sh) * 2 - 1).mul_(s).requires_grad_() for sh in shapes]
    h = torch.cat([og.OracleGenerator._lstm_dir(x, *pf, reverse=False),
                   og.OracleGenerator._lstm_dir(x, *pb, reverse=True)], -1)
    gh = torch.randn_like(h)
    h.backward(gh)
    xd = x.detach().to(cuda).requires_grad_()
    pfd = [p.detach().to(cuda).requires_grad_() for p in pf]
    pbd = [p.detach().to(cuda).requires_grad_() for p in pb]
    hd = AF.BLSTMLayerFn.apply(xd, *pfd, *pbd, True)
    hd.backward(gh.to(cuda))
    assert rel(hd, h) < FWD_TOL
    assert rel(xd.grad, x.grad) < 1e-4
    for a, b in zip(pfd + pbd, pf + pb):
        assert rel(a.grad, b.grad) < 1e-4


def test_code_gather_bit_exact(cuda):
    from autovc_amd import functional as AF
    h = torch.randn(5, 128, 64)
    codes = AF.CodeGatherFn.apply(h.to(cuda), 32).cpu()
    ref = torch.cat([torch.cat((h[:, i + 31, :32], h[:, i, 32:]), -1) for i in range(0, 128, 32)], -1)
    assert torch.equal(codes, ref)
    hd = h.to(cuda).requires_grad_()
    g = torch.randn(5, 256)
    AF.CodeGatherFn.apply(hd, 32).backward(g.to(cuda))
    hr = h.clone().requires_grad_()
    torch.cat([torch.cat((hr[:, i + 31, :32], hr[:, i, 32:]), -1) for i in range(0, 128, 32)], -1).backward(g)
    assert torch.equal(hd.grad.cpu(), hr.grad)


def test_frame_concat_upsample_bit_exact(cuda):
    from autovc_amd import functional as AF
    codes = torch.randn(3, 4, 64)
    e = torch.randn(3, 256)
    out = AF.FrameConcatFn.apply(codes.to(cuda), e.to(cuda), 128, 32).cpu()
    ref = torch.cat((codes.repeat_interleave(32, 1), e.unsqueeze(1).expand(-1, 128, -1)), -1)
    assert torch.equal(out, ref)


# ------------------------------------------------------------------ Generator
def test_generator_train_forward_vs_reference_golden(cuda):
    g = build(cuda)
    g.train()
    x = torch.from_numpy(G["x"]).to(cuda)
    e = torch.from_numpy(G["emb"]).to(cuda)
    with torch.no_grad():
        x_id, x_psnt, code = g(x, e, e)
        code_rec = g(x_psnt, e, None)
    assert x_id.shape == (2, 1, 128, 80) and x_psnt.shape == (2, 1, 128, 80) and code.shape == (2, 256)
    assert rel(x_id, G["train_x_identic"]) < FWD_TOL
    assert rel(x_psnt, G["train_x_psnt"]) < FWD_TOL
    assert rel(code, G["train_code_real"]) < FWD_TOL
    assert rel(code_rec, G["train_code_reconst"]) < FWD_TOL


def test_generator_eval_and_t160(cuda):
    g = build(cuda)
    g.eval()
    e = torch.from_numpy(G["emb"]).to(cuda)
    with torch.no_grad():
        _, x_psnt, code = g(torch.from_numpy(G["x"]).to(cuda), e, e)
    assert rel(x_psnt, G["eval_x_psnt"]) < FWD_TOL and rel(code, G["eval_code_real"]) < FWD_TOL
    g2 = build(cuda)
    with torch.no_grad():
        _, x_psnt, code = g2(torch.from_numpy(G["x160"]).to(cuda), e, e)
    assert code.shape == (2, 320)
    assert rel(x_psnt, G["t160_x_psnt"]) < FWD_TOL and rel(code, G["t160_code_real"]) < FWD_TOL


def test_generator_t_not_multiple_of_freq_raises(cuda):
    g = build(cuda)
    with pytest.raises(IndexError):
        g(torch.rand(1, 130, 80, device=cuda), torch.rand(1, 256, device=cuda), None)


def test_one_training_step_grads_vs_reference_golden(cuda):
    from autovc_amd import functional as AF
    g = build(cuda)
    g.train()
    x = torch.from_numpy(G["x"]).to(cuda)
    e = torch.from_numpy(G["emb"]).to(cuda)
    x_id, x_psnt, code = g(x, e, e)
    l_id = AF.mse_loss(x.squeeze(), x_id.squeeze())
    l_psnt = AF.mse_loss(x, x_psnt.squeeze())
    l_cd = AF.l1_loss(code, g(x_psnt, e, None))
    (l_id + l_psnt + l_cd).backward()
    assert rel(torch.stack([l_id, l_psnt, l_cd]), G["train_losses"]) < FWD_TOL
    params = dict(g.named_parameters())
    for i, n in enumerate(G["param_names"]):
        gn = params[n].grad.norm().item()
        if n.endswith("0.conv.bias"):
            assert abs(gn - G["grad_norm"][i]) < 1e-6, n
        else:
            assert abs(gn - G["grad_norm"][i]) <= 1e-2 * G["grad_norm"][i], (n, gn, G["grad_norm"][i])
    # elementwise: first 64 gradient elements of every tensor vs the reference's float32 and
    # float64 backward (tests/parity_tol.py; pre-BN conv biases |g| <= 1e-6)
    check_grad_slices({n: p.grad.detach().cpu().numpy() for n, p in params.items()})
    bufs = dict(g.named_buffers())
    got = np.concatenate([bufs[k].float().flatten().cpu().numpy() for k in G["step1_buffer_names"]])
    assert rel(got, G["step1_buffers"]) < FWD_TOL  # encoder BN updated twice, decoder/postnet once


def test_full_size_step_vs_oracle(cuda):
    """B=64, T=128 (BASELINE config 2 shape): forward outputs and gradients vs the CPU oracle."""
    from autovc_amd import functional as AF
    gen = torch.Generator().manual_seed(1234)
    x = torch.clamp(torch.randn(64, 128, 80, generator=gen) * 0.18 + 0.43, 0, 1)
    e = torch.randn(64, 256, generator=gen)
    e = e / e.norm(dim=1, keepdim=True) * 0.8
    P = og.make_weights()
    params = {k: v for k, v in P.items() if v.dtype == torch.float32 and "running_" not in k}
    for v in params.values():
        v.requires_grad_(True)
    torch.set_num_threads(min(16, os.cpu_count() or 1))  # GPU boxes show many host CPUs
    g_loss, a, b, c = og.solver_losses(og.OracleGenerator(P), x, e)
    g_loss.backward()
    gd = build(cuda)
    xd, ed = x.to(cuda), e.to(cuda)
    x_id, x_psnt, code = gd(xd, ed, ed)
    la = AF.mse_loss(xd, x_id.squeeze())
    lb = AF.mse_loss(xd, x_psnt.squeeze())
    lc = AF.l1_loss(code, gd(x_psnt, ed, None))
    (la + lb + lc).backward()
    assert rel(torch.stack([la, lb, lc]), torch.stack([a, b, c])) < FWD_TOL
    for n, p in gd.named_parameters():
        ref = params[n].grad
        if n.endswith("0.conv.bias"):
            assert p.grad.norm().item() < 1e-4 + ref.norm().item() * 10, n
            continue
        err = (p.grad.cpu().double() - ref.double()).norm() / ref.double().norm()
        assert err < 1e-2, (n, float(err))


# ------------------------------------------------------------------ 513-bin variant, conversion caller
def test_generator_stft_513_vs_reference_golden(cuda):
    """model_vc_stft.GeneratorSTFT (513-bin, `model.` keys): the working arithmetic of the
    reference (G.model(x, e, e), Appendix A-1) against its golden, through .forward."""
    from autovc_amd.model_vc_stft import GeneratorSTFT
    g = GeneratorSTFT(32, 256, 512, 32)
    g.load_state_dict(og.make_weights(prefix="model.", n_in=513, n_out=513))
    g = g.to(cuda).train()
    x = torch.from_numpy(G["stft_x"]).to(cuda)
    e = torch.from_numpy(G["emb"]).to(cuda)
    with torch.no_grad():
        x_id, x_psnt, code = g(x, e, e)
    assert x_psnt.shape == G["stft_x_psnt"].shape and code.shape == G["stft_code_real"].shape
    assert rel(x_id, G["stft_x_identic"]) < FWD_TOL
    assert rel(x_psnt, G["stft_x_psnt"]) < FWD_TOL
    assert rel(code, G["stft_code_real"]) < FWD_TOL


def test_conversion_caller_flow(cuda):
    """conversion.py:40-44,90-102 as a caller would run it: pad to a multiple of 32, B=1
    eval forward with (emb_org, emb_trg), un-pad; the output is the oracle's."""
    g = build(cuda).eval()
    x = G["x160"][0, :150]                                  # (150, 80): not a multiple of 32
    len_pad = 32 - x.shape[0] % 32
    uttr = np.pad(x, ((0, len_pad), (0, 0)), "constant")
    e_org = torch.from_numpy(G["emb"][0:1]).to(cuda)
    e_trg = torch.from_numpy(G["emb"][1:2]).to(cuda)
    with torch.no_grad():
        _, x_psnt, _ = g(torch.from_numpy(uttr[None]).to(cuda), e_org, e_trg)
    out = x_psnt[0, 0, :-len_pad, :].cpu()
    ref_gen = og.OracleGenerator(og.make_weights(), training=False)
    with torch.no_grad():
        _, ref_psnt, _ = ref_gen.forward(torch.from_numpy(uttr[None]), torch.from_numpy(G["emb"][0:1]),
                                         torch.from_numpy(G["emb"][1:2]))
    assert out.shape == (150, 80)
    assert rel(out, ref_psnt[0, 0, :-len_pad, :]) < FWD_TOL


def _colsum_order(X, out0=None):
    """numpy restatement of autovc_colsum_f32's fixed summation order (float32): RS row blocks
    of 4 row-strided sums added in wave order, then 16 row groups of partials, groups in order."""
    M, N = X.shape
    RS = min(128, M)
    part = np.zeros((RS, N), np.float32)
    for rs in range(RS):
        r0, r1 = M * rs // RS, M * (rs + 1) // RS
        ws = []
        for w in range(4):
            s = np.zeros(N, np.float32)
            for r in range(r0 + w, r1, 4):
                s = s + X[r]
            ws.append(s)
        part[rs] = ((ws[0] + ws[1]) + ws[2]) + ws[3]
    groups = []
    for g in range(16):
        t = np.zeros(N, np.float32)
        for q in range(g, RS, 16):
            t = t + part[q]
        groups.append(t)
    tot = np.zeros(N, np.float32)
    for t in groups:
        tot = tot + t
    return tot if out0 is None else out0 + tot


@pytest.mark.parametrize("M,N", [(8192, 300), (37, 64), (5, 1000), (1000, 4096)])
def test_colsum_bit_exact(cuda, M, N):
    """autovc_colsum_f32 (the bias gradients' column sums: partial rows, then a fixed-order
    finalize) equals the numpy restatement of its summation order bit for bit, with
    accumulate and the second output, at ragged widths and row counts below the 128 splits."""
    from autovc_amd import functional as Fh
    rs = np.random.RandomState(M + N)
    X = rs.standard_normal((M, N)).astype(np.float32)
    base = rs.standard_normal(N).astype(np.float32)
    xd = torch.from_numpy(X).to(cuda)
    out = torch.from_numpy(base.copy()).to(cuda)
    out2 = torch.from_numpy(base.copy()).to(cuda)
    Fh.colsum(xd, out, out2, accumulate=True)
    want = _colsum_order(X, base)
    assert np.array_equal(out.cpu().numpy(), want) and np.array_equal(out2.cpu().numpy(), want)
    n3 = max(1, N // 3)
    o3 = torch.empty(n3, device=cuda)
    Fh.colsum(xd[:, :n3], o3)
    assert np.array_equal(o3.cpu().numpy(), _colsum_order(X[:, :n3]))
