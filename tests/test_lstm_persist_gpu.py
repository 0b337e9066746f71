"""Decoder lstm2 forward as one persistent, weight-stationary launch
(autovc_lstm2_fwd_persist_f32, csrc/lstm2_persist.hip) against the per-step wavefront
launches (autovc_lstm2_fwd_f32), which the Generator tests pin to the reference: same
inputs, every output (h0, c0, gates0, h1, c1, gates1) within fp32 summation-order noise,
no barrier timeout, and graph replay identical to a direct call."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(B, T, H, dev, seed=5):
    g = torch.Generator().manual_seed(seed)
    s = 1.0 / H ** 0.5
    W = [((torch.rand(4 * H, H, generator=g) * 2 - 1) * s).to(dev) for _ in range(3)]
    b1, b2 = ((torch.rand(4 * H, generator=g) * 0.2 - 0.1).to(dev) for _ in range(2))
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    return gx, W, b1, b2


def _run(name, B, T, H, gx, W, b1, b2, dev, ws=None):
    from autovc_amd import _lib
    outs = [torch.full((B, T, H), float("nan"), device=dev) for _ in range(4)]
    gts = [torch.full((B, T, 4 * H), float("nan"), device=dev) for _ in range(2)]
    h0, c0, h1, c1 = outs
    g0, g1 = gts
    args = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W[0].data_ptr(), b1.data_ptr(), b2.data_ptr(),
            W[1].data_ptr(), W[2].data_ptr(), h0.data_ptr(), c0.data_ptr(), g0.data_ptr(), h1.data_ptr(),
            c1.data_ptr(), g1.data_ptr()]
    if ws is not None:
        args.append(ws.data_ptr())
    _lib.call(name, *args, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    return h0, c0, g0, h1, c1, g1


def _supported(B, H):
    from autovc_amd import _lib
    return bool(_lib.load().autovc_lstm2_persist_supported(B, H))


@pytest.fixture(params=["0", "1"], ids=["lag1", "lag2"])
def lag2(request, monkeypatch):
    """Both wavefront forms of the persistent stacked forward: layer 1 one step behind layer 0
    (AVC_LSTM2_LAG2=0, the bf16 default) and two steps behind (=1, the fp32 default: layer 1's
    input product runs while the workgroup waits at the grid barrier)."""
    monkeypatch.setenv("AVC_LSTM2_LAG2", request.param)
    return request.param


@pytest.mark.parametrize("T", [3, 128])
def test_persistent_matches_per_step_launches(cuda, T, lag2):
    from autovc_amd import _lib
    B, H = 64, 1024
    if not _supported(B, H):
        pytest.skip("persistent lstm2 needs one CU per workgroup on this device")
    gx, W, b1, b2 = _inputs(B, T, H, cuda)
    ref = _run("autovc_lstm2_fwd_f32", B, T, H, gx, W, b1, b2, cuda)
    ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=cuda)
    got = _run("autovc_lstm2_fwd_persist_f32", B, T, H, gx, W, b1, b2, cuda, ws)
    assert _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), _lib.stream_ptr(cuda)) == 0
    for name, a, r in zip(["h0", "c0", "gates0", "h1", "c1", "gates1"], got, ref):
        assert bool(torch.isfinite(a).all()), name
        err = (a.double() - r.double()).abs().max().item() / max(r.abs().max().item(), 1e-30)
        assert err < 2e-5, (name, err)
    # a second call into the same workspace (barrier words re-zeroed) is identical
    again = _run("autovc_lstm2_fwd_persist_f32", B, T, H, gx, W, b1, b2, cuda, ws)
    for a, b in zip(got, again):
        assert torch.equal(a, b)


def test_persistent_unsupported_shape_rejected(cuda):
    from autovc_amd import _lib
    assert not _supported(2, 1024) and not _supported(64, 512)
    gx, W, b1, b2 = _inputs(2, 4, 1024, cuda)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=cuda)
    with pytest.raises(ValueError):
        _run("autovc_lstm2_fwd_persist_f32", 2, 4, 1024, gx, W, b1, b2, cuda, ws)


@pytest.mark.parametrize("H,T", [(512, 3), (512, 128), (1024, 17)])
def test_single_layer_persistent_matches_per_step_launches(cuda, H, T):
    """autovc_lstm_fwd_persist_f32 (decoder lstm1's recurrence as one launch) against the
    per-step launches of autovc_lstm_fwd_f32, h written into a strided buffer."""
    from autovc_amd import _lib
    B = 64
    if not _lib.load().autovc_lstm_persist_supported(B, H):
        pytest.skip("persistent lstm needs one CU per workgroup on this device")
    g = torch.Generator().manual_seed(H + T)
    W = ((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(cuda)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(cuda)
    st = _lib.stream_ptr(cuda)

    def run(persist):
        hbuf = torch.full((B, T, H + 8), float("nan"), device=cuda)       # row stride T*(H+8)
        c = torch.full((B, T, H), float("nan"), device=cuda)
        gates = torch.full((B, T, 4 * H), float("nan"), device=cuda)
        if persist:
            ws = torch.empty(_lib.load().autovc_lstm_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=cuda)
            _lib.call("autovc_lstm_fwd_persist_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(),
                      hbuf.data_ptr(), T * (H + 8), H + 8, c.data_ptr(), gates.data_ptr(), ws.data_ptr(), st)
            assert _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), st) == 0
        else:
            _lib.call("autovc_lstm_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(),
                      hbuf.data_ptr(), T * (H + 8), H + 8, c.data_ptr(), gates.data_ptr(), 0, st)
        torch.cuda.synchronize()
        return hbuf, c, gates

    ref, got = run(False), run(True)
    assert bool(torch.isnan(got[0][:, :, H:]).all())                        # pad columns untouched
    for name, a, r in zip(["h", "c", "gates"], (got[0][:, :, :H], got[1], got[2]), (ref[0][:, :, :H], ref[1], ref[2])):
        assert bool(torch.isfinite(a).all()), name
        err = (a.double() - r.double()).abs().max().item() / max(r.abs().max().item(), 1e-30)
        assert err < 2e-5, (name, err)


@pytest.mark.parametrize("T", [3, 128])
def test_bf16_persistent_matches_bf16_per_step_launches(cuda, T, lag2):
    """autovc_lstm2_fwd_persist_bf16 against the per-step bf16 wavefront (autovc_lstm2_fwd_bf16):
    the same RNE-rounded weights and h copies, fp32 accumulation in a different order."""
    from autovc_amd import _lib
    B, H = 64, 1024
    if not _supported(B, H):
        pytest.skip("persistent lstm2 needs one CU per workgroup on this device")
    gx, W, b1, b2 = _inputs(B, T, H, cuda)
    Wb = [w.bfloat16().contiguous() for w in W]
    st = _lib.stream_ptr(cuda)

    def run(persist):
        outs = [torch.full((B, T, H), float("nan"), device=cuda) for _ in range(4)]
        gts = [torch.full((B, T, 4 * H), float("nan"), device=cuda) for _ in range(2)]
        h0, c0, h1, c1 = outs
        if persist:
            ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8,
                             device=cuda)
            _lib.call("autovc_lstm2_fwd_persist_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb[0].data_ptr(),
                      b1.data_ptr(), b2.data_ptr(), Wb[1].data_ptr(), Wb[2].data_ptr(), h0.data_ptr(), c0.data_ptr(),
                      gts[0].data_ptr(), h1.data_ptr(), c1.data_ptr(), gts[1].data_ptr(), ws.data_ptr(), st)
            assert _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), st) == 0
        else:
            hb = [torch.empty((B, T, H), device=cuda, dtype=torch.bfloat16) for _ in range(2)]
            _lib.call("autovc_lstm2_fwd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb[0].data_ptr(),
                      b1.data_ptr(), b2.data_ptr(), Wb[1].data_ptr(), Wb[2].data_ptr(), h0.data_ptr(),
                      hb[0].data_ptr(), c0.data_ptr(), gts[0].data_ptr(), h1.data_ptr(), hb[1].data_ptr(),
                      c1.data_ptr(), gts[1].data_ptr(), st)
        torch.cuda.synchronize()
        return [h0, c0, gts[0], h1, c1, gts[1]]

    ref, got = run(False), run(True)
    for name, a, r in zip(["h0", "c0", "gates0", "h1", "c1", "gates1"], got, ref):
        assert bool(torch.isfinite(a).all()), name
        d = (a.double() - r.double()).abs()
        # summation order moves a bf16 rounding of h now and then: bounded, and rare
        assert d.max().item() < 2e-2 * max(r.abs().max().item(), 1e-30), (name, d.max().item())
        assert d.mean().item() < 1e-4 * max(r.abs().max().item(), 1e-30), (name, d.mean().item())


@pytest.mark.parametrize("T", [3, 128])
@pytest.mark.parametrize("bf16", [False, True], ids=["fp32", "bf16"])
def test_row_split_persistent_bit_identical(cuda, T, bf16, lag2, monkeypatch):
    """The row-split stacked forward (lstm2_rs_kernel, AVC_LSTM2_RS=1: workgroup pairs split the
    64 batch rows, each owns 8 units) sums the same products in the same k order as
    lstm_persist_kernel, so every output is bit-identical, in both wavefront forms."""
    from autovc_amd import _lib
    B, H = 64, 1024
    if not _supported(B, H):
        pytest.skip("persistent lstm2 needs one CU per workgroup on this device")
    gx, W, b1, b2 = _inputs(B, T, H, cuda, seed=11)
    if bf16:
        W = [w.bfloat16().contiguous() for w in W]
    name = "autovc_lstm2_fwd_persist_bf16" if bf16 else "autovc_lstm2_fwd_persist_f32"
    ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=cuda)
    res = {}
    for rs in ("0", "1"):
        monkeypatch.setenv("AVC_LSTM2_RS", rs)
        res[rs] = _run(name, B, T, H, gx, W, b1, b2, cuda, ws)
        assert _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), _lib.stream_ptr(cuda)) == 0
    diff = {nm: (a - r).abs().max().item() for nm, a, r in zip(["h0", "c0", "gates0", "h1", "c1", "gates1"],
                                                                 res["1"], res["0"])}
    assert all(bool(torch.isfinite(a).all()) for a in res["1"])
    assert all(v == 0 for v in diff.values()), diff


def test_row_split_timeout_surfaces(cuda, monkeypatch):
    """A row-split launch whose grid barrier times out writes NaN over what it owns and sets the
    lstm2 forward's fault bit, like lstm_persist_kernel."""
    from autovc_amd import _lib, functional as AF
    B, T, H = 64, 8, 1024
    if not _supported(B, H):
        pytest.skip("persistent lstm2 needs one CU per workgroup on this device")
    AF.check_device_faults(cuda)
    monkeypatch.setenv("AVC_LSTM2_RS", "1")
    gx, W, b1, b2 = _inputs(B, T, H, cuda)
    ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=cuda)
    _lib.call("autovc_lstm_persist_set_timeout_ticks", 1)
    try:
        got = _run("autovc_lstm2_fwd_persist_f32", B, T, H, gx, W, b1, b2, cuda, ws)
    finally:
        _lib.call("autovc_lstm_persist_set_timeout_ticks", 0)
    assert not bool(torch.isfinite(got[3]).all())
    with pytest.raises(AF.DeviceFault, match="lstm_persist_kernel"):
        AF.check_device_faults(cuda)
    got = _run("autovc_lstm2_fwd_persist_f32", B, T, H, gx, W, b1, b2, cuda, ws)
    assert all(bool(torch.isfinite(a).all()) for a in got)
    AF.check_device_faults(cuda)


def test_barrier_timeout_surfaces_as_error(cuda):
    """A persistent launch whose grid barrier times out (forced with a 1-tick spin budget)
    must not let training continue on garbage: its h / c become NaN (so the losses do) and
    check_device_faults raises DeviceFault naming the kernel; the fault word is then clear
    and the next step with the normal budget is finite again."""
    import bench
    from autovc_amd import _lib, functional as AF
    B, H = 64, 1024
    if not _supported(B, H):
        pytest.skip("persistent lstm2 needs one CU per workgroup on this device")
    AF.check_device_faults(cuda)                 # nothing pending from earlier tests
    torch.manual_seed(0)
    solver = bench.make_solver(cuda, B)
    solver.G.train()
    x, e = bench.synthetic_batch(B, 32, cuda, 5)
    _lib.call("autovc_lstm_persist_set_timeout_ticks", 1)
    try:
        losses = solver.train_step(x, e)
        torch.cuda.synchronize()
    finally:
        _lib.call("autovc_lstm_persist_set_timeout_ticks", 0)
    assert not bool(torch.isfinite(losses[1]).item())          # loss_id went through the NaN h
    with pytest.raises(AF.DeviceFault, match="lstm_persist_kernel"):
        AF.check_device_faults(cuda)
    AF.check_device_faults(cuda)                 # cleared by the raising check
    torch.manual_seed(0)
    solver = bench.make_solver(cuda, B)
    solver.G.train()
    losses = solver.train_step(x, e)
    assert bool(torch.isfinite(torch.stack([v.reshape(()) for v in losses])).all())
    AF.check_device_faults(cuda)


def _xcd_supported():
    from autovc_amd import _lib
    return bool(_lib.load().autovc_lstm_xcd_supported(64, 512))


def _run1(name, B, T, H, gx, W, dev, ws=None):
    from autovc_amd import _lib
    h, c = (torch.full((B, T, H), float("nan"), device=dev) for _ in range(2))
    g = torch.full((B, T, 4 * H), float("nan"), device=dev)
    args = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(), T * H, H, c.data_ptr(), g.data_ptr()]
    if ws is not None:
        args.append(ws.data_ptr())
    else:
        args.append(0)   # autovc_lstm_fwd_f32's `reverse`
    _lib.call(name, *args, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    return h, c, g


@pytest.mark.parametrize("T", [1, 2, 128])
def test_xcd_local_lstm_matches_per_step_launches(cuda, T):
    """Decoder lstm1 forward as one XCD-local persistent launch (autovc_lstm_fwd_xcd_f32:
    batch rows split over the 8 XCDs, every hand-off inside one XCD's L2) against the
    per-step launches: h, c, gates within fp32 summation-order noise; a second call is
    bit-identical; no fault recorded."""
    from autovc_amd import _lib, functional as AF
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H = 64, 512
    AF.check_device_faults(cuda)
    gx, W, _, _ = _inputs(B, T, H, cuda, seed=9)
    ref = _run1("autovc_lstm_fwd_f32", B, T, H, gx, W[0], cuda)
    ws = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
    got = _run1("autovc_lstm_fwd_xcd_f32", B, T, H, gx, W[0], cuda, ws)
    AF.check_device_faults(cuda)
    for name, a, r in zip(["h", "c", "gates"], got, ref):
        assert bool(torch.isfinite(a).all()), name
        err = (a.double() - r.double()).abs().max().item() / max(r.abs().max().item(), 1e-30)
        assert err < 2e-5, (name, err)
    again = _run1("autovc_lstm_fwd_xcd_f32", B, T, H, gx, W[0], cuda, ws)
    for a, b in zip(got, again):
        assert torch.equal(a, b)


def test_xcd_local_lstm_timeout_surfaces(cuda):
    from autovc_amd import _lib, functional as AF
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H, T = 64, 512, 16
    AF.check_device_faults(cuda)
    gx, W, _, _ = _inputs(B, T, H, cuda, seed=9)
    ws = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
    _lib.call("autovc_lstm_persist_set_timeout_ticks", 1)
    try:
        h, _, _ = _run1("autovc_lstm_fwd_xcd_f32", B, T, H, gx, W[0], cuda, ws)
    finally:
        _lib.call("autovc_lstm_persist_set_timeout_ticks", 0)
    assert bool(torch.isnan(h[:, -1]).any())
    # the fault names this kernel and its own switch (not the lstm2 forward's)
    with pytest.raises(AF.DeviceFault, match="lstm_xcd_fwd_kernel.*AVC_LSTM_XCD=0") as ei:
        AF.check_device_faults(cuda)
    assert "AVC_LSTM2_PERSIST" not in str(ei.value)


@pytest.mark.parametrize("T", [3, 128])
def test_xcd_local_lstm_bf16_matches_bf16_per_step_launches(cuda, T):
    """autovc_lstm_fwd_xcd_bf16 against the per-step bf16 launches (autovc_lstm_fwd_bf16): the
    same RNE-rounded W_hh and h copies, fp32 accumulation in a different order."""
    from autovc_amd import _lib
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H = 64, 512
    gx, W, _, _ = _inputs(B, T, H, cuda, seed=13)
    Wb = W[0].bfloat16().contiguous()
    st = _lib.stream_ptr(cuda)
    outs = []
    for xcd in (False, True):
        h, c = (torch.full((B, T, H), float("nan"), device=cuda) for _ in range(2))
        g = torch.full((B, T, 4 * H), float("nan"), device=cuda)
        if xcd:
            ws = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
            _lib.call("autovc_lstm_fwd_xcd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(),
                      h.data_ptr(), T * H, H, c.data_ptr(), g.data_ptr(), ws.data_ptr(), st)
        else:
            hb = torch.empty((B, T, H), device=cuda, dtype=torch.bfloat16)
            _lib.call("autovc_lstm_fwd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(), h.data_ptr(),
                      hb.data_ptr(), c.data_ptr(), g.data_ptr(), 0, st)
        torch.cuda.synchronize()
        outs.append((h, c, g))
    for name, a, r in zip(["h", "c", "gates"], outs[1], outs[0]):
        assert bool(torch.isfinite(a).all()), name
        d = (a.double() - r.double()).abs()
        assert d.max().item() < 2e-2 * max(r.abs().max().item(), 1e-30), (name, d.max().item())
        assert d.mean().item() < 1e-4 * max(r.abs().max().item(), 1e-30), (name, d.mean().item())


def _bwd_inputs(B, T, H, dev, seed):
    gx, W, _, _ = _inputs(B, T, H, dev, seed=seed)
    _, c, g = _run1("autovc_lstm_fwd_f32", B, T, H, gx, W[0], dev)
    dh = (torch.randn(B, T, H, generator=torch.Generator().manual_seed(seed + 1)) * 0.1).to(dev)
    return W[0], c, g, dh


@pytest.mark.parametrize("T", [1, 2, 128])
def test_xcd_local_lstm_backward_matches_split_k_launches(cuda, T):
    """Decoder lstm1 backward as one XCD-local persistent launch (autovc_lstm_bwd_xcd_f32)
    against the per-step split-K launches (autovc_lstm_bwd_f32) on the same W_hh^T: dG within
    fp32 summation-order noise (relative to its max), a second call bit-identical, no fault."""
    from autovc_amd import _lib, functional as AF
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H = 64, 512
    AF.check_device_faults(cuda)
    W, c, g, dh = _bwd_inputs(B, T, H, cuda, 11)
    WT = W.t().contiguous()
    st = _lib.stream_ptr(cuda)
    ref = torch.full((B, T, 4 * H), float("nan"), device=cuda)
    ws = torch.empty(4 * _lib.load().autovc_lstm_bwd_workspace_floats(B, H, 8), dtype=torch.uint8, device=cuda)
    _lib.call("autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, g.data_ptr(), c.data_ptr(), WT.data_ptr(),
              ref.data_ptr(), 0, 8, ws.data_ptr(), st)
    wx = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
    outs = []
    for _ in range(2):
        got = torch.full((B, T, 4 * H), float("nan"), device=cuda)
        _lib.call("autovc_lstm_bwd_xcd_f32", B, T, H, dh.data_ptr(), T * H, H, g.data_ptr(), c.data_ptr(),
                  WT.data_ptr(), got.data_ptr(), wx.data_ptr(), st)
        torch.cuda.synchronize()
        outs.append(got)
    AF.check_device_faults(cuda)
    assert bool(torch.isfinite(outs[0]).all())
    err = (outs[0].double() - ref.double()).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("T", [3, 128])
def test_xcd_local_lstm_backward_bf16_matches_bf16_launches(cuda, T):
    """autovc_lstm_bwd_xcd_bf16 against the per-step bf16 backward (autovc_lstm_bwd_bf16):
    the same RNE bf16 W_hh^T and dG copies in the product, fp32 accumulation in another
    order; dG and its bf16 copy dGb both compared, dGb = RNE(dG) exactly."""
    from autovc_amd import _lib
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H = 64, 512
    W, c, g, dh = _bwd_inputs(B, T, H, cuda, 17)
    WTb = W.t().contiguous().bfloat16()
    st = _lib.stream_ptr(cuda)
    outs = []
    for xcd in (False, True):
        dG = torch.full((B, T, 4 * H), float("nan"), device=cuda)
        dGb = torch.full((B, T, 4 * H), float("nan"), device=cuda, dtype=torch.bfloat16)
        if xcd:
            ws = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
            _lib.call("autovc_lstm_bwd_xcd_bf16", B, T, H, dh.data_ptr(), T * H, H, g.data_ptr(), c.data_ptr(),
                      WTb.data_ptr(), dG.data_ptr(), dGb.data_ptr(), ws.data_ptr(), st)
        else:
            ws = torch.empty(4 * _lib.load().autovc_lstm_bwd_workspace_floats(B, H, 4), dtype=torch.uint8,
                             device=cuda)
            _lib.call("autovc_lstm_bwd_bf16", B, T, H, dh.data_ptr(), T * H, H, g.data_ptr(), c.data_ptr(),
                      WTb.data_ptr(), dG.data_ptr(), dGb.data_ptr(), 0, 4, ws.data_ptr(), st)
        torch.cuda.synchronize()
        outs.append((dG, dGb))
    (r, rb), (a, ab) = outs
    assert bool(torch.isfinite(a).all())
    assert torch.equal(ab, a.bfloat16())
    d = (a.double() - r.double()).abs()
    scale = r.abs().max().item()
    assert d.max().item() < 2e-2 * scale, d.max().item()
    assert d.mean().item() < 1e-4 * scale, d.mean().item()


def test_xcd_local_lstm_backward_timeout_surfaces(cuda):
    """A backward group that times out writes NaN over its dG and names its own kernel."""
    from autovc_amd import _lib, functional as AF
    if not _xcd_supported():
        pytest.skip("XCD-local LSTM needs 8 XCDs x 32 CUs")
    B, H, T = 64, 512, 16
    AF.check_device_faults(cuda)
    W, c, g, dh = _bwd_inputs(B, T, H, cuda, 11)
    WT = W.t().contiguous()
    dG = torch.zeros(B, T, 4 * H, device=cuda)
    wx = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=cuda)
    _lib.call("autovc_lstm_persist_set_timeout_ticks", 1)
    try:
        _lib.call("autovc_lstm_bwd_xcd_f32", B, T, H, dh.data_ptr(), T * H, H, g.data_ptr(), c.data_ptr(),
                  WT.data_ptr(), dG.data_ptr(), wx.data_ptr(), _lib.stream_ptr(cuda))
        torch.cuda.synchronize()
    finally:
        _lib.call("autovc_lstm_persist_set_timeout_ticks", 0)
    assert bool(torch.isnan(dG).any())
    with pytest.raises(AF.DeviceFault, match="lstm_xcd_bwd_kernel.*AVC_LSTM_XCD_BWD=0"):
        AF.check_device_faults(cuda)
