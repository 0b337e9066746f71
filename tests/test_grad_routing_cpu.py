"""Host logic of the weight-gradient routing (no GPU): which BLSTM / conv weight gradients go to
the gradient side stream, by precision and by encoder pass (functional.blstm_last_pass; the
Generator's full pass is differentiated last)."""
from autovc_amd import functional as AF


def test_blstm_last_pass_flag_nests_and_restores():
    assert AF._BLSTM_LAST_PASS[0] is False
    with AF.blstm_last_pass(True):
        assert AF._BLSTM_LAST_PASS[0] is True
        with AF.blstm_last_pass(False):
            assert AF._BLSTM_LAST_PASS[0] is False
        assert AF._BLSTM_LAST_PASS[0] is True
    assert AF._BLSTM_LAST_PASS[0] is False


def test_blstm_side_defaults_by_precision(monkeypatch):
    monkeypatch.setattr(AF, "_BLSTM_SIDE_ENV", None)
    for prec in ("fp32", "bf16"):   # mode 2: every pass but the last-differentiated one
        with AF.precision(prec):
            assert AF._blstm_side(last_pass=False) is True
            assert AF._blstm_side(last_pass=True) is False


def test_lstm1_backward_routing_defaults(monkeypatch):
    """The XCD-local lstm1 backward in both precisions (AVC_LSTM_XCD_BWD forces it)."""
    monkeypatch.setattr(AF, "_XCD_BWD_ENV", None)
    for prec in ("fp32", "bf16"):
        with AF.precision(prec):
            assert AF._xcd_bwd() is True
    monkeypatch.setattr(AF, "_XCD_BWD_ENV", "0")
    assert AF._xcd_bwd() is False


def test_blstm_side_overrides(monkeypatch):
    for mode, expect in (("0", (False, False)), ("1", (True, True)), ("2", (True, False))):
        monkeypatch.setattr(AF, "_BLSTM_SIDE_ENV", mode)
        for prec in ("fp32", "bf16"):
            with AF.precision(prec):
                assert (AF._blstm_side(False), AF._blstm_side(True)) == expect


def test_last_conv_main_defaults_and_override(monkeypatch):
    monkeypatch.setattr(AF, "_LAST_CONV_MAIN_ENV", None)
    with AF.precision("fp32"):
        assert AF._last_conv_main() is False
    with AF.precision("bf16"):
        assert AF._last_conv_main() is True
    monkeypatch.setattr(AF, "_LAST_CONV_MAIN_ENV", "0")
    with AF.precision("bf16"):
        assert AF._last_conv_main() is False


def test_generator_marks_only_the_full_pass(monkeypatch):
    """Generator.forward wraps the encoder of the full pass (c_trg given) in
    blstm_last_pass(True) and the code-only pass in blstm_last_pass(False)."""
    import torch
    from autovc_amd import model_vc_mel as MV

    seen = []

    class Probe(torch.nn.Module):
        dim_neck = 1

        def encode(self, x, c_org):
            seen.append(AF._BLSTM_LAST_PASS[0])
            return torch.zeros(x.shape[0], 2)

    g = MV.Generator.__new__(MV.Generator)
    torch.nn.Module.__init__(g)
    g.encoder = Probe()
    x = torch.zeros(1, 4, 80)
    g.forward(x, torch.zeros(1, 256), None)
    assert seen == [False]

    class Stop(Exception):
        pass

    def stop(*a):   # the full pass stops right after its encoder
        raise Stop()

    monkeypatch.setattr(AF.FrameConcatFn, "apply", staticmethod(stop))
    try:
        g.forward(x, torch.zeros(1, 256), torch.zeros(1, 256))
    except Stop:
        pass
    assert seen == [False, True]
    assert AF._BLSTM_LAST_PASS[0] is False


class _FakeStream:
    def __init__(self, log):
        self.log = log

    def wait_event(self, ev):
        self.log.append(("wait", ev))


def _out(flat, lo, hi, acc=True):
    import types
    return types.SimpleNamespace(acc=acc, buf=flat[lo:hi])


def test_main_stream_gradient_orders_after_side_writes_of_the_same_range(monkeypatch):
    """a parameter whose gradient one encoder pass accumulates on the side
    stream and the other on the main stream.  _main_grad joins the side queue behind a queued
    launch into an overlapping flat range, waits for the event of a released side batch that
    wrote one, and runs at once (no wait) for a disjoint range."""
    import torch
    flat = torch.zeros(64)
    log = []
    monkeypatch.setattr(AF, "_GRAD_STREAM_ON", True)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda dev=None: _FakeStream(log))
    monkeypatch.setattr(AF, "_GRAD_QUEUE", [])
    monkeypatch.setattr(AF, "_SIDE_WRITES", [])
    dev = torch.device("cpu")

    # (1) a launch into [8, 24) is still queued for the side stream: an overlapping main-stream
    # launch is queued behind it, not run
    AF._GRAD_QUEUE.append((dev, lambda: log.append("side"), (), "fp32", (_out(flat, 8, 24),)))
    AF._main_grad(dev, _out(flat, 16, 20), lambda: log.append("main1"))
    assert log == [] and len(AF._GRAD_QUEUE) == 2
    AF._GRAD_QUEUE.clear()

    # (2) a released side batch wrote [8, 24): the main stream waits for its event, then runs
    ev = object()
    AF._SIDE_WRITES.append((flat[8:24].data_ptr(), flat[24:].data_ptr(), ev))
    AF._main_grad(dev, (_out(flat, 0, 4), _out(flat, 20, 28)), lambda: log.append("main2"))
    assert log == [("wait", ev), "main2"]

    # (3) a disjoint range runs at once, with no wait
    log.clear()
    AF._main_grad(dev, _out(flat, 32, 40), lambda: log.append("main3"))
    assert log == ["main3"]

    # (4) destinations outside the flat buffer (acc False) never wait
    log.clear()
    AF._main_grad(dev, _out(flat, 8, 24, acc=False), lambda: log.append("main4"))
    assert log == ["main4"]

    # (5) the join orders the main stream after everything: the record is dropped
    monkeypatch.setattr(AF, "_GRAD_PENDING", set())
    AF.join_grad_stream(dev)
    assert AF._SIDE_WRITES == []
