"""Autograd ops of the Generator step, each forward/backward a sequence of C-ABI calls
into libautovc_hip.so (no torch compute on the hot path, no fallback).

Activations are frame-major / channel-last "NTC" (B, T, C) contiguous fp32 CUDA tensors:
the layout the reference's LSTMs and mel tensors already use (model_vc_mel.py:64,70,112,
116) — the reference's (B, C, T) conv layout is never materialised, the convolutions
read NTC through the GEMM's implicit im2col operand.
"""
from __future__ import annotations

import contextlib
import os

import torch

from . import _lib

ACT = {"none": 0, "relu": 1, "tanh": 2}
KS = 5      # ConvNorm kernel_size (model_vc_mel.py:53,96,137,147,157)
PAD = 2     # ConvNorm padding


# ---------------------------------------------------------------- helpers
def _s():
    return _lib.stream_ptr()


def _p(t):
    return 0 if t is None else t.data_ptr()


def _check(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: autovc_amd ops run on the GPU only (got a {t.device} tensor)")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")


class _Workspace:
    """Per-device scratch buffer reused by every op (one stream: ops never overlap).

    A slot that has to grow gets a new buffer, but the old one is never handed back to the
    caching allocator: a captured step graph (autovc_amd.graph) keeps using the raw pointer
    it was captured with, and replaying it into memory that now belongs to another tensor
    would corrupt that tensor.  Slots grow geometrically, so the retired buffers cost at
    most the size of the live one."""
    _bufs: dict = {}
    _retired: list = []

    @classmethod
    def get(cls, device, nbytes, slot="main"):
        key = (device, slot)
        buf = cls._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            size = max(int(nbytes), 1) + 256
            if buf is not None:
                cls._retired.append(buf)
                size = max(size, 2 * buf.numel())
            # zeroed: workspaces holding tile counters (the fused LSTM backward's) start at zero
            buf = torch.zeros(size, dtype=torch.uint8, device=device)
            cls._bufs[key] = buf
        return buf


def _ws(device, nbytes, slot="main"):
    # the gradient stream has scratch of its own (its GEMMs run beside the main stream's)
    if _GRAD_STREAM_ACTIVE[0]:
        slot = slot + "@grad"
    return _Workspace.get(device, nbytes, slot).data_ptr()


# ---------------------------------------------------------------- gradient stream
# Weight-gradient GEMMs (and the bias column sums next to them) are off the backward's
# critical path: nothing reads them before the optimizer.  When a gradient lives in the
# optimizer's flat buffer, its kernels go to a per-device side stream that first waits for
# everything the main stream has issued so far (so its inputs exist), marks those inputs
# as in use by the side stream (the caching allocator then keeps them until the side
# stream is past them), and runs beside the main stream — the LSTM and BLSTM recurrences
# there leave most of the chip idle.  Their fp32 GEMM workgroups carry LDS padding so that
# a recurrence step workgroup (37 KB LDS) still fits next to them on every CU
# (tools/lstm_concurrency.py: a conv-GEMM batch beside a 128-step chain costs 0.46 ms
# instead of 0.85 with the pad, 0.61 without).  FusedAdam.step (and join_grad_stream)
# make the main stream wait before the gradients are read.  AVC_GRAD_STREAM=0 disables.
_GRAD_STREAM_ON = os.environ.get("AVC_GRAD_STREAM", "1") != "0"
_GRAD_STREAM_ACTIVE = [False]
# (the side stream at high priority measured 32.9 vs 14.6 ms/step, DESIGN.md §9 2a: default priority)
_GRAD_STREAMS: dict = {}
# LDS left free per CU for the recurrence's step workgroup (37 KB) while side GEMMs run;
# measured per precision (bench.py, same box, alternating): fp32 21.1 ms/step with room
# kept vs 21.9 without (round 5 again: 14.06-14.08 vs 14.16-14.20); bf16 13.1 without vs 13.3
# with in round 2, but with round 5's 256-row side GEMMs and the BLSTM weight gradients beside
# the recurrences the room pays there too: 7.85-7.88 vs 7.91-7.93 (profiles/r05/ab_lds_reserve_r5.txt)
GRAD_LDS_RESERVE = {"fp32": 38912, "bf16": 38912}


def _grad_stream(dev):
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _GRAD_STREAMS.get(idx)
    if st is None:
        st = torch.cuda.Stream(torch.device("cuda", idx))
        _GRAD_STREAMS[idx] = st
    return st


_GRAD_QUEUE: list = []
_GRAD_PENDING: set = set()   # device indices whose side stream has work not yet joined


def _grad_launch(dev, outs, fn, *inputs):
    """Queue the gradient launches `fn` for the side stream when their destinations `outs`
    (a _GradOut or a tuple of them) accumulate into the flat buffer and the side stream is
    enabled; else run them now.  Queued work is released at the next recurrence
    (_flush_grad_queue) so that it runs beside a latency-bound chain rather than beside the
    main stream's own GEMMs (measured: released immediately it only competed with them:
    22.2 -> 22.9 ms/step)."""
    outs = outs if isinstance(outs, tuple) else (outs,)
    if not (all(o.acc for o in outs) and _GRAD_STREAM_ON):
        _main_grad(dev, outs, fn, *inputs)
        return
    # run later under the same precision; the destinations are final once the batch is done
    _GRAD_QUEUE.append((dev, fn, inputs, _PRECISION[0], outs))


# flat-buffer byte ranges [lo, hi) that a released side-stream batch accumulates into, each
# with the event recorded on the side stream right after that batch (cleared at the join)
_SIDE_WRITES: list = []


def _ranges(outs):
    return [(o.buf.data_ptr(), o.buf.data_ptr() + o.buf.numel() * o.buf.element_size()) for o in outs if o.acc]


def _main_grad(dev, outs, fn, *inputs):
    """Run the gradient launches `fn` on the main stream NOW, ordered after every side-stream
    write to the same flat-buffer ranges.  A parameter used twice in a step (the encoder runs
    twice per Generator step) has both passes' gradients accumulated into one .grad slice;
    when one pass's launches went to the side stream and the other's run on the main stream
    (blstm_last_pass / _last_conv_main routing), the two read-modify-writes must not overlap:
    if a launch into the range is still queued, this one joins the queue behind it (same
    stream, same order); if a released batch wrote it, the main stream waits for that batch's
    event first (in a step-graph capture: an edge from the side branch)."""
    outs = outs if isinstance(outs, tuple) else (outs,)
    mine = _ranges(outs)
    if mine and _GRAD_STREAM_ON:
        def hit(rs):
            return any(lo < h and l < hi for lo, hi in mine for l, h in rs)
        if any(hit(_ranges(item[4])) for item in _GRAD_QUEUE):
            _GRAD_QUEUE.append((dev, fn, inputs, _PRECISION[0], outs))
            return
        main = torch.cuda.current_stream(dev)
        waited = set()
        for lo, hi, ev in _SIDE_WRITES:
            if id(ev) not in waited and hit([(lo, hi)]):
                main.wait_event(ev)
                waited.add(id(ev))
    fn()


def _grad_mark(dev):
    """Event on the main stream marking that every queued gradient launch's inputs exist;
    taken just before a recurrence is enqueued, and handed to _flush_grad_queue after it,
    so that the host launches the chain first (the side launches are Python-paced: issued
    first they left the main stream idle for up to 1.3 ms) while the side stream still only
    waits for the work before the chain."""
    if not _GRAD_QUEUE:
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return ev


def _flush_grad_queue(beside_recurrence=True, after=None, lds_reserve=None):
    """Issue every queued gradient launch on the side stream, ordered after `after` (an
    event from _grad_mark) or else after all main-stream work issued so far (their
    inputs), inputs marked as in use by the side stream.  The LDS reserve only pays beside
    a recurrence; the final flush (join) runs unpadded."""
    if not _GRAD_QUEUE:
        if MARKS.active and beside_recurrence:
            MARKS.mark(torch.device("cuda", torch.cuda.current_device()), None, [])
        return
    items = list(_GRAD_QUEUE)
    _GRAD_QUEUE.clear()
    dev = items[0][0]
    main = torch.cuda.current_stream(dev)
    side = _grad_stream(dev)
    if after is not None:
        side.wait_event(after)
    else:
        side.wait_stream(main)
    _GRAD_STREAM_ACTIVE[0] = True
    _GRAD_PENDING.add(side.device.index)
    prev_prec = _PRECISION[0]
    if lds_reserve is None:
        lds_reserve = GRAD_LDS_RESERVE[items[0][3]] if beside_recurrence else 0
    _lib.call("autovc_gemm_set_lds_reserve", lds_reserve)
    try:
        with torch.cuda.stream(side):
            for _, fn, inputs, prec, _outs in items:
                for t in inputs:
                    if t is not None:
                        t.record_stream(side)
                _PRECISION[0] = prec
                fn()
    finally:
        _PRECISION[0] = prev_prec
        _lib.call("autovc_gemm_set_lds_reserve", 0)
        _GRAD_STREAM_ACTIVE[0] = False
    written = [r for item in items for r in _ranges(item[4])]
    if written:
        ev = torch.cuda.Event()
        ev.record(side)
        _SIDE_WRITES.extend((lo, hi, ev) for lo, hi in written)
    if MARKS.active:
        MARKS.mark(dev, side, [o for item in items for o in item[4]])


def join_grad_stream(dev=None):
    """Release queued gradient work and make the current stream wait for the gradient
    stream (before anything reads the gradients).  (Running the batch still queued here on the
    idle main stream instead measured fp32 13.93-13.98 vs 13.94, bf16 7.87-7.92 vs 7.81-7.85
    ms/step: profiles/r06/ab_join_{fp32,bf16}.txt.)"""
    _flush_grad_queue(beside_recurrence=False)
    _SIDE_WRITES.clear()
    if not _GRAD_PENDING:
        return
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _GRAD_STREAMS.get(idx)
    if st is not None and idx in _GRAD_PENDING:
        # only a side stream with work since the last join is waited on: inside a graph
        # capture (autovc_amd.graph) the wait must be on work of the same capture
        torch.cuda.current_stream(dev).wait_stream(st)
        _GRAD_PENDING.discard(idx)


class GradMarks:
    """Gradient-ready marks of the backward, for the data-parallel exchange (autovc_amd.ddp)
    to overlap with the rest of the backward (not in the reference, which is single-device).

    While `active`, every backward recurrence (where the queued weight gradients are released
    to the side stream) and the final join record a mark: an event on the main stream and,
    when the side stream has work, one on the side stream, both through
    autovc_event_record_any — inside a step-graph capture these become event-record nodes that
    every replay re-records.  Every flat-buffer gradient destination (_GradOut with acc) is
    logged with the first mark after which it is final: a main-stream write at the next mark,
    a side-stream batch at the mark taken right after it is issued.  ddp.reduce_and_step then
    starts each bucket's collective as soon as the events of its latest write's mark fire."""

    def __init__(self):
        self.active = False
        self.events = []          # mark k (1-based) -> (main event handle, side event handle)
        self.n = 0                # marks recorded in the current backward
        self.ready = {}           # flat-buffer byte range (ptr, nbytes) -> mark index
        self.side_at = {}         # mark index -> whether its side event was recorded

    def begin(self):
        self.n = 0
        self.ready = {}
        self.side_at = {}

    def _event(self, k, which):
        import ctypes
        while len(self.events) < k:
            pair = []
            for _ in range(2):
                h = ctypes.c_void_p()
                _lib.call("autovc_event_create", ctypes.byref(h))
                pair.append(h.value)
            self.events.append(tuple(pair))
        return self.events[k - 1][which]

    # a flat-buffer gradient that autograd accumulates after the op returns (not through
    # _GradOut's in-place path): final only at the last mark
    FINAL = 1 << 30

    def log(self, buf, k):
        key = (buf.data_ptr(), buf.numel() * buf.element_size())
        self.ready[key] = max(self.ready.get(key, 0), k)

    def snapshot(self):
        """The mark structure of the backward just recorded (a captured step graph keeps it:
        graph.StepGraphs restores it before each of that graph's replays)."""
        return self.n, dict(self.ready), dict(self.side_at)

    def restore(self, snap):
        self.n, ready, side_at = snap
        self.ready, self.side_at = dict(ready), dict(side_at)

    def mark(self, dev, side, outs):
        self.n += 1
        k = self.n
        _lib.call("autovc_event_record_any", self._event(k, 0), torch.cuda.current_stream(dev).cuda_stream)
        self.side_at[k] = side is not None
        if side is not None:
            _lib.call("autovc_event_record_any", self._event(k, 1), side.cuda_stream)
        for o in outs:
            self.log(o.buf, k)

    def final(self, dev):
        """The join at the end of the backward: everything is final at this mark."""
        self.n += 1
        _lib.call("autovc_event_record_any", self._event(self.n, 0), torch.cuda.current_stream(dev).cuda_stream)
        self.side_at[self.n] = False
        return self.n

    def ready_mark(self, ptr, nbytes):
        """Mark index after which the flat-buffer bytes [ptr, ptr + nbytes) are final (the
        last mark when nothing wrote them)."""
        r = 0
        for (p, n), k in self.ready.items():
            if p < ptr + nbytes and ptr < p + n:
                r = max(r, k)
        return min(r, self.n) if r else self.n

    def wait(self, stream_ptr, k):
        """Make `stream_ptr` wait for mark k's events."""
        _lib.call("autovc_stream_wait_event", stream_ptr, self._event(k, 0))
        if self.side_at.get(k):
            _lib.call("autovc_stream_wait_event", stream_ptr, self._event(k, 1))


MARKS = GradMarks()


_PRECISION = ["fp32"]


@contextlib.contextmanager
def precision(mode):
    """Matmul precision inside the block: "fp32" (BASELINE config 2, exact fp32 MFMA) or
    "bf16" (config 3: bf16-rounded operands, fp32 accumulation and fp32 everything else —
    master weights, optimizer, BatchNorm, losses, recurrent cell math).  Wrap forward AND
    backward (autograd runs the backward kernels after the forward block has exited)."""
    if mode not in ("fp32", "bf16"):
        raise ValueError(f"precision must be 'fp32' or 'bf16', got {mode!r}")
    prev = _PRECISION[0]
    _PRECISION[0] = mode
    try:
        yield
    finally:
        _PRECISION[0] = prev


def current_precision():
    return _PRECISION[0]


def gemm(M, N, K, A, lda, a_trans, B, ldb, b_trans, C, ldc, *, a_conv=None, b_conv=None,
         bias1=None, bias2=None, accumulate=False, splits=1, a_off=0, b_off=0, c_off=0, a_bf16=None,
         b_bf16=None):
    """C[M,N] (+)= A(m,k) B(k,n) (+bias); offsets are in floats from the tensors' data.
    bf16 MFMA under precision("bf16"), exact fp32 MFMA otherwise.  a_bf16 / b_bf16: bf16
    tensors laid out like A / B holding RNE(A) / RNE(B) (a producer's own copy, a per-step
    weight copy); under bf16 the GEMM reads them instead (autovc_gemm_bf16src_f32, half of
    those operands' bytes, the same result)."""
    ac = a_conv or (0, 0, 0)
    bc = b_conv or (0, 0, 0)
    ws = 0
    if _PRECISION[0] == "bf16":   # the library plans large GEMMs' split-K itself
        splits = _lib.load().autovc_gemm_bf16_splits(M, N, K, splits)
    else:
        splits = _lib.load().autovc_gemm_f32_splits(M, N, K, splits)
    if splits > 1:
        ws = _ws(C.device, 4 * _lib.load().autovc_gemm_workspace_floats(M, N, splits), "gemm")
    src = 0
    if _PRECISION[0] == "bf16" and _BF16_SRC:
        src = (1 if a_bf16 is not None and a_conv is None else 0) | (2 if b_bf16 is not None and b_conv is None else 0)
    if src:
        pa = a_bf16.data_ptr() + 2 * a_off if src & 1 else A.data_ptr() + 4 * a_off
        pb = b_bf16.data_ptr() + 2 * b_off if src & 2 else B.data_ptr() + 4 * b_off
        _lib.call("autovc_gemm_bf16src_f32", M, N, K, pa, lda, a_trans, pb, ldb, b_trans, bc[0], bc[1], bc[2],
                  C.data_ptr() + 4 * c_off, ldc, _p(bias1), _p(bias2), int(accumulate), splits, ws, src, _s())
        return
    fn = "autovc_gemm_bf16_f32" if _PRECISION[0] == "bf16" else "autovc_gemm_f32"
    _lib.call(fn, M, N, K,
              A.data_ptr() + 4 * a_off, lda, a_trans, ac[0], ac[1], ac[2],
              B.data_ptr() + 4 * b_off, ldb, b_trans, bc[0], bc[1], bc[2],
              C.data_ptr() + 4 * c_off, ldc, _p(bias1), _p(bias2), int(accumulate), splits, ws, _s())


# the LSTM weight / input gradients read the backward's bf16 dG copy, and the LSTM input
# projections / input gradients the step's bf16 W_ih copy (AVC_BF16_SRC=0: the fp32 tensors;
# the W_ih copies alone measured within noise, profiles/r05/ab_bf16_wsrc.txt, and are kept)
_BF16_SRC = os.environ.get("AVC_BF16_SRC", "1") != "0"


def _wbf16(W):
    """The step's cached bf16 copy of a 2-D LSTM weight under bf16 (None otherwise)."""
    if (_PRECISION[0] != "bf16" or not _BF16_SRC or not _cacheable(W) or W.dim() != 2
            or W.shape[1] % 8):
        return None
    return conv_weight(W, 6)
_DW_MIN_BLOCKS = 1024   # (2048 / 4096: no faster, profiles/r02/ab_dw_min_blocks.txt)


def _splits_for(M, N, K):
    """Split-K factor for the long-K weight-gradient GEMMs (fp32; capping it at 2 or 1 measured
    slower, 14.48-14.50 / 14.70-14.79 vs 14.39-14.42 ms/step, profiles/r05/ab_bf16_dw_splits.txt;
    the bf16 plan caps its own at 2): >= 1024 blocks of 64x64 output
    tiles (4 per CU) while each split keeps >= 1024 k (tools/gemm_bench.hip sweep: conv dW
    512x2560x8192 42.7 TF unsplit -> 81.6 TF at 4 splits).  Tiny outputs (the BLSTM weight
    gradients, 128 x 32..512 over K = B*T = 8192: 2-16 tiles) split deep instead — up to 64
    ways with >= 256 k each — so the serial k loop stops dominating (42 us -> a few us)."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    s = 1
    while tiles * s < _DW_MIN_BLOCKS and K // (s + 1) >= 1024 and s < 8:
        s += 1
    if tiles < 64:
        s = max(s, min(64, K // 256, max(1, 1024 // tiles)))
    return s


def colsum(X2d, out, out2=None, accumulate=False):
    M, N = X2d.shape
    ws = _ws(X2d.device, 4 * _lib.load().autovc_colsum_workspace_floats(N), "colsum")
    _lib.call("autovc_colsum_f32", M, N, X2d.data_ptr(), X2d.stride(0), _p(out), _p(out2),
              int(accumulate), ws, _s())


class _GradOut:
    """Destination of one parameter gradient.  Parameters managed by FusedAdam carry
    `_avc_flat` and a .grad view into the optimizer's flat gradient buffer: backward then
    accumulates straight into it (kernel-side accumulate) and hands autograd None, instead
    of returning a fresh tensor that AccumulateGrad adds in a separate pass."""

    def __init__(self, param, shape, device):
        g = param.grad if (param is not None and getattr(param, "_avc_flat", False)) else None
        self.acc = g is not None and tuple(g.shape) == tuple(shape) and g.is_contiguous()
        self.buf = g if self.acc else torch.empty(shape, device=device, dtype=torch.float32)
        if self.acc and MARKS.active:
            MARKS.log(self.buf, MARKS.n + 1)      # a main-stream write: final at the next mark
        elif g is not None and MARKS.active:
            # returned to autograd (padded / mixed destinations), which adds it into the flat
            # .grad later, in no mark's view: the bucket holding it waits for the last mark
            MARKS.log(g, GradMarks.FINAL)

    def result(self):
        return None if self.acc else self.buf


def _bias_outs(p_ih, p_hh, shape, dev):
    """Destinations of an LSTM layer's two bias gradients (one column-sum launch writes both):
    both in place when both live in the flat buffer, else two fresh tensors handed to autograd
    (whose later accumulation the gradient-ready marks then see only at the last mark)."""
    gi, gh = _GradOut(p_ih, shape, dev), _GradOut(p_hh, shape, dev)
    if gi.acc == gh.acc:
        return gi, gh
    if MARKS.active:
        for o in (gi, gh):
            if o.acc:
                MARKS.log(o.buf, GradMarks.FINAL)
    return _GradOut(None, shape, dev), _GradOut(None, shape, dev)


# ---------------------------------------------------------------- Conv1d + BN + act
def _ceil4(n):
    return (n + 3) // 4 * 4


def _pad_last(x, n):
    if x.shape[-1] == n:
        return x.contiguous()
    return torch.nn.functional.pad(x, (0, n - x.shape[-1])).contiguous()


def _padded_weight(W, Cop, Cip):
    """(Co, Ci, K) -> zero-padded (Cop, Cip, K) (only for channel counts % 4 != 0, e.g.
    the 513/769-channel STFT generator)."""
    Co, Ci, K = W.shape
    if (Co, Ci) == (Cop, Cip):
        return W.contiguous()
    Wp = W.new_zeros((Cop, Cip, K))
    Wp[:Co, :Ci] = W
    return Wp


_WINOGRAD = os.environ.get("AVC_WINOGRAD", "1") != "0"
_WINO_KEEP_XT = True   # (False transforms x again: tests/test_generator_gpu.py; r02 ab_wino_keep_xt.txt)

# ---------------------------------------------------------------- step-scoped weight transforms
# Inside weight_scope() (the Solver's forward + backward: no parameter changes until the
# optimizer step) every conv weight transform — Winograd W~ forward (kind 0) / flipped
# (kind 1), im2col packs Wf (kind 2) / Wd (kind 3) — is computed at most once and kept
# until the scope ends; prepare_conv_weights() computes all of a model's in ONE launch
# (autovc_conv_weights_batched_f32) instead of one launch per layer and pass (the encoder
# runs twice per step, solver_encoder.py:226-236).  Outside a scope nothing is cached.
_WSCOPE = [None]
_WBATCH = True   # (False: per-layer transforms, bit-identical; tests/test_solver_gpu.py)
_WSHAPE = {0: lambda Co, Ci: (8, Co, Ci), 1: lambda Co, Ci: (8, Ci, Co),
           2: lambda Co, Ci: (Co, KS * Ci), 3: lambda Co, Ci: (KS * Co, Ci),
           4: lambda Co, Ci: (Co, KS * Ci), 5: lambda Co, Ci: (KS * Co, Ci),   # 4 / 5: bf16 packs
           # 2-D (LSTM) weights (R, C): 6 = bf16 copy, 7 = fp32 transpose, 8 = bf16 transpose
           6: lambda R, C: (R, C), 7: lambda R, C: (C, R), 8: lambda R, C: (C, R)}


def _wdtype(kind):
    return torch.float32 if kind in (0, 1, 2, 3, 7) else torch.bfloat16


@contextlib.contextmanager
def weight_scope():
    prev = _WSCOPE[0]
    if prev is None and _WBATCH:
        _WSCOPE[0] = {}
    try:
        yield
    finally:
        _WSCOPE[0] = prev


def _cacheable(W):
    # parameters only (a leaf that requires grad): a padded copy is a fresh tensor per call
    return _WSCOPE[0] is not None and W.is_leaf and W.requires_grad and W.is_contiguous()


def _run_weight_jobs(jobs):
    import ctypes
    n = len(jobs)
    kinds = (ctypes.c_int * n)(*[k for k, _, _ in jobs])
    cos = (ctypes.c_int * n)(*[W.shape[0] for _, W, _ in jobs])
    cis = (ctypes.c_int * n)(*[W.shape[1] for _, W, _ in jobs])
    ws = (ctypes.c_void_p * n)(*[W.data_ptr() for _, W, _ in jobs])
    outs = (ctypes.c_void_p * n)(*[o.data_ptr() for _, _, o in jobs])
    _lib.call("autovc_conv_weights_batched_f32", n, ctypes.addressof(kinds), ctypes.addressof(cos),
              ctypes.addressof(cis), ctypes.addressof(ws), ctypes.addressof(outs), _s())


def conv_weight(W, kind):
    """The kind-`kind` transform of conv weight W (Co, Ci, 5) (see above), from the scope's
    cache when there is one."""
    Co, Ci = W.shape[0], W.shape[1]
    key = (kind, W.data_ptr(), Co, Ci)
    cache = _WSCOPE[0] if _cacheable(W) else None
    if cache is not None and key in cache:
        return cache[key]
    out = torch.empty(_WSHAPE[kind](Co, Ci), device=W.device, dtype=_wdtype(kind))
    if kind <= 1:
        _lib.call("autovc_wino5_weights_f32", Co, Ci, W.data_ptr(), kind, out.data_ptr(), _s())
    elif kind <= 3:
        _lib.call("autovc_conv_pack_f32", Co, Ci, KS, W.data_ptr(), _p(out if kind == 2 else None),
                  _p(out if kind == 3 else None), _s())
    else:
        _run_weight_jobs([(kind, W.contiguous(), out)])
    if cache is not None:
        cache[key] = out
    return out


def _cat_scoped(a, b):
    """torch.cat((a, b)) of two parameters, once per weight scope (the encoder runs twice)."""
    cache = _WSCOPE[0] if (_cacheable(a) and _cacheable(b)) else None
    key = ("cat", a.data_ptr(), b.data_ptr(), tuple(a.shape), tuple(b.shape))
    if cache is not None and key in cache:
        return cache[key]
    out = torch.cat((a.detach(), b.detach()), 0)
    if cache is not None:
        cache[key] = out
    return out


def prepare_weights(convs, lstms, T, training, B=None):
    """Inside a weight_scope: compute, in one launch, every transform the ConvNorm layers
    `convs` (nn.Conv1d, k=5) will use for sequences of T frames — the Winograd pair for
    fp32 Winograd shapes, else the im2col packs — and the large-H LSTMs `lstms` (model_vc_mel
    LSTM modules) their recurrences use — bf16 copies of the recurrent weights under bf16,
    the transposes the backward reads (B: the batch, which decides whether the persistent
    lstm2 backward, reading the untransposed weights, runs) — and cache them for the scope."""
    cache = _WSCOPE[0]
    if cache is None:
        return
    jobs = []

    def add(kind, W):
        key = (kind, W.data_ptr(), W.shape[0], W.shape[1])
        if key not in cache:
            out = torch.empty(_WSHAPE[kind](W.shape[0], W.shape[1]), device=W.device, dtype=_wdtype(kind))
            cache[key] = out
            jobs.append((kind, W, out))

    for m in lstms:
        H = m.hidden_size
        if m.bidirectional or m.num_layers not in (1, 2) or H < 256:
            continue
        mats = [m.weight_hh_l0] if m.num_layers == 1 else [m.weight_hh_l0, m.weight_ih_l1, m.weight_hh_l1]
        kinds = ((6, 8) if training else (6,)) if _bf16_rec(H) else ((7,) if training else ())
        for W in mats:
            if _cacheable(W):
                for kind in kinds:
                    add(kind, W)
        W = m.weight_ih_l0   # the input projection's (and input gradient's) bf16 operand (_wbf16)
        if _bf16_rec(H) and _BF16_SRC and _cacheable(W) and W.shape[1] % 8 == 0:
            add(6, W)
    for conv in convs:
        W = conv.weight
        if not _cacheable(W) or W.shape[2] != KS:
            continue
        Co, Ci = W.shape[0], W.shape[1]
        if _wino_ok(T, Ci, Co):
            kinds = (0, 1)
        elif _PRECISION[0] == "bf16" and _CHAIN_BF16_MODE == 2 and Co % 8 == 0 and Ci % 8 == 0:
            kinds = (4, 5)
        elif Co % 4 == 0 and Ci % 4 == 0:
            kinds = (2, 3)
        else:
            kinds = ()
        for kind in kinds[:2 if training else 1]:
            add(kind, W)
    if jobs:
        _run_weight_jobs(jobs)


def prepare_conv_weights(convs, T, training):
    prepare_weights(convs, [], T, training)


def _wino_conv(x, Wp, bias, T, flip, keep_xt=False):
    """Winograd F(4,5) conv (csrc/winograd.hip): flip=0 -> conv(x, W) + bias (B,T,Cop);
    flip=1 -> the input-gradient correlation of x = dy (B,T,Cop) with W: (B,T,Cip).
    keep_xt: also return the input transform X~ (8, B*T/4, Cin), which the weight gradient
    of the same conv reuses instead of transforming x again."""
    B, _, Cin = x.shape
    Cop, Cip, _ = Wp.shape
    Cout = Cip if flip else Cop
    nt = B * T // 4
    dev = x.device
    Wt = conv_weight(Wp, int(flip))
    Xt = torch.empty((8, nt, Cin), device=dev, dtype=torch.float32)
    Yt = torch.empty((8, nt, Cout), device=dev, dtype=torch.float32)
    _lib.call("autovc_wino5_input_f32", B, T, Cin, x.data_ptr(), x.stride(1), Xt.data_ptr(), _s())
    _lib.call("autovc_gemm_batched_f32", 8, nt, Cout, Cin, Xt.data_ptr(), Cin, nt * Cin, 0, Wt.data_ptr(), Cin,
              Cout * Cin, 0, Yt.data_ptr(), Cout, nt * Cout, 0, _s())
    y = torch.empty((B, T, Cout), device=dev, dtype=torch.float32)
    _lib.call("autovc_wino5_output_f32", B, T, Cout, Yt.data_ptr(), _p(bias), y.data_ptr(), Cout, _s())
    return (y, Xt) if keep_xt else y


def _wino_wgrad(x, dy, T, dW, acc, Xt=None):
    """dW (Co,Ci,5) (+)= Winograd F(4,5) weight gradient of conv(x) against dy (B,T,Co):
    dY~ and X~ transforms, 8 GEMMs over the B*T/4 tiles (M_i = dY~_i^T X~_i), G^T combine.
    Xt: X~ kept from the forward (the same transform of the same x), else computed here."""
    B, _, Cin = x.shape
    Cout = dy.shape[2]
    nt = B * T // 4
    dev = x.device
    Dt = torch.empty((8, nt, Cout), device=dev, dtype=torch.float32)
    Mt = torch.empty((8, Cout, Cin), device=dev, dtype=torch.float32)
    if Xt is None:
        Xt = torch.empty((8, nt, Cin), device=dev, dtype=torch.float32)
        _lib.call("autovc_wino5_input_f32", B, T, Cin, x.data_ptr(), x.stride(1), Xt.data_ptr(), _s())
    _lib.call("autovc_wino5_dy_f32", B, T, Cout, dy.data_ptr(), dy.stride(1), Dt.data_ptr(), _s())
    _lib.call("autovc_gemm_batched_f32", 8, Cout, Cin, nt, Dt.data_ptr(), Cout, nt * Cout, 1, Xt.data_ptr(), Cin,
              nt * Cin, 1, Mt.data_ptr(), Cin, Cout * Cin, 0, _s())
    _lib.call("autovc_wino5_wgrad_f32", Cout, Cin, Mt.data_ptr(), dW.data_ptr(), int(acc), _s())


def _wino_ok(T, *channels):
    # fp32 only: rounding the TRANSFORMED operands to bf16 (coefficients up to 5.25 and 8)
    # measured 1.6e-2 relative error vs 2e-5 for bf16 operands of the plain conv, so under
    # precision("bf16") the conv stays the bf16 im2col GEMM (exact-operand semantics).
    return _WINOGRAD and _PRECISION[0] == "fp32" and T % 4 == 0 and all(c % 4 == 0 for c in channels)


def _conv_fwd(x, Wp, bp, T, keep_xt=False):
    """y (B,T,Cop) = conv1d_k5p2(x (B,T,Cip)) + b: Winograd F(4,5) (8 batched GEMMs) when T
    is a multiple of 4, else one implicit-im2col GEMM.  keep_xt: return (y, X~ or None)."""
    B, _, Cip = x.shape
    Cop = Wp.shape[0]
    if _wino_ok(T, Cip, Cop) and x.is_contiguous():
        return _wino_conv(x, Wp, bp, T, 0, keep_xt)
    Wf = conv_weight(Wp, 2)
    y = torch.empty((B, T, Cop), device=x.device, dtype=torch.float32)
    gemm(B * T, Cop, KS * Cip, x, Cip, 0, Wf, KS * Cip, 0, y, Cop, a_conv=(T, Cip, -PAD), bias1=bp)
    return (y, None) if keep_xt else y


def _conv_bwd(dy, x, Wp, need_x, need_w, need_b, W=None, b=None, Xt=None):
    """Backward of _conv_fwd given dy (B,T,Cop): (dx (B,T,Cip), dW, db).  W / b are the
    parameters: when their gradients live in a flat buffer (and no channel padding is in
    play) dW / db are accumulated there and returned as None.  Xt: the forward's Winograd
    input transform of x (_conv_fwd keep_xt), reused by the weight gradient."""
    B, T, Cip = x.shape
    Cop = Wp.shape[0]
    M = B * T
    dev = x.device
    dx = dW = db = None
    padded = W is None or tuple(W.shape) != tuple(Wp.shape)
    if need_b:
        go = _GradOut(None if padded else b, (Cop,), dev)
        _grad_launch(dev, go, lambda go=go: colsum(dy.view(M, Cop), go.buf, accumulate=go.acc), dy)
        db = go.result()
    if need_w:
        go = _GradOut(None if padded else W, (Cop, Cip, KS), dev)

        def dw(go=go):
            if _wino_ok(T, Cip, Cop) and dy.is_contiguous() and x.is_contiguous():
                _wino_wgrad(x, dy, T, go.buf, go.acc, Xt)
                return
            dWf = torch.empty((Cop, KS * Cip), device=dev, dtype=torch.float32)
            gemm(Cop, KS * Cip, M, dy, Cop, 1, x, Cip, 1, dWf, KS * Cip, b_conv=(T, Cip, -PAD),
                 splits=_splits_for(Cop, KS * Cip, M))
            _lib.call("autovc_conv_unpack_grad_f32", Cop, Cip, KS, dWf.data_ptr(), go.buf.data_ptr(), int(go.acc),
                      _s())
        _grad_launch(dev, go, dw, dy, x, *(() if Xt is None else (Xt,)))
        dW = go.result()
    if need_x:
        if _wino_ok(T, Cip, Cop) and dy.is_contiguous():
            dx = _wino_conv(dy, Wp, None, T, 1)
        else:
            Wd = conv_weight(Wp, 3)
            dx = torch.empty((B, T, Cip), device=dev, dtype=torch.float32)
            gemm(M, Cip, KS * Cop, dy, Cop, 0, Wd, Cip, 1, dx, Cip, a_conv=(T, Cop, -PAD))
    return dx, dW, db


class ConvBNActFn(torch.autograd.Function):
    """ConvNorm (k=5, p=2) -> BatchNorm1d -> act [-> + residual], NTC in/out.

    Forward: conv as one implicit-im2col MFMA GEMM (bias fused), BN statistics (train)
    or running stats (eval), fused normalise + activation (+ residual) pass.
    """

    @staticmethod
    def forward(ctx, x, W, b, gamma, beta, running_mean, running_var, nbt, training, act,
                momentum, eps, residual):
        _check(x, "conv_bn_act")
        B, T, Ci = x.shape
        Co = W.shape[0]
        Cip, Cop = _ceil4(Ci), _ceil4(Co)
        M = B * T
        dev = x.device
        xp = _pad_last(x, Cip)
        Wp = _padded_weight(W, Cop, Cip)
        bp = b if (b is None or Cop == Co) else _pad_last(b, Cop)
        # the weight gradient reuses the forward's Winograd input transform (_WINO_KEEP_XT False:
        # recompute it in backward)
        keep = bool(training and _WINO_KEEP_XT and ctx.needs_input_grad[1])
        y, ctx.xt = _conv_fwd(xp, Wp, bp, T, keep_xt=True) if keep else (_conv_fwd(xp, Wp, bp, T), None)
        if training:
            mean = torch.empty(Co, device=dev, dtype=torch.float32)
            var = torch.empty(Co, device=dev, dtype=torch.float32)
            ws = _ws(dev, _lib.load().autovc_bn_workspace_bytes(Co), "bn")
            _lib.call("autovc_bn_stats_f32", M, Co, y.data_ptr(), Cop, mean.data_ptr(), var.data_ptr(),
                      _p(running_mean), _p(running_var), float(momentum), _p(nbt), ws, _s())
        else:
            mean, var = running_mean, running_var
        z = torch.empty((B, T, Co), device=dev, dtype=torch.float32)
        res = residual.contiguous() if residual is not None else None
        _lib.call("autovc_bn_act_fwd_f32", M, Co, y.data_ptr(), Cop, mean.data_ptr(), var.data_ptr(),
                  _p(gamma), _p(beta), float(eps), ACT[act], _p(res), Co, z.data_ptr(), Co, _s())
        ctx.training = training
        ctx.act, ctx.eps = act, eps
        ctx.has_res = residual is not None
        ctx.dims = (Ci, Co, Cip, Cop)
        ctx.params = (W, b, gamma, beta)
        # the activation backward reads the forward output; the residual layer has act none
        ctx.save_for_backward(xp, Wp, gamma, y, None if ctx.has_res else z, mean, var)
        return z

    @staticmethod
    def backward(ctx, dz):
        xp, Wp, gamma, y, z, mean, var = ctx.saved_tensors
        if not ctx.training:
            raise NotImplementedError("autovc_amd: backward through eval-mode BatchNorm is not supported")
        Ci, Co, Cip, Cop = ctx.dims
        dz = dz.contiguous()
        B, T, _ = xp.shape
        M = B * T
        dev = xp.device
        W_param, b_param, g_param, be_param = ctx.params
        dy = (torch.zeros if Cop != Co else torch.empty)((B, T, Cop), device=dev, dtype=torch.float32)
        need_g, need_b = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        gg = _GradOut(g_param, (Co,), dev) if need_g else None
        gb = _GradOut(be_param, (Co,), dev) if need_b else None
        acc = bool(gg is not None and gb is not None and gg.acc and gb.acc)
        if not acc:  # both-or-neither: one accumulate flag for the pair
            gg = _GradOut(None, (Co,), dev) if need_g else None
            gb = _GradOut(None, (Co,), dev) if need_b else None
        ws = _ws(dev, _lib.load().autovc_bn_workspace_bytes(Co), "bn")
        _lib.call("autovc_bn_act_bwd_f32", M, Co, dz.data_ptr(), Co, _p(z), Co, y.data_ptr(), Cop,
                  mean.data_ptr(), var.data_ptr(), _p(gamma), float(ctx.eps), ACT[ctx.act],
                  dy.data_ptr(), Cop, _p(gg.buf if gg else None), _p(gb.buf if gb else None), int(acc), ws, _s())
        dgamma = gg.result() if gg else None
        dbeta = gb.result() if gb else None
        dx, dW, db = _conv_bwd(dy, xp, Wp, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               ctx.needs_input_grad[2], W_param, b_param, ctx.xt)
        ctx.xt = None
        if dx is not None and Cip != Ci:
            dx = dx[..., :Ci].contiguous()
        if dW is not None and (Cop, Cip) != (Co, Ci):
            dW = dW[:Co, :Ci].contiguous()
        if db is not None and Cop != Co:
            db = db[:Co].contiguous()
        dres = dz if ctx.has_res else None
        return dx, dW, db, dgamma, dbeta, None, None, None, None, None, None, None, dres


def conv_bn_act(x, conv, bn, act, residual=None):
    """x (B,T,Ci) -> act(bn(conv(x))) (+ residual); conv: nn.Conv1d, bn: nn.BatchNorm1d."""
    training = bn.training
    momentum = bn.momentum if bn.momentum is not None else 0.0
    nbt = bn.num_batches_tracked if (training and bn.track_running_stats) else None
    if not training and (bn.running_mean is None or bn.running_var is None):
        raise RuntimeError("eval-mode BatchNorm without running stats is not supported")
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return ConvBNActFn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, rm, rv, nbt, training, act,
                             momentum, bn.eps, residual)


# ---------------------------------------------------------------- fused Conv-BN stacks
# A whole ConvNorm -> BatchNorm1d -> act stack (encoder 3 x relu, decoder 3 x relu, postnet
# 4 x tanh + 1 x none with the residual, model_vc_mel.py:49-59,68-69,92-102,113-115,132-169)
# as one autograd op whose BatchNorm passes live inside the Winograd transforms
# (csrc/winograd.hip "fused Conv-BN chain"): every pre-BN activation y_l is written once and
# read by the next layer's input transform, which applies BN_l + act on load; only the
# stack's output is materialised.  AVC_CONV_CHAIN=0 selects the per-layer ConvBNActFn path.
_CHAIN_ON = os.environ.get("AVC_CONV_CHAIN", "1") != "0"


# (The stacks' BatchNorm statistics finalized inside the launch that reduces them measured
# slower than the separate 5 us finalize launch — fp32 14.58-14.63 vs 14.51-14.52 ms/step, bf16
# 9.11 vs 8.96-8.98, profiles/r04/ab_bn_fused_stats.txt — and is retired to tools/retired/.)


def _chain_ok(x, layers, training):
    if not (_CHAIN_ON and _WINOGRAD and _PRECISION[0] == "fp32" and x.is_cuda and x.dim() == 3
            and x.dtype == torch.float32):
        return False
    T = x.shape[1]
    if T % 4 or x.shape[2] % 4 or _lib.load().autovc_wino5_rows(x.shape[0], T) <= 0:
        return False
    for conv, bn, _ in layers:
        if (conv.kernel_size[0] != KS or conv.padding[0] != PAD or conv.stride[0] != 1 or conv.dilation[0] != 1
                or conv.groups != 1 or conv.out_channels % 4 or conv.in_channels % 4):
            return False
        if bn.training != training or not bn.track_running_stats or bn.running_mean is None or not bn.affine:
            return False
    return True


def _bn_bwd_finalize(pending, rows, C, part, var, eps, sums, gg, gb, acc):
    """A stack layer's BatchNorm-backward sums (+ dgamma / dbeta), in the same launch as the
    deeper layer's pending conv bias finalize when there is one."""
    if pending is None:
        _lib.call("autovc_bn_bwd_finalize_f32", rows, C, part, var.data_ptr(), float(eps), sums,
                  _p(gg.buf if gg else None), _p(gb.buf if gb else None), int(acc), _s())
        return
    rs_b, c_b, bpart, go = pending
    _lib.call("autovc_bn_bwd_finalize_bias_f32", rows, C, part, var.data_ptr(), float(eps), sums,
              _p(gg.buf if gg else None), _p(gb.buf if gb else None), int(acc), rs_b, c_b, bpart,
              go.buf.data_ptr(), int(go.acc), _s())


def _bias_finalize(pending):
    if pending is not None:
        rs_b, c_b, bpart, go = pending
        _lib.call("autovc_colsum_f64_finalize_f32", rs_b, c_b, bpart, go.buf.data_ptr(), int(go.acc), _s())


class ConvBNChainFn(torch.autograd.Function):
    """Forward / backward of a Conv-BN-act stack (see above).  apply(spec, x, residual,
    *per-layer (W, b, gamma, beta, running_mean, running_var, num_batches_tracked));
    spec = (training, acts, momenta, epss)."""

    @staticmethod
    def forward(ctx, spec, x, residual, *tensors):
        training, acts, moms, epss = spec
        L = len(acts)
        x = x.contiguous()
        B, T, _ = x.shape
        M, nt = B * T, B * T // 4
        dev = x.device
        lib = _lib.load()
        RS = int(lib.autovc_wino5_rows(B, T))
        ys, coefs, means, varis, xts = [], [], [], [], []
        for l in range(L):
            W, b, g, be, rm, rv, nbt = tensors[7 * l:7 * l + 7]
            Co, Ci = W.shape[0], W.shape[1]
            Wt = conv_weight(W, 0)
            Xt = torch.empty((8, nt, Ci), device=dev, dtype=torch.float32)
            if l == 0:
                _lib.call("autovc_wino5_input_f32", B, T, Ci, x.data_ptr(), Ci, Xt.data_ptr(), _s())
            else:
                _lib.call("autovc_wino5_input_bn_f32", B, T, Ci, ys[-1].data_ptr(), Ci, coefs[-1].data_ptr(),
                          ACT[acts[l - 1]], Xt.data_ptr(), _s())
            Yt = torch.empty((8, nt, Co), device=dev, dtype=torch.float32)
            _lib.call("autovc_gemm_batched_f32", 8, nt, Co, Ci, Xt.data_ptr(), Ci, nt * Ci, 0, Wt.data_ptr(), Ci,
                      Co * Ci, 0, Yt.data_ptr(), Co, nt * Co, 0, _s())
            del Wt
            y = torch.empty((B, T, Co), device=dev, dtype=torch.float32)
            coef = torch.empty((4, Co), device=dev, dtype=torch.float32)
            if training:
                mean = torch.empty(Co, device=dev, dtype=torch.float32)
                var = torch.empty(Co, device=dev, dtype=torch.float32)
                part = _ws(dev, RS * Co * 16, "chain_fwd")
                _lib.call("autovc_wino5_output_stats_f32", B, T, Co, Yt.data_ptr(), _p(b), y.data_ptr(), Co, part,
                          _s())
                _lib.call("autovc_bn_finalize_f32", RS, M, Co, part, _p(g), _p(be), float(epss[l]),
                          mean.data_ptr(), var.data_ptr(), coef.data_ptr(), _p(rm), _p(rv), float(moms[l]), _p(nbt),
                          _s())
            else:
                _lib.call("autovc_wino5_output_f32", B, T, Co, Yt.data_ptr(), _p(b), y.data_ptr(), Co, _s())
                mean, var = rm, rv
                _lib.call("autovc_bn_coef_f32", Co, rm.data_ptr(), rv.data_ptr(), _p(g), _p(be), float(epss[l]),
                          coef.data_ptr(), _s())
            del Yt
            ys.append(y)
            coefs.append(coef)
            means.append(mean)
            varis.append(var)
            xts.append(Xt if training else None)
            del Xt
        C = ys[-1].shape[2]
        g, be = tensors[7 * (L - 1) + 2], tensors[7 * (L - 1) + 3]
        z = torch.empty((B, T, C), device=dev, dtype=torch.float32)
        res = residual.contiguous() if residual is not None else None
        _lib.call("autovc_bn_act_fwd_f32", M, C, ys[-1].data_ptr(), C, means[-1].data_ptr(), varis[-1].data_ptr(),
                  _p(g), _p(be), float(epss[-1]), ACT[acts[-1]], _p(res), C, z.data_ptr(), C, _s())
        if training:
            ctx.spec = spec
            ctx.last_pass = _BLSTM_LAST_PASS[0]
            ctx.ys, ctx.coefs, ctx.means, ctx.varis, ctx.xts = ys, coefs, means, varis, xts
            ctx.x = x
            ctx.z = z if acts[-1] != "none" else None
            ctx.has_res = residual is not None
            ctx.params = tensors
        else:
            ctx.spec = None
        return z

    @staticmethod
    def backward(ctx, dz):
        if ctx.spec is None:
            raise NotImplementedError("autovc_amd: backward through eval-mode BatchNorm is not supported")
        training, acts, moms, epss = ctx.spec
        L = len(acts)
        needs = ctx.needs_input_grad
        x, ys, coefs, means, varis, xts = ctx.x, ctx.ys, ctx.coefs, ctx.means, ctx.varis, ctx.xts
        tensors = ctx.params
        B, T, _ = x.shape
        M, nt = B * T, B * T // 4
        dev = x.device
        lib = _lib.load()
        RS = int(lib.autovc_wino5_rows(B, T))
        dres = dz.contiguous() if ctx.has_res else None
        dz = dz.contiguous()
        grads = [None] * len(tensors)
        dx = None
        part, rows = None, 0
        pending = None   # the previous layer's conv bias partials, finalized in the next launch
        for l in range(L - 1, -1, -1):
            W, b, g, be = tensors[7 * l:7 * l + 4]
            Co, Ci = W.shape[0], W.shape[1]
            act = ACT[acts[l]]
            y = ys[l]
            # BatchNorm backward sums of layer l (the stack's last layer reduces its dz here;
            # the others got them from the output transform that produced dz)
            if l == L - 1:
                rows = int(lib.autovc_bn_partial_rows(M))
                part = _ws(dev, rows * Co * 16, "chain_bwd")
                _lib.call("autovc_bn_bwd_partial_f32", M, Co, dz.data_ptr(), Co, _p(ctx.z), Co, y.data_ptr(), Co,
                          means[l].data_ptr(), act, part, _s())
            ng, nb = needs[3 + 7 * l + 2], needs[3 + 7 * l + 3]
            gg = _GradOut(g, (Co,), dev) if ng else None
            gb = _GradOut(be, (Co,), dev) if nb else None
            acc = bool(gg is not None and gb is not None and gg.acc and gb.acc)
            if not acc:
                gg = _GradOut(None, (Co,), dev) if ng else None
                gb = _GradOut(None, (Co,), dev) if nb else None
            sums = _ws(dev, 8 * Co, "chain_sums")
            _bn_bwd_finalize(pending, rows, Co, part, varis[l], epss[l], sums, gg, gb, acc)
            pending = None
            if gg is not None:
                grads[7 * l + 2] = gg.result()
            if gb is not None:
                grads[7 * l + 3] = gb.result()
            need_w, need_b = needs[3 + 7 * l], b is not None and needs[3 + 7 * l + 1]
            need_dx = l > 0 or needs[1]
            Dt = torch.empty((8, nt, Co), device=dev, dtype=torch.float32) if need_w else None
            Xd = torch.empty((8, nt, Co), device=dev, dtype=torch.float32) if need_dx else None
            bpart = _ws(dev, RS * Co * 8, "chain_bias") if need_b else 0
            if Dt is not None or Xd is not None or need_b:
                _lib.call("autovc_wino5_bnbwd_f32", B, T, Co, dz.data_ptr(), Co, y.data_ptr(), Co,
                          coefs[l].data_ptr(), act, sums, _p(Dt), _p(Xd), bpart, _s())
            if need_b:   # finalized with the next layer's BatchNorm sums (one launch) or after the loop
                go = _GradOut(b, (Co,), dev)
                pending = (RS, Co, bpart, go)
                grads[7 * l + 1] = go.result()
            if need_w:
                go = _GradOut(W, (Co, Ci, KS), dev)
                Xt = xts[l]

                def dw(go=go, Dt=Dt, Xt=Xt, Co=Co, Ci=Ci):
                    Mt = torch.empty((8, Co, Ci), device=dev, dtype=torch.float32)
                    _lib.call("autovc_gemm_batched_f32", 8, Co, Ci, nt, Dt.data_ptr(), Co, nt * Co, 1, Xt.data_ptr(),
                              Ci, nt * Ci, 1, Mt.data_ptr(), Ci, Co * Ci, 0, _s())
                    _lib.call("autovc_wino5_wgrad_f32", Co, Ci, Mt.data_ptr(), go.buf.data_ptr(), int(go.acc), _s())
                # (AVC_LAST_CONV_MAIN=1: the last-differentiated encoder pass's conv weight
                # gradients on the main stream instead of the final side batch)
                if ctx.last_pass and _last_conv_main():
                    _main_grad(dev, go, dw, Dt, Xt)
                else:
                    _grad_launch(dev, go, dw, Dt, Xt)
                grads[7 * l] = go.result()
            xts[l] = None
            if need_dx:
                Wd = conv_weight(W, 1)
                Yd = torch.empty((8, nt, Ci), device=dev, dtype=torch.float32)
                _lib.call("autovc_gemm_batched_f32", 8, nt, Ci, Co, Xd.data_ptr(), Co, nt * Co, 0, Wd.data_ptr(), Co,
                          Ci * Co, 0, Yd.data_ptr(), Ci, nt * Ci, 0, _s())
                del Wd, Xd
                dzp = torch.empty((B, T, Ci), device=dev, dtype=torch.float32)
                if l > 0:
                    rows = RS
                    part = _ws(dev, RS * Ci * 16, "chain_bwd")
                    _lib.call("autovc_wino5_output_bnbwd_f32", B, T, Ci, Yd.data_ptr(), ys[l - 1].data_ptr(), Ci,
                              coefs[l - 1].data_ptr(), ACT[acts[l - 1]], dzp.data_ptr(), Ci, part, _s())
                    dz = dzp
                else:
                    _lib.call("autovc_wino5_output_f32", B, T, Ci, Yd.data_ptr(), 0, dzp.data_ptr(), Ci, _s())
                    dx = dzp
                del Yd
        _bias_finalize(pending)
        ctx.ys = ctx.xts = ctx.coefs = None
        return (None, dx, dres, *grads)


# AVC_CONV_CHAIN_BF16: 0 = per-layer ConvBNActFn under bf16; 1 = the stacks with BatchNorm
# applied while the GEMMs stage fp32 operands; 2 = the stacks on bf16 copies written by the
# producers (BatchNorm + activation -> bf16 z, dy -> bf16, bf16 weight packs)
_CHAIN_BF16_MODE = int(os.environ.get("AVC_CONV_CHAIN_BF16", "2"))
_CHAIN_BF16_ON = _CHAIN_BF16_MODE != 0


def _chain_ok_bf16(x, layers, training):
    q = 8 if _CHAIN_BF16_MODE == 2 else 4
    if not (_CHAIN_BF16_ON and _PRECISION[0] == "bf16" and x.is_cuda and x.dim() == 3
            and x.dtype == torch.float32 and x.shape[2] % q == 0):
        return False
    for conv, bn, _ in layers:
        if (conv.kernel_size[0] != KS or conv.padding[0] != PAD or conv.stride[0] != 1 or conv.dilation[0] != 1
                or conv.groups != 1 or conv.out_channels % q or conv.in_channels % q):
            return False
        if bn.training != training or not bn.track_running_stats or bn.running_mean is None or not bn.affine:
            return False
    return True


class ConvBNChainBf16Fn(torch.autograd.Function):
    """The Conv-BN-act stack under precision("bf16") (BASELINE config 3), where the convs
    are bf16 im2col GEMMs (csrc/gemm.hip "fused Conv-BN stacks (bf16)").  Every conv GEMM's
    split-K reduce writes its pre-BN output y together with y's BatchNorm partials (no
    statistics pass), the input-gradient GEMM's reduce emits the previous layer's
    BatchNorm-backward sums, and one kernel per layer turns (dz, y) into dy and the conv
    bias partials.  How the next GEMMs get act(BN(y)):
      mode 1: applied while they stage y (fp32) into their bf16 LDS tiles;
      mode 2: one pass writes a bf16 copy z = bf16(act(BN(y))) that they read as is (as
              dy and the packed weights: bf16-source operands, half the operand bytes).
    Only the stack's output is materialised in fp32.  Same apply(spec, x, residual,
    *tensors) as ConvBNChainFn."""

    @staticmethod
    def forward(ctx, spec, x, residual, *tensors):
        training, acts, moms, epss = spec
        mode = _CHAIN_BF16_MODE
        h = mode == 2
        L = len(acts)
        x = x.contiguous()
        B, T, _ = x.shape
        M = B * T
        dev = x.device
        lib = _lib.load()
        RS = int(lib.autovc_bnconv_stats_rows(M))
        ys, coefs, means, varis, zbs = [], [], [], [], []
        for l in range(L):
            W, b, g, be, rm, rv, nbt = tensors[7 * l:7 * l + 7]
            Co, Ci = W.shape[0], W.shape[1]
            Wf = conv_weight(W, 4 if h else 2)
            y = torch.empty((B, T, Co), device=dev, dtype=torch.float32)
            part = _ws(dev, RS * Co * 16, "chain_fwd")
            ws = _ws(dev, 4 * lib.autovc_bnconv_workspace_floats(B, T, Ci, Co), "bnconv")
            if l == 0:
                xin, xcoef, xact, src = x, None, 0, (2 if h else 0)
            elif h:
                xin, xcoef, xact, src = zbs[-1], None, 0, 3
            else:
                xin, xcoef, xact, src = ys[-1], coefs[-1], ACT[acts[l - 1]], 0
            coef = torch.empty((4, Co), device=dev, dtype=torch.float32)
            _lib.call("autovc_bnconv_fwd_bf16_f32", B, T, Ci, Co, xin.data_ptr(), _p(xcoef), xact, Wf.data_ptr(),
                      _p(b), y.data_ptr(), part, src, ws, _s())
            if training:
                mean = torch.empty(Co, device=dev, dtype=torch.float32)
                var = torch.empty(Co, device=dev, dtype=torch.float32)
                _lib.call("autovc_bn_finalize_f32", RS, M, Co, part, _p(g), _p(be), float(epss[l]), mean.data_ptr(),
                          var.data_ptr(), coef.data_ptr(), _p(rm), _p(rv), float(moms[l]), _p(nbt), _s())
            elif not training:
                mean, var = rm, rv
                _lib.call("autovc_bn_coef_f32", Co, rm.data_ptr(), rv.data_ptr(), _p(g), _p(be), float(epss[l]),
                          coef.data_ptr(), _s())
            if h and l < L - 1:
                zb = torch.empty((B, T, Co), device=dev, dtype=torch.bfloat16)
                _lib.call("autovc_bn_apply_bf16", M, Co, y.data_ptr(), coef.data_ptr(), ACT[acts[l]], zb.data_ptr(),
                          _s())
                zbs.append(zb)
            ys.append(y)
            coefs.append(coef)
            means.append(mean)
            varis.append(var)
        C = ys[-1].shape[2]
        g, be = tensors[7 * (L - 1) + 2], tensors[7 * (L - 1) + 3]
        z = torch.empty((B, T, C), device=dev, dtype=torch.float32)
        res = residual.contiguous() if residual is not None else None
        _lib.call("autovc_bn_act_fwd_f32", M, C, ys[-1].data_ptr(), C, means[-1].data_ptr(), varis[-1].data_ptr(),
                  _p(g), _p(be), float(epss[-1]), ACT[acts[-1]], _p(res), C, z.data_ptr(), C, _s())
        if training:
            ctx.spec, ctx.mode = spec, mode
            ctx.last_pass = _BLSTM_LAST_PASS[0]
            ctx.ys, ctx.coefs, ctx.means, ctx.varis, ctx.zbs = ys, coefs, means, varis, zbs
            ctx.x = x
            ctx.z = z if acts[-1] != "none" else None
            ctx.has_res = residual is not None
            ctx.params = tensors
        else:
            ctx.spec = None
        return z

    @staticmethod
    def backward(ctx, dz):
        if ctx.spec is None:
            raise NotImplementedError("autovc_amd: backward through eval-mode BatchNorm is not supported")
        training, acts, moms, epss = ctx.spec
        h = ctx.mode == 2
        L = len(acts)
        needs = ctx.needs_input_grad
        x, ys, coefs, means, varis, zbs = ctx.x, ctx.ys, ctx.coefs, ctx.means, ctx.varis, ctx.zbs
        tensors = ctx.params
        B, T, _ = x.shape
        M = B * T
        dev = x.device
        lib = _lib.load()
        RS = int(lib.autovc_bnconv_stats_rows(M))
        PR = int(lib.autovc_bn_partial_rows(M))
        dres = dz.contiguous() if ctx.has_res else None
        dz = dz.contiguous()
        grads = [None] * len(tensors)
        dx = None
        part, rows = None, 0
        pending = None   # the previous layer's conv bias partials, finalized in the next launch
        for l in range(L - 1, -1, -1):
            W, b, g, be = tensors[7 * l:7 * l + 4]
            Co, Ci = W.shape[0], W.shape[1]
            y = ys[l]
            if l == L - 1:
                rows = PR
                part = _ws(dev, max(PR, RS) * Co * 16, "chain_bwd")
                _lib.call("autovc_bn_bwd_partial_f32", M, Co, dz.data_ptr(), Co, _p(ctx.z), Co, y.data_ptr(), Co,
                          means[l].data_ptr(), ACT[acts[l]], part, _s())
            ng, nb = needs[3 + 7 * l + 2], needs[3 + 7 * l + 3]
            gg = _GradOut(g, (Co,), dev) if ng else None
            gb = _GradOut(be, (Co,), dev) if nb else None
            acc = bool(gg is not None and gb is not None and gg.acc and gb.acc)
            if not acc:
                gg = _GradOut(None, (Co,), dev) if ng else None
                gb = _GradOut(None, (Co,), dev) if nb else None
            sums = _ws(dev, 8 * Co, "chain_sums")
            _bn_bwd_finalize(pending, rows, Co, part, varis[l], epss[l], sums, gg, gb, acc)
            pending = None
            if gg is not None:
                grads[7 * l + 2] = gg.result()
            if gb is not None:
                grads[7 * l + 3] = gb.result()
            dy = torch.empty((B, T, Co), device=dev, dtype=torch.bfloat16 if h else torch.float32)
            bpart = _ws(dev, PR * Co * 8, "chain_bias")
            _lib.call("autovc_bn_dy_f32", M, Co, dz.data_ptr(), y.data_ptr(), coefs[l].data_ptr(), ACT[acts[l]], sums,
                      0 if h else dy.data_ptr(), dy.data_ptr() if h else 0, bpart, _s())
            if b is not None and needs[3 + 7 * l + 1]:
                go = _GradOut(b, (Co,), dev)
                pending = (PR, Co, bpart, go)
                grads[7 * l + 1] = go.result()
            if l == 0:
                xin, xcoef, xact, wsrc = x, None, 0, (1 if h else 0)
            elif h:
                xin, xcoef, xact, wsrc = zbs[l - 1], None, 0, 3
            else:
                xin, xcoef, xact, wsrc = ys[l - 1], coefs[l - 1], ACT[acts[l - 1]], 0
            if needs[3 + 7 * l]:
                go = _GradOut(W, (Co, Ci, KS), dev)

                def dw(go=go, dy=dy, xin=xin, xcoef=xcoef, xact=xact, wsrc=wsrc, Co=Co, Ci=Ci):
                    dWf = torch.empty((Co, KS * Ci), device=dev, dtype=torch.float32)
                    ws = _ws(dev, 4 * _lib.load().autovc_bnconv_workspace_floats(B, T, Ci, Co), "bnconv")
                    _lib.call("autovc_bnconv_dw_bf16_f32", B, T, Co, Ci, dy.data_ptr(), xin.data_ptr(), _p(xcoef),
                              xact, dWf.data_ptr(), wsrc, ws, _s())
                    _lib.call("autovc_conv_unpack_grad_f32", Co, Ci, KS, dWf.data_ptr(), go.buf.data_ptr(),
                              int(go.acc), _s())
                if ctx.last_pass and _last_conv_main():   # (as ConvBNChainFn)
                    _main_grad(dev, go, dw, dy, xin, xcoef)
                else:
                    _grad_launch(dev, go, dw, dy, xin, xcoef)
                grads[7 * l] = go.result()
            if l > 0 or needs[1]:
                Wd = conv_weight(W, 5 if h else 3)
                dzp = torch.empty((B, T, Ci), device=dev, dtype=torch.float32)
                ws = _ws(dev, 4 * lib.autovc_bnconv_workspace_floats(B, T, Ci, Co), "bnconv")
                src = 3 if h else 0
                if l > 0:
                    rows = RS
                    part = _ws(dev, max(PR, RS) * Ci * 16, "chain_bwd")
                    _lib.call("autovc_bnconv_dx_bf16_f32", B, T, Co, Ci, dy.data_ptr(), Wd.data_ptr(), dzp.data_ptr(),
                              ys[l - 1].data_ptr(), coefs[l - 1].data_ptr(), ACT[acts[l - 1]], part, src, ws, _s())
                    dz = dzp
                else:
                    _lib.call("autovc_bnconv_dx_bf16_f32", B, T, Co, Ci, dy.data_ptr(), Wd.data_ptr(), dzp.data_ptr(),
                              0, 0, 0, 0, src, ws, _s())
                    dx = dzp
        _bias_finalize(pending)
        ctx.ys = ctx.coefs = ctx.zbs = None
        return (None, dx, dres, *grads)


def conv_bn_chain(x, layers, residual=None):
    """x (B,T,C) -> a Conv-BN-act stack; layers = [(nn.Conv1d, nn.BatchNorm1d, act), ...],
    residual (optional) is added to the last layer's output.  The fused ConvBNChainFn where
    it applies (fp32, Winograd shapes) or ConvBNChainBf16Fn (bf16), else one ConvBNActFn
    per layer."""
    training = layers[0][1].training
    fn = ConvBNChainFn
    if _chain_ok_bf16(x, layers, training):
        fn = ConvBNChainBf16Fn
    elif not _chain_ok(x, layers, training):
        for i, (conv, bn, act) in enumerate(layers):
            x = conv_bn_act(x, conv, bn, act, residual=residual if i == len(layers) - 1 else None)
        return x
    tensors = []
    for conv, bn, _ in layers:
        nbt = bn.num_batches_tracked if training else None
        tensors += [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var, nbt]
    spec = (training, tuple(a for _, _, a in layers),
            tuple((bn.momentum if bn.momentum is not None else 0.0) for _, bn, _ in layers),
            tuple(bn.eps for _, bn, _ in layers))
    return fn.apply(spec, x, residual, *tensors)


class ConvFn(torch.autograd.Function):
    """Plain ConvNorm (k=5, p=2) on NTC activations (ConvNorm.forward API path)."""

    @staticmethod
    def forward(ctx, x, W, b):
        _check(x, "conv")
        B, T, Ci = x.shape
        Co = W.shape[0]
        Cip, Cop = _ceil4(Ci), _ceil4(Co)
        xp = _pad_last(x, Cip)
        Wp = _padded_weight(W, Cop, Cip)
        bp = b if (b is None or Cop == Co) else _pad_last(b, Cop)
        y = _conv_fwd(xp, Wp, bp, T)
        ctx.save_for_backward(xp, Wp)
        ctx.dims = (Ci, Co, Cip, Cop)
        ctx.has_b = b is not None
        ctx.params = (W, b)
        return y if Cop == Co else y[..., :Co].contiguous()

    @staticmethod
    def backward(ctx, dy):
        xp, Wp = ctx.saved_tensors
        Ci, Co, Cip, Cop = ctx.dims
        dyp = _pad_last(dy, Cop)
        dx, dW, db = _conv_bwd(dyp, xp, Wp, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               ctx.has_b and ctx.needs_input_grad[2], *ctx.params)
        if dx is not None and Cip != Ci:
            dx = dx[..., :Ci].contiguous()
        if dW is not None and (Cop, Cip) != (Co, Ci):
            dW = dW[:Co, :Ci].contiguous()
        if db is not None and Cop != Co:
            db = db[:Co].contiguous()
        return dx, dW, db


def conv_only(x, W, b):
    return ConvFn.apply(x, W, b)


# ---------------------------------------------------------------- Linear
class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        _check(x, "linear")
        x = x.contiguous()
        lead = x.shape[:-1]
        K = x.shape[-1]
        N = W.shape[0]
        M = x.numel() // K
        y = torch.empty((*lead, N), device=x.device, dtype=torch.float32)
        gemm(M, N, K, x, K, 0, W, K, 0, y, N, bias1=b)
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        ctx.params = (W, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        W_param, b_param = ctx.params
        K = x.shape[-1]
        N = W.shape[0]
        M = x.numel() // K
        dev = x.device
        Np = _ceil4(N)  # 513-bin projection: pad the output axis for the float4 GEMM operands
        dy = _pad_last(dy.reshape(M, N), Np)
        Wp = W.contiguous() if Np == N else torch.cat([W, W.new_zeros(Np - N, K)], 0)
        dx = dW = db = None
        if ctx.needs_input_grad[1]:
            go = _GradOut(W_param if Np == N else None, (Np, K), dev)
            _grad_launch(dev, go, lambda go=go: gemm(Np, K, M, dy, Np, 1, x, K, 1, go.buf, K,
                                                         splits=_splits_for(Np, K, M), accumulate=go.acc), dy, x)
            dW = go.result()
            dW = dW if (dW is None or Np == N) else dW[:N].contiguous()
        if ctx.has_b and ctx.needs_input_grad[2]:
            go = _GradOut(b_param if Np == N else None, (Np,), dev)
            _grad_launch(dev, go, lambda go=go: colsum(dy, go.buf, accumulate=go.acc), dy)
            db = go.result()
            db = db if (db is None or Np == N) else db[:N].contiguous()
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            gemm(M, K, Np, dy, Np, 0, Wp, K, 1, dx, K)
        return dx, dW, db


def linear(x, W, b):
    return LinearFn.apply(x, W, b)


# ---------------------------------------------------------------- LSTM layers
class LSTMLayerFn(torch.autograd.Function):
    """One unidirectional nn.LSTM layer with large H (decoder lstm1 / lstm2)."""

    @staticmethod
    def forward(ctx, x, W_ih, W_hh, b_ih, b_hh, save):
        _check(x, "lstm")
        x = x.contiguous()
        B, T, I = x.shape
        H = W_hh.shape[1]
        dev = x.device
        gx = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32)
        gemm(B * T, 4 * H, I, x, I, 0, W_ih, I, 0, gx, 4 * H, bias1=b_ih, bias2=b_hh,
             b_bf16=_wbf16(W_ih) if _bf16_rec(H) else None)
        h = torch.empty((B, T, H), device=dev, dtype=torch.float32)
        c = torch.empty((B, T, H), device=dev, dtype=torch.float32)
        gates = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32) if save else None
        if _bf16_rec(H) and lstm_xcd(B, H):
            Wb = conv_weight(W_hh, 6)
            ws = _ws(dev, _lib.load().autovc_lstm_xcd_workspace_bytes(), "lstmx")
            _lib.call("autovc_lstm_fwd_xcd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(),
                      h.data_ptr(), T * H, H, c.data_ptr(), _p(gates), ws, _s())
        elif _bf16_rec(H):
            hb = torch.empty((B, T, H), device=dev, dtype=torch.bfloat16)
            Wb = conv_weight(W_hh, 6)   # held until the launches are enqueued (stream-ordered reuse after)
            _lib.call("autovc_lstm_fwd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(),
                      h.data_ptr(), hb.data_ptr(), c.data_ptr(), _p(gates), 0, _s())
        elif lstm_xcd(B, H):
            ws = _ws(dev, _lib.load().autovc_lstm_xcd_workspace_bytes(), "lstmx")
            _lib.call("autovc_lstm_fwd_xcd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W_hh.data_ptr(),
                      h.data_ptr(), T * H, H, c.data_ptr(), _p(gates), ws, _s())
        elif lstm_persistent(B, H):
            ws = _ws(dev, _lib.load().autovc_lstm_persist_workspace_bytes(B, T, H), "lstmp")
            _lib.call("autovc_lstm_fwd_persist_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W_hh.data_ptr(),
                      h.data_ptr(), T * H, H, c.data_ptr(), _p(gates), ws, _s())
        else:
            _lib.call("autovc_lstm_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W_hh.data_ptr(),
                      h.data_ptr(), T * H, H, c.data_ptr(), _p(gates), 0, _s())
        ctx.save_for_backward(x, W_ih, W_hh, h, c, gates)
        ctx.params = (W_ih, W_hh, b_ih, b_hh)
        return h

    @staticmethod
    def backward(ctx, dh):
        x, W_ih, W_hh, h, c, gates = ctx.saved_tensors
        return _lstm_layer_backward(dh, x, W_ih, W_hh, h, c, gates, ctx.params, ctx.needs_input_grad[:5]) + (None,)


def set_fp32_gemm(mode):
    """precision fp32's GEMMs: "x6" (bf16 MFMA on exact three-plane operand splits, the default,
    fp32-accurate: csrc/gemm.hip) or "mfma" (v_mfma_f32_32x32x2_f32).  Returns the previous mode."""
    if mode not in ("x6", "mfma"):
        raise ValueError("set_fp32_gemm: 'x6' or 'mfma'")
    return "x6" if _lib.load().autovc_gemm_set_fp32_x6(1 if mode == "x6" else 0) else "mfma"


def fp32_gemm_mode():
    return "x6" if _lib.load().autovc_gemm_fp32_x6() else "mfma"


def _bf16_rec(H):
    """Recurrent products in bf16 under precision("bf16") (H a multiple of 128)."""
    return _PRECISION[0] == "bf16" and H % 128 == 0


def _lstm_layer_backward(dh, x, W_ih, W_hh, h, c, gates, params, needs):
    """BPTT of one large-H layer: recurrence (C-ABI), weight/bias gradients straight into
    the flat gradient buffer where the optimizer owns one, dx.  Returns (dx, dW_ih, dW_hh,
    db_ih, db_hh) for autograd (None where accumulated in place or not needed)."""
    p_ih, p_hh, p_bih, p_bhh = params
    if gates is None:
        raise RuntimeError("LSTM backward needs the forward run with gradients enabled")
    dh = dh.contiguous()
    B, T, I = x.shape
    H = W_hh.shape[1]
    dev = x.device
    # W_hh^T (fp32, or its bf16 copy under bf16): from the step's weight scope when there is one
    WT = conv_weight(W_hh, 8 if _bf16_rec(H) else 7)
    # split-K of the recurrent product (same box, alternating): fp32 4 ways at H=1024 (256
    # workgroups; 8 ways: +0.1 ms/step), 8 ways at H=512 (fills the chip: -0.15 ms); bf16
    # 4 ways with the fused steps (decoder lstm1: 8.46-8.52 vs 8.55-8.57 ms/step for 8 ways,
    # profiles/r05/ab_lstm1_splits.txt; 8 ways measured best with the launch pair, round 2).
    splits = 4 if _bf16_rec(H) else (8 if H <= 512 else 4)
    # the recurrent K (4H fp32 floats, 2H bf16 pairs) must cut into multiples of 64 per split
    kdim = 2 * H if _bf16_rec(H) else 4 * H
    while splits > 1 and kdim % (64 * splits):
        splits //= 2
    dG = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32)
    if lstm_xcd(B, H) and _xcd_bwd():
        # one XCD-local persistent launch (csrc/lstm2_persist.hip lstm_xcd_bwd_kernel)
        ws = _ws(dev, _lib.load().autovc_lstm_xcd_workspace_bytes(), "lstmxb")
        mark = _grad_mark(dev)
        if _bf16_rec(H):
            dGb = torch.empty((B, T, 4 * H), device=dev, dtype=torch.bfloat16)
            _lib.call("autovc_lstm_bwd_xcd_bf16", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), c.data_ptr(),
                      WT.data_ptr(), dG.data_ptr(), dGb.data_ptr(), ws, _s())
        else:
            _lib.call("autovc_lstm_bwd_xcd_f32", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), c.data_ptr(),
                      WT.data_ptr(), dG.data_ptr(), ws, _s())
        # the queued GEMMs unpadded beside it: the launch holds 80.5 KB of LDS on every CU for
        # its whole length, which no per-step recurrence workgroup needs to share
        _flush_grad_queue(after=mark, lds_reserve=0)
        return _lstm_grads_from_dG(dG, x, W_ih, h, params, needs, dGb=dGb if _bf16_rec(H) else None)
    ws = _ws(dev, 4 * _lib.load().autovc_lstm_bwd_workspace_floats(B, H, splits), "lstm")
    # (keeping the batch past this recurrence, to run beside the encoder BLSTMs instead,
    # measured slower: bf16 9.06-9.07 vs 9.03, fp32 15.62-15.64 vs 14.41-14.46 ms,
    # profiles/r05/ab_grad_defer.txt)
    mark = _grad_mark(dev)   # queued weight gradients run beside this latency-bound recurrence
    if _bf16_rec(H):
        dGb = torch.empty((B, T, 4 * H), device=dev, dtype=torch.bfloat16)
        _lib.call("autovc_lstm_bwd_bf16", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), c.data_ptr(),
                  WT.data_ptr(), dG.data_ptr(), dGb.data_ptr(), 0, splits, ws, _s())
    else:
        _lib.call("autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), c.data_ptr(),
                  WT.data_ptr(), dG.data_ptr(), 0, splits, ws, _s())
    _flush_grad_queue(after=mark)
    return _lstm_grads_from_dG(dG, x, W_ih, h, params, needs, dGb=dGb if _bf16_rec(H) else None)


def _lstm_grads_from_dG(dG, x, W_ih, h, params, needs, dGb=None):
    """Parameter gradients (queued beside the next recurrence, into the flat gradient
    buffer) and dx of one large-H layer from its gate gradients dG (B, T, 4H).  dGb: the
    recurrence's bf16 copy of dG (bf16 recurrences), which the GEMMs read instead of dG."""
    p_ih, p_hh, p_bih, p_bhh = params
    kb = {"a_bf16": dGb} if dGb is not None else {}
    keep = (dGb,) if dGb is not None else ()
    B, T, I = x.shape
    H = h.shape[2]
    dev = x.device
    M = B * T
    dx = dWih = dWhh = dbih = dbhh = None
    if needs[1]:
        go = _GradOut(p_ih, W_ih.shape, dev)
        _grad_launch(dev, go, lambda go=go: gemm(4 * H, I, M, dG, 4 * H, 1, x, I, 1, go.buf, I,
                                                     splits=_splits_for(4 * H, I, M), accumulate=go.acc, **kb),
                     dG, x, *keep)
        dWih = go.result()
    if needs[2]:
        go = _GradOut(p_hh, (4 * H, H), dev)
        _grad_launch(dev, go, lambda go=go: gemm(4 * H, H, M, dG, 4 * H, 1, h, H, 1, go.buf, H, b_conv=(T, H, -1),
                                                     splits=_splits_for(4 * H, H, M), accumulate=go.acc, **kb),
                     dG, h, *keep)
        dWhh = go.result()
    if needs[3] or needs[4]:
        gi, gh = _bias_outs(p_bih, p_bhh, (4 * H,), dev)
        _grad_launch(dev, (gi, gh), lambda gi=gi, gh=gh: colsum(dG.view(M, 4 * H), gi.buf, gh.buf, accumulate=gi.acc),
                     dG)
        dbih, dbhh = gi.result(), gh.result()
    if needs[0]:
        dx = torch.empty_like(x)
        gemm(M, I, 4 * H, dG, 4 * H, 0, W_ih, I, 1, dx, I, b_bf16=_wbf16(W_ih) if dGb is not None else None, **kb)
    return dx, dWih, dWhh, dbih, dbhh


# Time-chunked LSTM weight gradients (round 5, AVC_DW_CHUNKS: lstm2's dW GEMMs started per
# finished time chunk) measured slower (fp32 14.53 vs 15.69-16.62 ms/step, bf16 9.02 vs
# 9.74-10.19; profiles/r05/ab_dw_chunks.txt) and are retired to tools/retired/ (buildable from
# 35d60fe): the whole-sequence GEMMs released beside lstm1's backward stay.


# decoder lstm2 forward (fp32) as ONE persistent weight-stationary launch
# (csrc/lstm2_persist.hip) where the shape and device allow it (H = 1024, B = 64, one
# workgroup per CU): 20.3 vs 23.7 us per wavefront iteration (profiles/r02/lstm2_persist_ab.txt);
# AVC_LSTM2_PERSIST=0 selects the per-step launches
_PERSIST_ON = os.environ.get("AVC_LSTM2_PERSIST", "1") != "0"


def lstm2_persistent(B, H):
    return _PERSIST_ON and bool(_lib.load().autovc_lstm2_persist_supported(B, H))


class DeviceFault(RuntimeError):
    """A kernel reported a failure through the device fault word (autovc_fault_status)."""


# fault-word bits (csrc/lstm2_persist.hip) -> (kernel, what it overwrote, the switch that avoids it)
_FAULT_BITS = (
    (1, "lstm_persist_kernel / lstm2_rs_kernel, two layers (decoder lstm2 forward)", "h/c", "AVC_LSTM2_PERSIST=0"),
    (2, "lstm_xcd_fwd_kernel (decoder lstm1 forward)", "h/c", "AVC_LSTM_XCD=0"),
    (4, "lstm_xcd_bwd_kernel (decoder lstm1 backward)", "gate gradients", "AVC_LSTM_XCD_BWD=0"),
    (8, "lstm_persist_kernel, one layer (decoder lstm1 forward)", "h/c", "AVC_LSTM_PERSIST=0"),
)


def check_device_faults(device=None):
    """Raise DeviceFault if a persistent LSTM launch's grid barrier timed out since the
    last check (the launch then wrote NaN over its outputs, so the losses are NaN too).
    Synchronises the current stream: called at the Solver's log steps and by bench.py,
    never per iteration."""
    import ctypes
    v = ctypes.c_int(0)
    _lib.call("autovc_fault_status", _lib.stream_ptr(device), 1, ctypes.byref(v))
    hit = [f for f in _FAULT_BITS if v.value & f[0]]
    if hit:
        names = "; ".join(f"{k} (its {what} were overwritten with NaN; {env} avoids it)" for _, k, what, env in hit)
        raise DeviceFault(
            f"persistent kernel grid barrier timed out: {names}.  Its workgroups were not all resident at once "
            "(another process's kernels held part of the GPU?): run one training process per GPU "
            "(INTEGRATION.md, Co-residency).")


# the single-layer recurrence (decoder lstm1, H = 512) the same way — opt-in
# (AVC_LSTM_PERSIST=1): at H = 512 the grid barrier costs what the launch boundary did
# (6.58 vs 6.75 us per step, profiles/r02/lstm_persist_ab.txt; 16.47-16.50 vs 16.49-16.55 ms
# per training step), so the per-step launches and their cell arithmetic stay the default
_PERSIST1_ON = os.environ.get("AVC_LSTM_PERSIST", "0") != "0"


def lstm_persistent(B, H):
    return _PERSIST1_ON and bool(_lib.load().autovc_lstm_persist_supported(B, H))


# decoder lstm1 forward (fp32, B = 64, H = 512) as one persistent launch whose batch rows are
# split over the 8 XCDs, every synchronisation inside one XCD's L2 (csrc/lstm2_persist.hip
# "XCD-local recurrences"); AVC_LSTM_XCD=0 selects the per-step launches
_XCD_ON = os.environ.get("AVC_LSTM_XCD", "1") != "0"


# The backward the same way (lstm_xcd_bwd_kernel, 1.0 vs 1.55 ms per call in the step graph):
# under precision fp32, once the X6 GEMMs had shortened the side stream (the main stream's
# lstm1 backward then ran 2.3 ms beside them), 12.43 vs 12.95-12.99 ms/step (profiles/r06/
# ab_lstm1_xcd_bwd.txt, ab_lstm1_xcd_bwd_x6.txt).  Under bf16 it alone is neutral (7.92-7.93 vs
# 7.83-7.85): the recurrence shrinks to 0.33 ms but the side stream, with lstm1's weight
# gradients queued behind lstm2's, becomes the tail (side_timeline_bf16_xcdbwd.txt); those three
# launches on the main stream gave 7.71-7.73 (ab_lstm1_dw_main.txt; fp32 slower, 12.78 vs 12.62),
# and once the BLSTM routing and the 3-split weight-gradient GEMMs had shortened the side
# stream, back on the side stream 7.49-7.54 vs 7.62-7.64 (ab_bf16_rebalance.txt).
# AVC_LSTM_XCD_BWD=0 / 1 forces the launch.
_XCD_BWD_ENV = os.environ.get("AVC_LSTM_XCD_BWD")


def _xcd_bwd():
    if _XCD_BWD_ENV is not None:
        return _XCD_BWD_ENV == "1"
    return True




def lstm_xcd(B, H):
    return _XCD_ON and bool(_lib.load().autovc_lstm_xcd_supported(B, H))


class LSTM2StackFn(torch.autograd.Function):
    """Two stacked unidirectional large-H layers (decoder lstm2 = nn.LSTM(512, 1024, 2),
    model_vc_mel.py:104,118).  Forward: one GEMM for the layer-0 input projection, then
    autovc_lstm2_fwd_f32 runs both recurrences as a one-step-lagged wavefront (T + 1
    launches; layer 1's input projection is the first K segment of its step).  Backward:
    layer 1 then layer 0, as two LSTMLayerFn backwards."""

    @staticmethod
    def forward(ctx, x, W_ih0, W_hh0, b_ih0, b_hh0, W_ih1, W_hh1, b_ih1, b_hh1, save):
        _check(x, "lstm")
        x = x.contiguous()
        B, T, I = x.shape
        H = W_hh0.shape[1]
        dev = x.device
        gx0 = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32)
        gemm(B * T, 4 * H, I, x, I, 0, W_ih0, I, 0, gx0, 4 * H, bias1=b_ih0, bias2=b_hh0,
             b_bf16=_wbf16(W_ih0) if _bf16_rec(H) else None)
        h0, c0, h1, c1 = (torch.empty((B, T, H), device=dev, dtype=torch.float32) for _ in range(4))
        g0 = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32) if save else None
        g1 = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32) if save else None
        if _bf16_rec(H):
            h0b, h1b = (torch.empty((B, T, H), device=dev, dtype=torch.bfloat16) for _ in range(2))
            # the bf16 weight copies must be alive together (a temporary's block would be
            # reused by the next conversion before the launches read it)
            W0b, Wi1b, W1b = conv_weight(W_hh0, 6), conv_weight(W_ih1, 6), conv_weight(W_hh1, 6)
            if lstm2_persistent(B, H):
                ws = _ws(dev, _lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), "lstm2p")
                _lib.call("autovc_lstm2_fwd_persist_bf16", B, T, H, gx0.data_ptr(), T * 4 * H, 4 * H,
                          W0b.data_ptr(), b_ih1.data_ptr(), b_hh1.data_ptr(), Wi1b.data_ptr(), W1b.data_ptr(),
                          h0.data_ptr(), c0.data_ptr(), _p(g0), h1.data_ptr(), c1.data_ptr(), _p(g1), ws, _s())
            else:
                _lib.call("autovc_lstm2_fwd_bf16", B, T, H, gx0.data_ptr(), T * 4 * H, 4 * H, W0b.data_ptr(),
                          b_ih1.data_ptr(), b_hh1.data_ptr(), Wi1b.data_ptr(), W1b.data_ptr(),
                          h0.data_ptr(), h0b.data_ptr(), c0.data_ptr(), _p(g0), h1.data_ptr(), h1b.data_ptr(),
                          c1.data_ptr(), _p(g1), _s())
        elif lstm2_persistent(B, H):
            ws = _ws(dev, _lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), "lstm2p")
            _lib.call("autovc_lstm2_fwd_persist_f32", B, T, H, gx0.data_ptr(), T * 4 * H, 4 * H, W_hh0.data_ptr(),
                      b_ih1.data_ptr(), b_hh1.data_ptr(), W_ih1.data_ptr(), W_hh1.data_ptr(), h0.data_ptr(),
                      c0.data_ptr(), _p(g0), h1.data_ptr(), c1.data_ptr(), _p(g1), ws, _s())
        else:
            _lib.call("autovc_lstm2_fwd_f32", B, T, H, gx0.data_ptr(), T * 4 * H, 4 * H, W_hh0.data_ptr(),
                      b_ih1.data_ptr(), b_hh1.data_ptr(), W_ih1.data_ptr(), W_hh1.data_ptr(), h0.data_ptr(),
                      c0.data_ptr(), _p(g0), h1.data_ptr(), c1.data_ptr(), _p(g1), _s())
        ctx.save_for_backward(x, W_ih0, W_hh0, h0, c0, g0, W_ih1, W_hh1, h1, c1, g1)
        ctx.params = ((W_ih0, W_hh0, b_ih0, b_hh0), (W_ih1, W_hh1, b_ih1, b_hh1))
        return h1

    @staticmethod
    def backward(ctx, dh1):
        x, W_ih0, W_hh0, h0, c0, g0, W_ih1, W_hh1, h1, c1, g1 = ctx.saved_tensors
        n = ctx.needs_input_grad
        need0 = (n[0],) + tuple(n[1:5])
        need1 = (any(need0),) + tuple(n[5:9])
        H = W_hh0.shape[1]
        if (any(need0) and g0 is not None and g1 is not None
                and os.environ.get("AVC_LSTM2_BWD", "1") != "0" and H % 64 == 0):
            return LSTM2StackFn._backward_stacked(ctx, dh1, need0, need1)
        dh0, *grads1 = _lstm_layer_backward(dh1, h0, W_ih1, W_hh1, h1, c1, g1, ctx.params[1], need1)
        if dh0 is None:
            grads0 = [None] * 5
        else:
            grads0 = _lstm_layer_backward(dh0, x, W_ih0, W_hh0, h0, c0, g0, ctx.params[0], need0)
        return (grads0[0], *grads0[1:], *grads1, None)

    @staticmethod
    def _backward_stacked(ctx, dh1, need0, need1):
        """Both recurrences as one backward wavefront (autovc_lstm2_bwd_f32): layer 0 runs
        one step behind layer 1, and layer 1's input gradient dG1 W_ih1 is computed inside
        its steps instead of by a GEMM over all frames between the two recurrences."""
        x, W_ih0, W_hh0, h0, c0, g0, W_ih1, W_hh1, h1, c1, g1 = ctx.saved_tensors
        dh1 = dh1.contiguous()
        B, T, _ = x.shape
        H = W_hh0.shape[1]
        dev = x.device
        # split-K of the stacked backward products (autovc_lstm2_bwd_f32): 4 / 2 = 32 x 32 tiles;
        # 8 = the wide-tile kernel (64 x 64 per workgroup), measured slower (fp32 23.5 vs 20.0 us
        # per launch, 15.87 vs 15.49 ms/step; bf16 9.6 vs 9.46 ms/step:
        # profiles/r03/ab_lstm2_bwd_wide.txt); AVC_LSTM2_SPLITS overrides
        kdim = 2 * H if _bf16_rec(H) else 4 * H
        splits = {8: 8, 4: 4}.get(int(os.environ.get("AVC_LSTM2_SPLITS", "4")), 2)
        while splits > 2 and (kdim % (64 * splits) or (splits == 8 and H % 64)):
            splits //= 2
        dG1 = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32)
        dG0 = torch.empty((B, T, 4 * H), device=dev, dtype=torch.float32)
        # the (H, 4H) transposes (bf16 copies under bf16), from the step's weight scope if any
        kt = 8 if _bf16_rec(H) else 7
        WT1, WIT1, WT0 = conv_weight(W_hh1, kt), conv_weight(W_ih1, kt), conv_weight(W_hh0, kt)
        ws = _ws(dev, 4 * _lib.load().autovc_lstm2_bwd_workspace_floats(B, H, splits), "lstm")
        bf = _bf16_rec(H)
        if bf:
            dG1b, dG0b = (torch.empty((B, T, 4 * H), device=dev, dtype=torch.bfloat16) for _ in range(2))

        mark = _grad_mark(dev)   # queued weight gradients run beside the recurrences
        if bf:
            _lib.call("autovc_lstm2_bwd_bf16", B, T, H, dh1.data_ptr(), T * H, H, g1.data_ptr(),
                      c1.data_ptr(), g0.data_ptr(), c0.data_ptr(), WT1.data_ptr(), WIT1.data_ptr(),
                      WT0.data_ptr(), dG1.data_ptr(), dG1b.data_ptr(), dG0.data_ptr(), dG0b.data_ptr(), splits,
                      ws, _s())
        else:
            _lib.call("autovc_lstm2_bwd_f32", B, T, H, dh1.data_ptr(), T * H, H, g1.data_ptr(),
                      c1.data_ptr(), g0.data_ptr(), c0.data_ptr(), WT1.data_ptr(), WIT1.data_ptr(),
                      WT0.data_ptr(), dG1.data_ptr(), dG0.data_ptr(), splits, ws, _s())
        _flush_grad_queue(after=mark)
        grads1 = _lstm_grads_from_dG(dG1, h0, W_ih1, h1, ctx.params[1], (False,) + tuple(need1[1:]),
                                     dGb=dG1b if bf else None)
        grads0 = _lstm_grads_from_dG(dG0, x, W_ih0, h0, ctx.params[0], need0, dGb=dG0b if bf else None)
        return (grads0[0], *grads0[1:], *grads1[1:], None)


# The persistent decoder-lstm2 backward (lstm2_bwd_persist_kernel: 28.9 vs 24.4 us per
# wavefront step fp32, 21.0 vs 14.8 bf16, profiles/r04/lstm2_bwd_persist_time.txt) is retired to
# tools/retired/ (round 5): its per-step K-slice reduction, hand-off and grid barrier cost more
# than the launch boundary it saves.


# the BLSTM weight/bias gradients on the side stream (bench, alternating, one box): bf16 all of
# them (mode 1: 8.03-8.04 vs 8.29-8.30 ms/step on the main stream; 7.98-8.00 vs 8.01-8.03 for
# mode 2); fp32 all but the last-differentiated pass's (mode 2: 14.00-14.02 vs 14.22-14.32 on
# the main stream; mode 1 14.46, where the side stream's tail then runs past the backward).
# profiles/r05/ab_blstm_side.txt, ab_blstm_side2.txt.  Round 6, with the XCD-local lstm1 backward
# and its weight gradients on the main stream, bf16 too is better in mode 2: 7.64-7.69 vs
# 7.72-7.74 (profiles/r06/ab_bf16_blstm_side_r06.txt).  AVC_BLSTM_SIDE=0 / 1 / 2 forces a mode
_BLSTM_SIDE_ENV = os.environ.get("AVC_BLSTM_SIDE")


_BLSTM_LAST_PASS = [False]   # set around the encoder pass whose backward ends the step
# the last-differentiated encoder pass's conv weight gradients on the main stream, as they are
# produced, instead of as the final side batch that runs alone after the join: bf16 7.90-7.93
# vs 7.96-7.97 ms/step, fp32 neutral (14.13 vs 14.11-14.16; profiles/r05/ab_last_conv_main.txt).
# AVC_LAST_CONV_MAIN=1 / 0 forces it; the default follows the precision
_LAST_CONV_MAIN_ENV = os.environ.get("AVC_LAST_CONV_MAIN")


def _last_conv_main():
    if _LAST_CONV_MAIN_ENV is not None:
        return _LAST_CONV_MAIN_ENV == "1"
    return _PRECISION[0] == "bf16"


@contextlib.contextmanager
def blstm_last_pass(flag=True):
    """Mark the BLSTM layers run inside the block as the ones whose backward comes last (the
    Generator's full pass: its encoder is differentiated after the code-only second pass's).
    Their weight gradients then stay on the main stream when AVC_BLSTM_SIDE=2: queued there
    they would only lengthen the side stream's tail past the end of the backward."""
    prev = _BLSTM_LAST_PASS[0]
    _BLSTM_LAST_PASS[0] = flag
    try:
        yield
    finally:
        _BLSTM_LAST_PASS[0] = prev


def _blstm_side(last_pass):
    mode = _BLSTM_SIDE_ENV if _BLSTM_SIDE_ENV is not None else "2"
    return mode == "1" or (mode == "2" and not last_pass)


class BLSTMLayerFn(torch.autograd.Function):
    """One bidirectional nn.LSTM layer with H=32 (encoder, model_vc_mel.py:61)."""

    @staticmethod
    def forward(ctx, x, Wih_f, Whh_f, bih_f, bhh_f, Wih_b, Whh_b, bih_b, bhh_b, save):
        _check(x, "blstm")
        x = x.contiguous()
        B, T, I = x.shape
        H = Whh_f.shape[1]
        G = 4 * H
        dev = x.device
        gx = torch.empty((B, T, 2 * G), device=dev, dtype=torch.float32)
        # both directions' projections as one GEMM over [W_ih_f; W_ih_b] (same sums; one 8192 x 256
        # output instead of two 128-column ones: bf16 -0.07, fp32 -0.01 ms/step,
        # profiles/r05/ab_bf16src_blstm_cat.txt), reused by the backward's dx
        Wcat = _cat_scoped(Wih_f, Wih_b)
        gemm(B * T, 2 * G, I, x, I, 0, Wcat, I, 0, gx, 2 * G, bias1=_cat_scoped(bih_f, bih_b),
             bias2=_cat_scoped(bhh_f, bhh_b))
        h = torch.empty((B, T, 2 * H), device=dev, dtype=torch.float32)
        c = torch.empty((B, T, 2 * H), device=dev, dtype=torch.float32)
        gates = torch.empty((B, T, 2 * G), device=dev, dtype=torch.float32) if save else None
        _lib.call("autovc_blstm_fwd_f32", B, T, H, 2, gx.data_ptr(), Whh_f.data_ptr(), Whh_b.data_ptr(),
                  h.data_ptr(), c.data_ptr(), _p(gates), _s())
        ctx.save_for_backward(x, Wih_f, Whh_f, Wih_b, Whh_b, h, c, gates, Wcat)
        ctx.params = ((Wih_f, Whh_f, bih_f, bhh_f), (Wih_b, Whh_b, bih_b, bhh_b))
        ctx.last_pass = _BLSTM_LAST_PASS[0]
        return h

    @staticmethod
    def backward(ctx, dh):
        x, Wih_f, Whh_f, Wih_b, Whh_b, h, c, gates, Wcat = ctx.saved_tensors
        if gates is None:
            raise RuntimeError("BLSTM backward needs the forward run with gradients enabled")
        dh = dh.contiguous()
        B, T, I = x.shape
        H = Whh_f.shape[1]
        G = 4 * H
        M = B * T
        dev = x.device
        dG = torch.empty((B, T, 2 * G), device=dev, dtype=torch.float32)
        mark = _grad_mark(dev)   # queued weight gradients run beside this latency-bound recurrence
        _lib.call("autovc_blstm_bwd_f32", B, T, H, 2, dh.data_ptr(), gates.data_ptr(), c.data_ptr(),
                  Whh_f.data_ptr(), Whh_b.data_ptr(), dG.data_ptr(), _s())
        _flush_grad_queue(after=mark)
        grads = [None] * 10
        dG2 = dG.view(M, 2 * G)
        # under bf16 the weight / bias gradients go to the side stream like the large LSTMs'
        # (_grad_launch, released beside the next recurrence; _blstm_side)
        launch = _grad_launch if _blstm_side(ctx.last_pass) else _main_grad
        for d, (iW, iH, iBi, iBh) in enumerate(((1, 2, 3, 4), (5, 6, 7, 8))):
            pW, pH, pBi, pBh = ctx.params[d]
            if ctx.needs_input_grad[iW]:
                go = _GradOut(pW, pW.shape, dev)
                launch(dev, go, lambda go=go, d=d: gemm(G, I, M, dG, 2 * G, 1, x, I, 1, go.buf, I, a_off=d * G,
                                                        splits=_splits_for(G, I, M), accumulate=go.acc), dG, x)
                grads[iW] = go.result()
            if ctx.needs_input_grad[iH]:
                go = _GradOut(pH, pH.shape, dev)
                # previous step in processing order: t-1 forward, t+1 backward direction
                launch(dev, go, lambda go=go, d=d: gemm(G, H, M, dG, 2 * G, 1, h, 2 * H, 1, go.buf, H, a_off=d * G,
                                                        b_off=d * H, b_conv=(T, H, -1 if d == 0 else 1),
                                                        splits=_splits_for(G, H, M), accumulate=go.acc), dG, h)
                grads[iH] = go.result()
            if ctx.needs_input_grad[iBi] or ctx.needs_input_grad[iBh]:
                gi, gh = _bias_outs(pBi, pBh, (G,), dev)
                launch(dev, (gi, gh), lambda gi=gi, gh=gh, d=d: colsum(dG2[:, d * G:(d + 1) * G], gi.buf, gh.buf,
                                                                        accumulate=gi.acc), dG)
                grads[iBi], grads[iBh] = gi.result(), gh.result()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            # dx = [dG_f dG_b] [W_ih_f; W_ih_b]: one K = 2G GEMM, no accumulate pass
            gemm(M, I, 2 * G, dG, 2 * G, 0, Wcat, I, 1, dx, I)
        grads[0] = dx
        return tuple(grads)


# ---------------------------------------------------------------- glue / bottleneck
class FrameConcatFn(torch.autograd.Function):
    """out[b, t] = [X[b, t // rep], E[b]]  (model_vc_mel.py:64-66 with rep=1; :186-192)."""

    @staticmethod
    def forward(ctx, X, E, T, rep):
        X = X.contiguous()
        E = E.contiguous()
        B = E.shape[0]
        C1 = X.shape[-1]
        C2 = E.shape[-1]
        out = torch.empty((B, T, C1 + C2), device=X.device, dtype=torch.float32)
        _lib.call("autovc_frame_concat_f32", B, T, C1, C2, rep, X.data_ptr(), C1, E.data_ptr(),
                  out.data_ptr(), _s())
        ctx.dims = (B, T, C1, C2, rep)
        ctx.xshape = X.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        B, T, C1, C2, rep = ctx.dims
        dout = dout.contiguous()
        dX = torch.empty(ctx.xshape, device=dout.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        dE = torch.empty((B, C2), device=dout.device, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        if dX is not None or dE is not None:
            _lib.call("autovc_frame_concat_bwd_f32", B, T, C1, C2, rep, dout.data_ptr(), _p(dX), C1, _p(dE),
                      0, _s())
        return dX, dE, None, None


class CodeGatherFn(torch.autograd.Function):
    """codes = cat_k [h_fwd[:, k*freq + freq-1], h_bwd[:, k*freq]] (model_vc_mel.py:74-79)."""

    @staticmethod
    def forward(ctx, h, freq):
        h = h.contiguous()
        B, T, D2 = h.shape
        if T % freq != 0:
            # the reference indexes out_forward[:, i+freq-1] past the end -> IndexError (F11)
            raise IndexError(f"index {T // freq * freq + freq - 1} is out of bounds for dimension 1 "
                             f"with size {T} (T must be a multiple of freq={freq})")
        codes = torch.empty((B, (T // freq) * D2), device=h.device, dtype=torch.float32)
        _lib.call("autovc_code_gather_f32", B, T, D2 // 2, freq, h.data_ptr(), codes.data_ptr(), _s())
        ctx.dims = (B, T, D2 // 2, freq)
        return codes

    @staticmethod
    def backward(ctx, dcodes):
        B, T, D, freq = ctx.dims
        dh = torch.empty((B, T, 2 * D), device=dcodes.device, dtype=torch.float32)
        _lib.call("autovc_code_gather_bwd_f32", B, T, D, freq, dcodes.contiguous().data_ptr(), dh.data_ptr(),
                  _s())
        return dh, None


# ---------------------------------------------------------------- losses
class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, kind):
        _check(a, "loss")
        a = a.contiguous()
        b = b.contiguous()
        if a.numel() != b.numel():
            raise ValueError(f"loss: size mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
        out = torch.empty((), device=a.device, dtype=torch.float32)
        ws = _ws(a.device, _lib.load().autovc_loss_workspace_bytes(), "loss")
        _lib.call("autovc_loss_f32", kind, a.numel(), a.data_ptr(), b.data_ptr(), out.data_ptr(), ws, _s())
        ctx.kind = kind
        ctx.save_for_backward(a, b)
        ctx.shapes = (a.shape, b.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(b) if ctx.needs_input_grad[1] else None
        if ga is not None or gb is not None:
            _lib.call("autovc_loss_bwd_f32", ctx.kind, a.numel(), a.data_ptr(), b.data_ptr(), g.data_ptr(),
                      _p(ga), _p(gb), 0, 0, _s())
        return ga, gb, None


def mse_loss(a, b):
    """F.mse_loss(a, b) (mean) for equal-numel tensors (solver_encoder.py:230,233)."""
    return _LossFn.apply(a, b, 0)


def l1_loss(a, b):
    """F.l1_loss(a, b) (mean) (solver_encoder.py:236)."""
    return _LossFn.apply(a, b, 1)
