"""Data parallelism for the Generator step: one process per GPU, torch.distributed with
backend "nccl" (= RCCL on ROCm) over xGMI.

The reference has no distributed code; the build shards utterances (crops)
across ranks, keeps per-rank BatchNorm statistics (the reference semantics at B=64/GPU),
and adds the one real exchange of the step: an all-reduce (mean) of the gradients.
Because FusedAdam keeps every gradient in ONE contiguous buffer, the exchange is a few
bucketed collectives over that buffer (no per-parameter calls).

Overlap with the backward: while the exchange is attached (world > 1), the backward records
gradient-ready marks (functional.GradMarks): an event at every recurrence and at the final
join, each flat-buffer gradient logged with the mark after which it is final.  The step's
forward+backward is one captured HIP graph (autovc_amd.graph) whose marks are event-record
nodes, so the collectives stay OUT of the graph (eager RCCL, never captured) and still start
inside the backward: after the replay is enqueued, `reduce_and_step` issues every bucket's
collective on a communication stream that first waits for that bucket's mark — the buckets
of postnet / linear / lstm2 / decoder convs (about 80 % of the bytes) become final when
lstm1's backward recurrence releases their weight-gradient GEMMs, and their exchange runs
beside the rest of the backward (lstm1, the encoder BLSTMs and convs, the side stream's
remaining GEMMs).  Each bucket's Adam update is queued on the compute stream as its mean
lands.  Without marks (overlap=False or a recording off) every collective waits for the whole
backward, as before.

Exchange precision: fp32 (113.7 MB per step, one ring all-reduce per bucket) or bf16
(BASELINE config 3) with fp32 accumulation: each rank rounds its bucket to
bf16 once, an all-to-all hands rank r the r-th shard of every rank's bucket, rank r sums
those N shards in fp32 in rank order (deterministic, identical on every rank) and scales
by 1/N, and an all-gather returns the mean rounded to bf16 once.  Two roundings whatever
N is (a bf16 ring all-reduce would round at every one of its N-1 hops), and
(N-1)/N x 56.8 MB x 2 on the wire per rank instead of (N-1)/N x 113.7 MB x 2.
`make_data_parallel(grad_dtype="auto")` (the default) picks bf16 while the Solver runs
under precision "bf16" and fp32 otherwise.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 16 << 20
last_schedule: list = []      # (bucket key, gradient-ready mark) of the last overlapped step, in issue order
comm_joins = 0                # explicit compute-stream waits on the communication stream (one per step)


def init_from_env(backend=None):
    """Initialise the default process group from RANK / WORLD_SIZE / MASTER_* (torchrun)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    if backend is None:
        # AVC_DIST_BACKEND: test hook (gloo ranks sharing one GPU of a 1-GPU box)
        backend = os.environ.get("AVC_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def _world():
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size()


def broadcast_parameters(optimizer, src=0):
    """Rank src's parameters (and nothing else) to every rank: one collective per flat buffer."""
    if _world() == 1:
        return
    for flat in optimizer.flat_params():
        dist.broadcast(flat, src)


def _buckets(n, bucket_bytes):
    nb = max(4, (bucket_bytes // 4) // 4 * 4)   # multiples of 4 floats: 16-byte aligned slices
    return [(s, min(nb, n - s)) for s in range(0, n, nb)]


class _Bf16Mean:
    """Mean of one fp32 bucket over the ranks, exchanged as bf16 and accumulated in fp32
    (module docstring).  issue() starts the all-to-all, reduce() sums this rank's shard and
    starts the all-gather, finish() writes the mean back into the fp32 bucket."""

    def __init__(self, chunk, world):
        self.chunk, self.world = chunk, world
        n = chunk.numel()
        self.shard = (n + world - 1) // world
        self.shard = (self.shard + 7) // 8 * 8          # 16-byte aligned bf16 shards
        padded = self.shard * world
        self.send = torch.zeros(padded, dtype=torch.bfloat16, device=chunk.device)
        self.send[:n].copy_(chunk)
        self.recv = torch.empty_like(self.send)
        self.work = dist.all_to_all_single(self.recv, self.send, async_op=True)

    def reduce(self):
        self.work.wait()
        parts = self.recv.view(self.world, self.shard)
        acc = parts[0].float()
        for r in range(1, self.world):                  # fixed rank order
            acc.add_(parts[r].float())
        mine = acc.mul_(1.0 / self.world).to(torch.bfloat16)
        self.gathered = torch.empty_like(self.send)
        self.work = dist.all_gather_into_tensor(self.gathered, mine, async_op=True)

    def finish(self):
        self.work.wait()
        self.chunk.copy_(self.gathered[:self.chunk.numel()])
        if self.chunk.is_cuda:   # buffers from the communication stream, read on this one
            for t in (self.send, self.recv, self.gathered):
                t.record_stream(torch.cuda.current_stream(self.chunk.device))


class _Fp32Mean:
    """Mean of one fp32 bucket: one all-reduce (sum) in place, then x 1/N."""

    def __init__(self, chunk, world):
        self.chunk, self.world = chunk, world
        self.work = dist.all_reduce(chunk, op=dist.ReduceOp.SUM, async_op=True)

    def reduce(self):
        pass

    def finish(self):
        self.work.wait()
        self.chunk.mul_(1.0 / self.world)


def _exchange(grad_dtype):
    if grad_dtype is None or grad_dtype == torch.float32:
        return _Fp32Mean
    if grad_dtype == torch.bfloat16:
        return _Bf16Mean
    raise ValueError(f"gradient exchange dtype must be float32 or bfloat16, got {grad_dtype}")


_COMM_STREAMS: dict = {}


def _comm_stream(dev):
    st = _COMM_STREAMS.get(dev.index)
    if st is None:
        st = torch.cuda.Stream(dev)
        _COMM_STREAMS[dev.index] = st
    return st


def _run_exchange(items, grad_dtype, world, after=None, gates=None):
    """items: (key, fp32 chunk) pairs.  Every bucket's first collective is issued before
    any is waited on; `after(key)` runs as each bucket's mean lands (the Adam slice).
    gates (CUDA only): key -> callable(stream_ptr) that makes the communication stream wait
    until the bucket's gradients are final (functional.GradMarks.wait); the collectives and
    the bf16 shard sums are then issued on that stream in gate order (bucket i's shard sum
    before bucket i+1's gate), and only the compute stream's finish (mean / copy back, Adam)
    waits for them."""
    cls = _exchange(grad_dtype)
    if not gates:
        ex = [(k, cls(chunk, world)) for k, chunk in items]
        for _, e in ex:
            e.reduce()
        for k, e in ex:
            e.finish()
            if after is not None:
                after(k)
        return
    dev = items[0][1].device
    if dev.type != "cuda":        # host tensors (tests): the gates only order the issue
        ex = []
        for k, chunk in items:
            gates[k](None)
            ex.append((k, cls(chunk, world)))
        for _, e in ex:
            e.reduce()
        for k, e in ex:
            e.finish()
            if after is not None:
                after(k)
        return
    comm = _comm_stream(dev)
    # no wait on the compute stream as a whole (that would wait for the entire backward): each
    # bucket's gate is an event recorded after the bucket's last gradient write of this step,
    # which the compute stream issued after everything earlier that touched the bucket (the
    # previous step's Adam and copy-back, this step's zero_grad)
    # bucket i's second phase (the bf16 shard sum + all-gather) is issued before bucket i+1's
    # gate wait, so it runs as soon as its own exchange lands instead of behind every gate
    ex = []
    with torch.cuda.stream(comm):
        for k, chunk in items:
            if ex:
                ex[-1][1].reduce()
            gates[k](comm.cuda_stream)
            ex.append((k, cls(chunk, world)))
        if ex:
            ex[-1][1].reduce()
    for k, e in ex:
        e.finish()
        if after is not None:
            after(k)
    # An explicit join, not an accident of ordering: the compute stream waits for everything
    # issued on the communication stream (its RCCL kernels and bf16 shard sums) before the next
    # step's graph replay, whose persistent kernels need every CU of the device to themselves
    # (Co-residency) — an RCCL kernel still holding CUs would make their grid
    # barriers time out.
    torch.cuda.current_stream(dev).wait_stream(comm)
    global comm_joins
    comm_joins += 1


def allreduce_gradients(optimizer, bucket_bytes=DEFAULT_BUCKET_BYTES, grad_dtype=None):
    """Mean of the flat gradient buffers over all ranks, in buckets of bucket_bytes (all
    buckets in flight at once)."""
    world = _world()
    if world == 1:
        return
    from .functional import join_grad_stream   # weight gradients may still be in flight
    join_grad_stream()
    items = [(None, flat[s:s + c]) for flat in optimizer.flat_grads() for s, c in _buckets(flat.numel(), bucket_bytes)]
    _run_exchange(items, grad_dtype, world)


def reduce_and_step(optimizer, bucket_bytes=DEFAULT_BUCKET_BYTES, grad_dtype=None, marks=None):
    """All-reduce (mean) + Adam, bucket by bucket: every bucket's collective is issued up
    front; bucket i's update is queued on the compute stream once its collective is done,
    overlapping the collectives of the later buckets.  Identical arithmetic to
    allreduce_gradients() followed by optimizer.step() (Adam is elementwise).
    marks (functional.GradMarks of the step just issued): each bucket's collective waits
    only for its own gradient-ready mark, not for the whole backward, and buckets are issued
    in mark order."""
    world = _world()
    optimizer.begin_step()          # joins the gradient side stream first
    if world == 1:
        for gi, f in enumerate(optimizer._flat):
            if f is not None:
                optimizer.update_range(gi, 0, f["p"].numel())
        return
    items = [((gi, s, c), f["g"][s:s + c]) for gi, f in enumerate(optimizer._flat) if f is not None
             for s, c in _buckets(f["g"].numel(), bucket_bytes)]
    gates = None
    if marks is not None and marks.n > 0:
        ready = {k: marks.ready_mark(chunk.data_ptr(), chunk.numel() * 4) for k, chunk in items}
        items.sort(key=lambda kc: ready[kc[0]])
        gates = {k: (lambda sp, r=ready[k]: marks.wait(sp, r)) for k, _ in items}
        global last_schedule
        last_schedule = [(k, ready[k]) for k, _ in items]
    _run_exchange(items, grad_dtype, world, after=lambda k: optimizer.update_range(*k), gates=gates)


def make_data_parallel(solver, bucket_bytes=DEFAULT_BUCKET_BYTES, grad_dtype="auto", overlap=True):
    """Attach the gradient exchange to an autovc_amd Solver and sync its initial weights.
    overlap=True: reduce_and_step with the backward's gradient-ready marks (each bucket's
    collective starts inside the backward, interleaved with the Adam update);
    overlap=False: allreduce_gradients after backward, then one Adam launch.
    grad_dtype "auto": bf16 while solver.precision is "bf16" (BASELINE config 3), else fp32;
    or torch.float32 / torch.bfloat16 for a fixed exchange precision."""
    broadcast_parameters(solver.g_optimizer)

    def dtype():
        if grad_dtype == "auto":
            return torch.bfloat16 if getattr(solver, "precision", "fp32") == "bf16" else torch.float32
        return grad_dtype

    if overlap:
        from .functional import MARKS
        MARKS.active = bool(torch.cuda.is_available())
        solver._optimizer_step = lambda: reduce_and_step(solver.g_optimizer, bucket_bytes, dtype(),
                                                         marks=MARKS if MARKS.active else None)
    else:
        solver._after_backward = lambda: allreduce_gradients(solver.g_optimizer, bucket_bytes, dtype())
    solver._ddp_grad_dtype = dtype
    return solver
