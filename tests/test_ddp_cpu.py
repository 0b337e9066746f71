"""Data-parallel logic (autovc_amd.ddp) on CPU with the gloo backend: bucketed all-reduce
(mean) of the flat gradient buffers and rank-0 parameter broadcast (world 2), and the bf16
exchange with fp32 accumulation (worlds 2, 4 and 8: the result is the same two roundings
whatever the world size)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pytest


class _FlatOpt:
    def __init__(self, rank):
        self.g = [torch.full((1000,), float(rank + 1)), torch.arange(37, dtype=torch.float32) * (rank + 1)]
        self.p = [torch.full((50,), float(10 * (rank + 1)))]

    def flat_grads(self):
        return self.g

    def flat_params(self):
        return self.p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from autovc_amd import ddp
    opt = _FlatOpt(rank)
    ddp.allreduce_gradients(opt, bucket_bytes=4 * 96)  # several buckets incl. a ragged tail
    ddp.broadcast_parameters(opt)
    q.put((rank, opt.g[0][:3].tolist(), opt.g[1][-1].item(), opt.p[0][0].item()))
    dist.barrier()
    dist.destroy_process_group()


def _rank_grads(rank, n=5003):
    g = torch.Generator().manual_seed(100 + rank)
    return (torch.randn(n, generator=g) * (rank + 1)).float()


def _bf16_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from autovc_amd import ddp
    opt = _FlatOpt(rank)
    opt.g = [_rank_grads(rank)]
    ddp.allreduce_gradients(opt, bucket_bytes=4 * 1000, grad_dtype=torch.bfloat16)  # ragged tail bucket
    q.put((rank, opt.g[0].clone().numpy()))  # numpy: pickled by value, no fd hand-off
    dist.barrier()
    dist.destroy_process_group()


def _run(target, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_allreduce_and_broadcast_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, g0, glast, p0 in res:
        assert g0 == [1.5, 1.5, 1.5]          # mean of 1 and 2
        assert abs(glast - 36 * 1.5) < 1e-6   # mean of 36*1 and 36*2
        assert p0 == 10.0                     # rank 0's parameters everywhere


def test_init_from_env_single_process():
    from autovc_amd import ddp
    os.environ.pop("WORLD_SIZE", None)
    assert ddp.init_from_env() == (0, 1)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bf16_exchange_fp32_accumulate(world):
    """Every rank ends with the same buffer, equal to: each rank's gradient rounded to bf16
    once, summed in fp32 in rank order, x 1/N, rounded to bf16 once — not a bf16 sum per
    ring hop.  Its error against the exact mean stays within two bf16 roundings
    at every world size."""
    res = _run(_bf16_worker, world)
    parts = [_rank_grads(r).bfloat16().float() for r in range(world)]
    acc = parts[0].clone()
    for p in parts[1:]:
        acc.add_(p)
    expected = acc.mul_(1.0 / world).bfloat16().float()
    exact = torch.stack([_rank_grads(r).double() for r in range(world)]).mean(0)
    for rank, got in res:
        got = torch.from_numpy(got)
        assert torch.equal(got, expected), f"rank {rank}"
        err = (got.double() - exact).abs()
        bound = 2 * 2.0 ** -8 * torch.stack([_rank_grads(r).double().abs() for r in range(world)]).max(0).values
        assert bool((err <= bound + 1e-30).all()), float((err - bound).max())


class _FakeMarks:
    """GradMarks stand-in for host tensors: fixed ready marks per flat-buffer range, and a log
    of the gates the exchange waited on (in issue order)."""

    def __init__(self, flat, cuts):
        self.n = len(cuts) + 1
        self.flat = flat
        self.cuts = cuts            # element offsets where the ready mark changes
        self.waited = []

    def ready_mark(self, ptr, nbytes):
        start = (ptr - self.flat.data_ptr()) // 4
        end = start + nbytes // 4
        # later ranges of the flat buffer are final earlier (the backward runs the model in
        # reverse): mark 1 for the tail, the last mark for the head
        return max(self.n - sum(1 for c in self.cuts if e > c) for e in range(start, end, max(1, (end - start) // 8)))

    def wait(self, stream, k):
        self.waited.append(k)


class _AdamLog:
    """FusedAdam stand-in: one flat group, update_range records the issue order."""

    def __init__(self, g):
        self._flat = [dict(g=g, p=torch.zeros_like(g))]
        self.updates = []

    def begin_step(self):
        pass

    def update_range(self, gi, s, c):
        self.updates.append(s)


def _marked_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from autovc_amd import ddp
    out = {}
    for dtype in (None, torch.bfloat16):
        plain = _AdamLog(_rank_grads(rank, 40003))
        ddp.reduce_and_step(plain, bucket_bytes=4 * 4000, grad_dtype=dtype)
        marked = _AdamLog(_rank_grads(rank, 40003))
        marks = _FakeMarks(marked._flat[0]["g"], cuts=[12000, 30000])
        ddp.reduce_and_step(marked, bucket_bytes=4 * 4000, grad_dtype=dtype, marks=marks)
        out[str(dtype)] = (plain._flat[0]["g"].clone().numpy(), marked._flat[0]["g"].clone().numpy(), marks.waited,
                           marked.updates, list(ddp.last_schedule))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_marked_exchange_equals_plain_gloo_world2():
    """The exchange gated by gradient-ready marks (buckets issued in mark order, each after
    its own gate; the overlap with the backward on the GPU) gives the same means, bit for
    bit, as the plain exchange, for the fp32 and the bf16 exchange; buckets final earlier
    (the flat buffer's tail) are issued and updated first."""
    res = _run(_marked_worker, 2)
    for rank, out in res:
        for dtype, (plain, marked, waited, updates, sched) in out.items():
            assert (plain == marked).all() and plain.shape == marked.shape, (rank, dtype)
            assert waited == sorted(waited) and waited[0] == 1 and waited[-1] == 3, waited
            assert updates[0] > updates[-1]                  # tail bucket first, head bucket last
            assert [r for _, r in sched] == waited
