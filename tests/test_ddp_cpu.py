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
    q.put((rank, opt.g[0].clone()))
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
        assert torch.equal(got, expected), f"rank {rank}"
        err = (got.double() - exact).abs()
        bound = 2 * 2.0 ** -8 * torch.stack([_rank_grads(r).double().abs() for r in range(world)]).max(0).values
        assert bool((err <= bound + 1e-30).all()), float((err - bound).max())
