"""Data-parallel logic (autovc_amd.ddp) on CPU with the gloo backend, world_size 2:
bucketed all-reduce (mean) of the flat gradient buffers and rank-0 parameter broadcast."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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
