"""Data parallelism for the Generator step: one process per GPU, torch.distributed with
backend "nccl" (= RCCL on ROCm) over xGMI.

The reference has no distributed code; the build shards utterances (crops)
across ranks, keeps per-rank BatchNorm statistics (the reference semantics at B=64/GPU),
and adds the one real exchange of the step: an all-reduce (mean) of the gradients.
Because FusedAdam keeps every gradient in ONE contiguous buffer, the exchange is one
bucketed collective over that buffer (no per-parameter calls), issued after backward.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from RANK / WORLD_SIZE / MASTER_* (torchrun)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def broadcast_parameters(optimizer, src=0):
    """Rank src's parameters (and nothing else) to every rank: one collective per flat buffer."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    for flat in optimizer.flat_params():
        dist.broadcast(flat, src)


def allreduce_gradients(optimizer, bucket_bytes=64 << 20):
    """Mean of the flat gradient buffers over all ranks, in buckets of bucket_bytes."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size()
    if world == 1:
        return
    from .functional import join_grad_stream   # weight gradients may still be in flight
    join_grad_stream()
    nb = max(1, bucket_bytes // 4)
    for flat in optimizer.flat_grads():
        for s in range(0, flat.numel(), nb):
            chunk = flat[s:s + nb]
            dist.all_reduce(chunk, op=dist.ReduceOp.SUM)
            chunk.mul_(1.0 / world)


def make_data_parallel(solver):
    """Attach gradient all-reduce to an autovc_amd Solver and sync its initial weights."""
    broadcast_parameters(solver.g_optimizer)
    solver._after_backward = lambda: allreduce_gradients(solver.g_optimizer)
    return solver
