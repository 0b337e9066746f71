"""The real data-parallel path on the GPU: two fresh processes on cuda:0, backend gloo
(RCCL refuses two ranks on one device; gloo reduces device tensors through the host), each
running bench.make_solver + ddp.make_data_parallel with the captured HIP-graph step, the
bucketed all-reduce interleaved with the per-bucket FusedAdam update (ddp.reduce_and_step).

Checked against ONE process that computes both ranks' gradients at the same parameters,
applies their mean and steps Adam: bit-identical parameters after 2 steps (a sum of two
floats is commutative, x 0.5 is exact, every kernel is deterministic and the graph replay
is bit-identical to eager, tests/test_solver_gpu.py).  The bf16 exchange (config 3) is
checked against the same reference within bf16 rounding of the mean gradient."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

B = 8
STEPS = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, grad_dtype, overlap):
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from autovc_amd import ddp
    torch.manual_seed(0)
    solver = bench.make_solver(dev, B)
    solver.G.train()
    solver.hip_graph = True
    ddp.make_data_parallel(solver, bucket_bytes=4 << 20, overlap=overlap,
                           grad_dtype=None if grad_dtype == "fp32" else torch.bfloat16)
    x, e = bench.synthetic_batch(B, 128, dev, 500 + 7 * rank)
    for _ in range(STEPS):
        solver.train_step(x, e)
    torch.cuda.synchronize()
    torch.save([f.cpu() for f in solver.g_optimizer.flat_params()], os.path.join(out_dir, f"rank{rank}.pt"))
    torch.save([r for _, r in ddp.last_schedule], os.path.join(out_dir, f"sched{rank}.pt"))
    torch.save(torch.tensor([ddp.comm_joins]), os.path.join(out_dir, f"joins{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(tmp_path, grad_dtype, overlap):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), grad_dtype, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0, p.exitcode
    _run_ranks.schedule = torch.load(os.path.join(tmp_path, "sched0.pt"), weights_only=True)
    _run_ranks.joins = [int(torch.load(os.path.join(tmp_path, f"joins{r}.pt"), weights_only=True)) for r in range(2)]
    return [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(2)]


def _reference(cuda):
    """One process: both ranks' gradients at the same parameters, their mean, Adam."""
    import bench
    torch.manual_seed(0)
    solver = bench.make_solver(cuda, B)
    solver.G.train()
    batches = [bench.synthetic_batch(B, 128, cuda, 500 + 7 * r) for r in range(2)]
    flat_g = solver.g_optimizer.flat_grads()
    for _ in range(STEPS):
        grads = []
        for x, e in batches:
            solver._forward_backward(x, e)
            grads.append([g.clone() for g in flat_g])
        for g, g0, g1 in zip(flat_g, *grads):
            g.copy_((g0 + g1) * 0.5)
        solver.g_optimizer.step()
    torch.cuda.synchronize()
    return [f.cpu() for f in solver.g_optimizer.flat_params()]


@pytest.mark.parametrize("overlap", [True, False])
def test_two_rank_graph_step_equals_mean_gradient_step(cuda, tmp_path, overlap):
    """overlap=True: each bucket's collective waits only for its gradient-ready mark inside
    the replayed backward (functional.GradMarks); the buckets of the late layers must be
    gated on an earlier mark than the encoder's, which is final only at the end."""
    ranks = _run_ranks(tmp_path, "fp32", overlap)
    if overlap:
        sched = _run_ranks.schedule
        assert sched == sorted(sched) and len(set(sched)) >= 2 and sched[0] < sched[-1], sched
        # every overlapped step ends with the explicit compute-stream wait on the communication
        # stream (the next replay's persistent kernels never share the device with a collective)
        assert _run_ranks.joins == [STEPS, STEPS], _run_ranks.joins
    ref = _reference(cuda)
    for a, b in zip(ranks[0], ranks[1]):
        assert torch.equal(a, b)                     # the ranks stay in lockstep
    for a, r in zip(ranks[0], ref):
        assert torch.equal(a, r), (a - r).abs().max().item()


def test_two_rank_bf16_gradient_exchange(cuda, tmp_path):
    ranks = _run_ranks(tmp_path, "bf16", True)
    ref = _reference(cuda)
    for a, b in zip(ranks[0], ranks[1]):
        assert torch.equal(a, b)
    # Adam moves each parameter by ~lr per step whatever the gradient's scale; a bf16-rounded
    # mean gradient can flip only the update of near-zero gradients: bound 2 x lr x steps
    for a, r in zip(ranks[0], ref):
        assert (a - r).abs().max().item() <= 2 * 1e-4 * STEPS + 1e-7
