"""bench.py's N > 1 flow (torchrun ranks, gradient all-reduce, barrier + max-over-ranks timing,
rank-0 JSON line) on a 1-GPU box: two ranks share cuda:0 over gloo (AVC_BENCH_SHARE_DEVICE=1).
The driver's 8-GPU run takes the same path with RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_json_line():
    env = dict(os.environ, AVC_BENCH_SHARE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--no-wavenet", "--no-e2e", "--no-cpu-baseline", "--no-roofline", "--no-bf16"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 128
    assert d["value"] > 0 and d["steps"] == 2 and d["scaling"] == "weak"
    # self-validating multi-rank line: the process group's own backend and size, every rank's
    # time, and the value computed from the slowest rank
    assert d["dist_backend"] == "gloo" and d["world_size"] == 2 and len(d["rank_ms_per_step"]) == 2
    assert abs(d["ms_per_step"] - max(d["rank_ms_per_step"])) < 1e-2


def test_plain_bench_gpus2_spawns_two_ranks():
    """`python bench.py --gpus 2` (no torchrun around it, the driver's command shape) starts
    its two ranks itself and reports them; the bf16 object runs with the bf16 gradient
    exchange (all-to-all + fp32 shard sums + all-gather)."""
    env = dict(os.environ, AVC_BENCH_SHARE_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "2", "--no-wavenet", "--no-e2e",
           "--no-cpu-baseline", "--no-roofline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 128
    assert d["value"] > 0 and d["bf16"]["value"] > 0
    assert d["bf16"]["grad_exchange"].startswith("bf16")
    assert d["final_loss"] == d["final_loss"] and d["bf16"]["final_loss"] == d["bf16"]["final_loss"]   # not NaN
