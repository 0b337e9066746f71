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
