"""What-if timing of the training step (tools only, results are WRONG by design): the same
B=64 graph-replayed step with a class of kernels skipped, to price how much of the step a
faster version of that class could save.  python tools/step_whatif.py [fp32|bf16]
  default      the product step
  no_lstm_dw   LSTM weight-gradient GEMMs (W_ih, W_hh) skipped
  no_conv_dw   conv weight-gradient GEMMs (Conv-BN stacks) skipped
  no_side      every queued weight-gradient launch skipped"""
import contextlib
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from autovc_amd import functional as AF  # noqa: E402


def run(prec, variant, steps=20, warm=5):
    orig_launch = AF._grad_launch
    orig_gemm = AF.gemm

    def launch(dev, outs, fn, *inputs):
        if variant == "no_side":
            return
        return orig_launch(dev, outs, fn, *inputs)

    def gemm(M, N, K, *a, **k):
        # the LSTM dW GEMMs: M = 4H rows, K = B*T, both operands transposed
        if variant == "no_lstm_dw" and M in (4096, 2048) and K == 8192 and a[2] == 1 and a[5] == 1:
            return
        return orig_gemm(M, N, K, *a, **k)
    AF._grad_launch = launch
    AF.gemm = gemm
    if variant == "no_conv_dw":
        os.environ["AVC_WHATIF_NO_CONV_DW"] = "1"
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        with contextlib.redirect_stdout(sys.stderr):
            s = bench.make_solver(dev, 64)
        s.G.train()
        s.precision = prec
        s.hip_graph = True
        x, e = bench.synthetic_batch(64, 128, dev, 1234)
        for _ in range(warm):
            s.train_step(x, e)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            s.train_step(x, e)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3
    finally:
        AF._grad_launch = orig_launch
        AF.gemm = orig_gemm
        os.environ.pop("AVC_WHATIF_NO_CONV_DW", None)


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    for v in ("default", "no_lstm_dw", "no_side", "default"):
        print(f"{prec} {v:12s} {run(prec, v):7.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
