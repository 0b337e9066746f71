"""What-if timing of the training step (tools only, results are WRONG by design): the same
B=64 graph-replayed step with a class of kernels skipped, to price how much of the step a
faster version of that class could save.  python tools/step_whatif.py [fp32|bf16]
  default      the product step
  no_lstm_dw   LSTM weight-gradient GEMMs (W_ih, W_hh) skipped
  no_conv_dw   conv weight-gradient GEMMs (Conv-BN stacks) skipped
  no_side      every queued weight-gradient launch skipped
  blas_lstm_dw the LSTM weight-gradient GEMMs on torch.mm (hipBLASLt; the h_{t-1} shift and
               its first-frame mask ignored: the price of a library-speed GEMM there)
  blas_plain   additionally every unmasked GEMM (no conv view) on torch.mm
  short_lstm_dw the LSTM weight-gradient GEMMs over 70 % of their K (same kernels and footprint:
               the price of a 1.43x faster GEMM kernel there)
Variants: python tools/step_whatif.py fp32 default blas_lstm_dw ..."""
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

    def blas(M, N, K, A, lda, ta, B, ldb, tb, C, ldc, accumulate=False, a_off=0, b_off=0, c_off=0, bias1=None,
             bias2=None, **_):
        Am = A.reshape(-1)[a_off:].as_strided((K, M) if ta else (M, K), (lda, 1))
        Am = Am.t() if ta else Am
        Bm = B.reshape(-1)[b_off:].as_strided((K, N) if tb else (N, K), (ldb, 1))
        Bm = Bm if tb else Bm.t()
        Cm = C.reshape(-1)[c_off:].as_strided((M, N), (ldc, 1))
        if accumulate:
            Cm.addmm_(Am, Bm)
        else:
            Cm.copy_(Am @ Bm)
        for b in (bias1, bias2):
            if b is not None:
                Cm.add_(b[:N])

    def gemm(M, N, K, *a, **k):
        # the LSTM dW GEMMs: M = 4H rows, K = B*T, both operands transposed
        lstm_dw = M in (4096, 2048) and K == 8192 and a[2] == 1 and a[5] == 1
        if variant == "no_lstm_dw" and lstm_dw:
            return
        plain = not k.get("a_conv") and not k.get("b_conv")
        if variant == "short_lstm_dw" and lstm_dw:   # the same kernels over 70 % of K: a 1.43x faster GEMM
            return orig_gemm(M, N, K * 7 // 10 // 64 * 64, *a, **k)
        if (variant == "blas_lstm_dw" and lstm_dw) or (variant == "blas_plain" and (lstm_dw or plain)):
            return blas(M, N, K, *a, **{n: v for n, v in k.items() if n not in ("a_conv", "b_conv", "splits")})
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
    torch.backends.cuda.matmul.allow_tf32 = False
    for v in sys.argv[2:] or ("default", "no_lstm_dw", "no_side", "default"):
        print(f"{prec} {v:12s} {run(prec, v):7.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
