"""The step's weight-gradient GEMM shapes on the library GEMM (autovc_gemm_f32 / _bf16_f32 with
the product's split-K plan) against torch.mm on the same operands (hipBLASLt / rocBLAS,
allow_tf32 off: exact fp32).  Tools only.   python tools/gemm_vs_blas.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autovc_amd import functional as AF  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    # (name, M = gate rows, N = input width, K = B*T): C[M,N] = dG^T (M x K) . X (K x N)
    shapes = [("lstm2 dW_hh/W_ih1", 4096, 1024, 8192), ("lstm2 dW_ih0", 4096, 512, 8192),
              ("lstm1 dW_hh", 2048, 512, 8192), ("lstm1 dW_ih", 2048, 320, 8192),
              ("chunk32 dW_hh", 4096, 1024, 2048), ("chunk16 dW_hh", 4096, 1024, 1024),
              ("conv dW im2col", 512, 2560, 8192)]
    print(f"{'shape':22s} {'M':>5s} {'N':>5s} {'K':>5s}  {'ours fp32':>10s} {'blas fp32':>10s}  "
          f"{'ours bf16':>10s} {'blas bf16':>10s}   (us; TF/s in brackets)")
    for name, M, N, K in shapes:
        dG = torch.randn(K, M, device=dev, generator=g)
        X = torch.randn(K, N, device=dev, generator=g)
        C = torch.zeros(M, N, device=dev)
        fl = 2.0 * M * N * K
        sp = AF._splits_for(M, N, K)

        def ours():
            AF.gemm(M, N, K, dG, M, 1, X, N, 1, C, N, splits=sp, accumulate=True)

        t_o = timed(ours)
        with AF.precision("bf16"):
            t_ob = timed(ours)
        t_b = timed(lambda: torch.mm(dG.t(), X, out=C))
        dGh, Xh = dG.to(torch.bfloat16), X.to(torch.bfloat16)
        Ch = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_bb = timed(lambda: torch.mm(dGh.t(), Xh, out=Ch))
        # correctness of ours against blas (fp32, one fresh call)
        C.zero_()
        ours()
        ref = torch.mm(dG.t(), X)
        err = float((C - ref).abs().max() / ref.abs().max())
        print(f"{name:22s} {M:5d} {N:5d} {K:5d}  {t_o:7.1f}[{fl / t_o / 1e6:4.0f}] {t_b:7.1f}[{fl / t_b / 1e6:4.0f}]  "
              f"{t_ob:7.1f}[{fl / t_ob / 1e6:4.0f}] {t_bb:7.1f}[{fl / t_bb / 1e6:4.0f}]  splits {sp} relerr {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
