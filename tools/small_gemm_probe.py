"""Isolated timing of the small-output GEMMs of the encoder BLSTMs (tools only): M = B*T = 8192
rows, N = 64..512, K = 64..512 — the forward projections x W^T (RR), and the input gradient
dG W (RC, lda = 2G, accumulate) — through autovc_gemm_f32 / autovc_gemm_bf16_f32, against
torch.mm (hipBLASLt) of the same operands.   python tools/small_gemm_probe.py [fp32|bf16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import functional as AF  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        torch.cuda.synchronize()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M = 8192
    with AF.precision(prec):
        for N, K, tb, lda, acc in [(128, 64, 0, 64, 0), (128, 128, 0, 128, 0), (128, 256, 0, 256, 0),
                                   (128, 512, 0, 512, 0), (512, 128, 1, 256, 0), (512, 128, 1, 256, 1),
                                   (64, 128, 1, 256, 0), (64, 128, 1, 256, 1), (512, 512, 0, 512, 0),
                                   (1024, 512, 0, 512, 0)]:
            A = torch.randn(M, lda, device=dev, generator=g)
            Bm = torch.randn(K, N, device=dev, generator=g) if tb else torch.randn(N, K, device=dev, generator=g)
            C = torch.zeros(M, N, device=dev)
            fn = lambda: AF.gemm(M, N, K, A, lda, 0, Bm, Bm.shape[1], tb, C, N, accumulate=bool(acc))  # noqa: E731
            us = timeit(fn)
            Ak = A[:, :K]
            Bk = Bm if tb else Bm.t()
            if prec == "bf16":
                Ab, Bb = Ak.to(torch.bfloat16), Bk.to(torch.bfloat16)
                blas = lambda: torch.mm(Ab, Bb)  # noqa: E731
            else:
                blas = lambda: torch.mm(Ak, Bk)  # noqa: E731
            ub = timeit(blas)
            copy = torch.empty_like(C)
            uc = timeit(lambda: copy.copy_(C))
            print(f"{prec} M={M} N={N:4d} K={K:3d} {'RC' if tb else 'RR'} lda={lda:3d} acc={acc}: ours {us:6.1f} us"
                  f"  blas {ub:6.1f} us  (C copy {uc:5.1f} us)", flush=True)


if __name__ == "__main__":
    main()
