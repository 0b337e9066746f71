"""Tile-configuration sweep of the fp32 weight-gradient GEMM (both operands K-strided, the
LSTM dW shapes) in isolation: one child process per AVC_GEMM_BIGK / AVC_GEMM_BIG value (the
library reads them once), each timing autovc_gemm_f32 with the product's split plan, and
torch.mm (hipBLASLt) once for comparison.  Tools only.
    python tools/gemm_cfg_sweep.py [cfg ...]        (default 2 4 7 9 12 14)
AVC_GEMM_BIG and AVC_GEMM_SMALL (the unsplit choices) are set to the same id."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (M, N, K, a_trans, b_trans): the LSTM weight gradients (both operands K-strided), an LSTM
# input projection X W^T and its input gradient dG W (conv forward / dX have the same forms)
SHAPES = [(4096, 1024, 8192, 1, 1), (4096, 512, 8192, 1, 1), (2048, 512, 8192, 1, 1),
          (8192, 4096, 1024, 0, 0), (8192, 1024, 4096, 0, 1), (8192, 512, 2560, 0, 0)]


def child(which):
    import torch
    sys.path.insert(0, ROOT)
    from autovc_amd import functional as AF
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for M, N, K, ta, tb in SHAPES:
        A = torch.randn(K, M, device=dev, generator=g) if ta else torch.randn(M, K, device=dev, generator=g)
        Bm = torch.randn(K, N, device=dev, generator=g) if tb else torch.randn(N, K, device=dev, generator=g)
        Am, Bk = (A.t() if ta else A), (Bm if tb else Bm.t())      # (M, K), (K, N) views
        C = torch.zeros(M, N, device=dev)
        sp = AF._splits_for(M, N, K) if ta else 1
        if which == "blas":
            fn = lambda: torch.mm(Am, Bk, out=C)  # noqa: E731
        else:
            fn = lambda: AF.gemm(M, N, K, A, A.shape[1], ta, Bm, Bm.shape[1], tb, C, N, splits=sp,  # noqa: E731
                                 accumulate=False)
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(3):
            torch.cuda.synchronize()
            a.record()
            for _ in range(10):
                fn()
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) / 10 * 1e3)
        ref = torch.mm(Am, Bk)
        fn()
        err = float((C - ref).abs().max() / ref.abs().max())
        out.append(f"{M}x{N}x{K}{'C' if ta else 'R'}{'C' if tb else 'R'} s{sp}: {best:7.1f} us {2.0 * M * N * K / best / 1e6:5.1f} TF err {err:.1e}")
    print(f"{which:>5s} | " + " | ".join(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    cfgs = sys.argv[1:] or ["2", "4", "7", "9", "12", "14"]
    for c in cfgs + ["blas"]:
        env = dict(os.environ)
        if c != "blas":
            env["AVC_GEMM_BIGK"] = c
            env["AVC_GEMM_BIG"] = c
            env["AVC_GEMM_SMALL"] = c
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", c], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
