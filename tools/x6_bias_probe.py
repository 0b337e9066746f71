"""Rounding bias of the fp32 GEMM modes (tools only): all-positive operands, so that a
truncating accumulation shows as a signed mean error; relative to the fp64 product.

    python tools/x6_bias_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


def run(M, N, K, A, B, mode, at=0, bt=0):
    dev = A.device
    _lib.load().autovc_gemm_set_fp32_x6(mode)
    C = torch.empty(M, N, device=dev)
    _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), M if at else K, at, 0, 0, 0, B.data_ptr(), N if bt else K, bt,
              0, 0, 0, C.data_ptr(), N, 0, 0, 0, 1, 0, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    return C


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in [(512, 512, 8192), (64, 64, 8192), (2048, 512, 512)]:
        for dist in ("pos", "normal"):
            A = torch.rand(M, K, generator=g, device=dev) if dist == "pos" else torch.randn(M, K, generator=g, device=dev)
            B = torch.rand(K, N, generator=g, device=dev) if dist == "pos" else torch.randn(K, N, generator=g, device=dev)
            Bt = B.t().contiguous()
            ref = A.double() @ B.double()
            s = ref.abs().mean().item()
            line = f"{M}x{N}x{K} {dist:6s}"
            for mode in (0, 1):
                C = run(M, N, K, A, Bt, mode)
                d = C.double() - ref
                line += (f" | mode {mode}: signed mean {d.mean().item() / s:+.2e} abs mean {d.abs().mean().item() / s:.2e}"
                         f" max {d.abs().max().item() / s:.2e}")
            torch.backends.cuda.matmul.allow_tf32 = False
            Ct = (A @ B).double() - ref
            line += f" | torch {Ct.mean().item() / s:+.2e} {Ct.abs().mean().item() / s:.2e}"
            print(line, flush=True)
    _lib.load().autovc_gemm_set_fp32_x6(1)


if __name__ == "__main__":
    main()
