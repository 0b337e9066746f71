"""One weight-gradient GEMM shape repeated (for rocprofv3 --pmc / --kernel-trace): ours
(autovc_gemm_f32 with the product's split plan) or torch.mm (hipBLASLt).  Tools only.
    python tools/gemm_pmc.py [ours|blas] [M N K] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autovc_amd import functional as AF  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "ours"
    M, N, K = (int(a) for a in (sys.argv[2:5] if len(sys.argv) > 4 else (4096, 1024, 8192)))
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    dG = torch.randn(K, M, device=dev, generator=g)
    X = torch.randn(K, N, device=dev, generator=g)
    C = torch.zeros(M, N, device=dev)
    sp = AF._splits_for(M, N, K)
    for _ in range(reps):
        if which == "ours":
            AF.gemm(M, N, K, dG, M, 1, X, N, 1, C, N, splits=sp, accumulate=True)
        else:
            torch.mm(dG.t(), X, out=C)
    torch.cuda.synchronize()
    print(which, M, N, K, "done")


if __name__ == "__main__":
    main()
