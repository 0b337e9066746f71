"""Isolated timing of the precision-"fp32" GEMMs: fp32 MFMA kernel vs the bf16-plane (X6) kernel
on the training step's shapes (CUDA events, 20 launches after 3 warm-ups each).

    python tools/gemm_x6_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402

SHAPES = [  # name, M, N, K, a_trans, b_trans, splits
    ("lstm2 dW_hh (4H x H over B*T)", 4096, 1024, 8192, 1, 1, 1),
    ("lstm1 dW_ih (4H x 512)", 2048, 512, 8192, 1, 1, 1),
    ("lstm2 dW_ih0 (4H x 512)", 4096, 512, 8192, 1, 1, 2),
    ("lstm2 input proj (B*T x 4H, K 512)", 8192, 4096, 512, 0, 0, 1),
    ("lstm2 dx (B*T x 512, K 4H)", 8192, 512, 4096, 0, 1, 1),
    ("wino GEMM (2048 x 512, K 512) x8", 2048, 512, 512, 0, 0, 8),
]


def main():
    dev = torch.device("cuda", 0)
    st = _lib.stream_ptr(dev)
    for name, M, N, K, at, bt, s in SHAPES:
        A = torch.randn(M * K, device=dev)
        B = torch.randn(K * N, device=dev)
        C = torch.empty(M * N * (s if "wino" in name else 1), device=dev)
        batched = "wino" in name
        res = {}
        for on in (0, 1):
            _lib.load().autovc_gemm_set_fp32_x6(on)
            # as functional.gemm: the library's split for the caller's request
            splits = 1 if batched else _lib.load().autovc_gemm_f32_splits(M, N, K, s)
            ws = torch.empty(4 * max(1, _lib.load().autovc_gemm_workspace_floats(M, N, splits)), dtype=torch.uint8,
                             device=dev)

            def launch():
                if batched:
                    _lib.call("autovc_gemm_batched_f32", s, M, N, K, A.data_ptr(), K, 0, 0, B.data_ptr(), K, 0, 0,
                              C.data_ptr(), N, M * N, 0, st)
                else:
                    _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), M if at else K, at, 0, 0, 0, B.data_ptr(),
                              N if bt else K, bt, 0, 0, 0, C.data_ptr(), N, 0, 0, 0, splits, ws.data_ptr(), st)
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                launch()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1000
            res[on] = us
        fl = 2.0 * M * N * K * (s if batched else 1)
        print(f"{name:40s} fp32 {res[0]:8.1f} us ({fl / res[0] / 1e6:6.1f} TF)   x6 {res[1]:8.1f} us "
              f"({fl / res[1] / 1e6:6.1f} TF)   x{res[0] / res[1]:.2f}", flush=True)
    _lib.load().autovc_gemm_set_fp32_x6(0)


if __name__ == "__main__":
    main()
