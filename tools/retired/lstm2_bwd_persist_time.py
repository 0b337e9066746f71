"""Kernel time of the persistent lstm2 backward (autovc_lstm2_bwd_persist_*) against the
per-step launches (autovc_lstm2_bwd_*), B=64, H=1024, for T = 16 and 128 (tools only).
Run with AVC_BWDP_ABLATE=<bits> to time ablated forms (lstm2_persist.hip BArgs::ablate)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_lstm_persist_gpu as tl  # noqa: E402


def timed(fn, n=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    xs = []
    for _ in range(n):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        xs.append(e0.elapsed_time(e1) * 1e3)
    return sorted(xs)[n // 2]


def main():
    dev = torch.device("cuda", 0)
    B, H = 64, 1024
    print("ablate", os.environ.get("AVC_BWDP_ABLATE", "0"), flush=True)
    for T in (16, 128):
        W, fw, dh1 = tl._bwd_inputs(B, T, H, dev)
        for bf16 in (False, True):
            p = timed(lambda: tl._bwd_persist(B, T, H, W, fw, dh1, dev, bf16))
            r = timed(lambda: tl._bwd_ref(B, T, H, W, fw, dh1, dev, bf16))
            print(f"T={T:4d} {'bf16' if bf16 else 'fp32'}: persistent {p:9.1f} us ({p / (T + 1):6.2f} per "
                  f"iteration)  per-step launches {r:9.1f} us ({r / (T + 1):6.2f})", flush=True)


if __name__ == "__main__":
    main()
