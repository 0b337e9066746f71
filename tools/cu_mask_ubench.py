"""Microbenchmark (tools only): does a weight-gradient GEMM on a CU-masked stream run beside a
latency-bound LSTM step chain?  Times the chain alone, the GEMM alone and both together for
several CU masks (autovc_stream_create_cu_mask).   python tools/cu_mask_ubench.py
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def masked_stream(dev, bits):
    words = (ctypes.c_uint32 * 8)()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    _lib.call("autovc_stream_create_cu_mask", 8, words, ctypes.byref(h))
    return torch.cuda.ExternalStream(h.value, device=dev)


def main():
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    print(f"CUs: {ncu}")
    g = torch.Generator().manual_seed(0)
    B, T = 64, 128
    # lstm1-shaped backward chain (H=512) and lstm2-shaped forward chain (H=1024)
    H = 512
    dh = (torch.randn(B, T, H, generator=g) * 0.1).to(dev)
    gates = torch.rand(B, T, 4 * H, generator=g).to(dev)
    cc = (torch.randn(B, T, H, generator=g) * 0.5).to(dev)
    WT = (torch.randn(H, 4 * H, generator=g) * 0.03).to(dev)
    dG = torch.empty(B, T, 4 * H, device=dev)
    splits = 8
    ws = torch.empty(_lib.load().autovc_lstm_bwd_workspace_floats(B, H, splits), device=dev)

    def chain(st):
        _lib.call("autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), cc.data_ptr(),
                  WT.data_ptr(), dG.data_ptr(), 0, splits, ws.data_ptr(), st.cuda_stream)

    M, N, K = 4096, 1024, B * T
    A = torch.randn(K, M, device=dev)      # dG^T-like operands: C = A^T B
    Bm = torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)

    def gemm(st, n=3):
        for _ in range(n):
            _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), M, 1, 0, 0, 0, Bm.data_ptr(), N, 1, 0, 0, 0,
                      C.data_ptr(), N, 0, 0, 0, 1, 0, st.cuda_stream)

    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)
    ch = timeit(lambda: chain(s1))
    print(f"lstm1-shaped backward chain alone: {ch:.3f} ms")
    # event-ordered forms (the training step's side stream waits for an event recorded on the
    # main stream just before the chain): wait issued before vs after the chain is enqueued
    def ev_before():
        ev = torch.cuda.Event()
        ev.record(s1)
        s2.wait_event(ev)
        chain(s1)
        gemm(s2)

    def ev_after():
        ev = torch.cuda.Event()
        ev.record(s1)
        chain(s1)
        s2.wait_event(ev)
        gemm(s2)
    gm0 = timeit(lambda: gemm(s2))
    print(f"event wait enqueued BEFORE the chain: {timeit(ev_before):.3f} ms; AFTER: {timeit(ev_after):.3f} ms "
          f"(chain {ch:.3f}, GEMMs {gm0:.3f})", flush=True)
    masks = {
        "none": None,
        "i%32<20": [i for i in range(ncu) if i % 32 < 20],
        "i<160": [i for i in range(min(160, ncu))],
        "i%8<5": [i for i in range(ncu) if i % 8 < 5],
        "i%4!=3": [i for i in range(ncu) if i % 4 != 3],
        "i%32<28": [i for i in range(ncu) if i % 32 < 28],
    }
    for name, bits in masks.items():
        st = s2 if bits is None else masked_stream(dev, bits)
        gm = timeit(lambda: gemm(st))
        both = timeit(lambda: (chain(s1), gemm(st)))
        print(f"mask {name:8s}: 3 dW GEMMs alone {gm:7.3f} ms; chain || GEMMs {both:7.3f} ms "
              f"(sum {ch + gm:7.3f}, max {max(ch, gm):7.3f})", flush=True)
    for lds in (38912,):
        _lib.call("autovc_gemm_set_lds_reserve", lds)
        gm = timeit(lambda: gemm(s2))
        both = timeit(lambda: (chain(s1), gemm(s2)))
        _lib.call("autovc_gemm_set_lds_reserve", 0)
        print(f"LDS reserve {lds}: 3 dW GEMMs alone {gm:7.3f} ms; chain || GEMMs {both:7.3f} ms "
              f"(sum {ch + gm:7.3f})", flush=True)


if __name__ == "__main__":
    main()
