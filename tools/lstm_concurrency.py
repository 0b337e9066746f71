"""Microbenchmark: do two latency-bound LSTM step chains (or a chain and a GEMM) overlap
when issued on two HIP streams?  Decides whether the stacked decoder lstm2 should run its
two layers as a time-lagged wavefront on two streams.

  python tools/lstm_concurrency.py      (GPU box)
"""
from __future__ import annotations

import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


def chain(B, T, H, gx, W, h, c, gates, stream):
    _lib.call("autovc_lstm_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(),
              T * H, H, c.data_ptr(), gates.data_ptr(), 0, stream.cuda_stream)


def gemm(M, N, K, A, Bm, C, stream):
    _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), K, 0, 0, 0, 0, Bm.data_ptr(), K, 0, 0, 0, 0,
              C.data_ptr(), N, 0, 0, 0, 1, 0, stream.cuda_stream)


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


def main():
    dev = torch.device("cuda:0")
    B, T, H = 64, 128, 1024
    g = torch.Generator().manual_seed(0)
    bufs = []
    for _ in range(2):
        gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
        W = (torch.randn(4 * H, H, generator=g) * 0.03).to(dev)
        bufs.append((gx, W, torch.empty(B, T, H, device=dev), torch.empty(B, T, H, device=dev),
                     torch.empty(B, T, 4 * H, device=dev)))
    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)
    A = torch.randn(B * T, 1024, device=dev)
    Wp = torch.randn(4096, 1024, device=dev)
    C = torch.empty(B * T, 4096, device=dev)

    one = timeit(lambda: chain(B, T, H, *bufs[0], s1))
    seq = timeit(lambda: (chain(B, T, H, *bufs[0], s1), chain(B, T, H, *bufs[1], s1)))
    par = timeit(lambda: (chain(B, T, H, *bufs[0], s1), chain(B, T, H, *bufs[1], s2)))
    gm = timeit(lambda: gemm(B * T, 4096, 1024, A, Wp, C, s2))
    gpar = timeit(lambda: (chain(B, T, H, *bufs[0], s1), gemm(B * T, 4096, 1024, A, Wp, C, s2)))
    g4 = timeit(lambda: [gemm(B * T, 4096, 1024, A, Wp, C, s2) for _ in range(4)])
    g4par = timeit(lambda: (chain(B, T, H, *bufs[0], s1), [gemm(B * T, 4096, 1024, A, Wp, C, s2) for _ in range(4)]))
    # stream priorities: the latency-bound chain on a high-priority stream, GEMMs low
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    sh = torch.cuda.Stream(dev, priority=-1)
    sl = torch.cuda.Stream(dev, priority=0)
    gpar_p = timeit(lambda: (chain(B, T, H, *bufs[0], sh), gemm(B * T, 4096, 1024, A, Wp, C, sl)))
    g4par_p = timeit(lambda: (chain(B, T, H, *bufs[0], sh), [gemm(B * T, 4096, 1024, A, Wp, C, sl) for _ in range(4)]))
    print(f"priorities: chain hi || GEMM lo:  {gpar_p:.3f} ms ; chain hi || 4 GEMMs lo: {g4par_p:.3f} ms")
    # conv-shaped GEMMs (64x64 tiles, 36.9 KB LDS each: 4 per CU leave no room for a 37 KB
    # step workgroup) with an LDS pad that caps them at 3 per CU
    Xc = torch.randn(B * T, 2560, device=dev)
    Wc = torch.randn(512, 2560, device=dev)
    Cc = torch.empty(B * T, 512, device=dev)
    conv4 = lambda st: [gemm(B * T, 512, 2560, Xc, Wc, Cc, st) for _ in range(4)]  # noqa: E731
    c4 = timeit(lambda: conv4(s2))
    c4par = timeit(lambda: (chain(B, T, H, *bufs[0], s1), conv4(s2)))
    res = {}
    for pad in (38912, 49152):
        _lib.call("autovc_gemm_set_lds_reserve", pad)
        res[pad] = (timeit(lambda: conv4(s2)), timeit(lambda: (chain(B, T, H, *bufs[0], s1), conv4(s2))))
    _lib.call("autovc_gemm_set_lds_reserve", 0)
    print(f"4 conv GEMMs alone {c4:.3f} ms; chain || 4 conv GEMMs {c4par:.3f} ms (sum {one + c4:.3f})")
    for pad, (a_, b_) in res.items():
        print(f"  LDS reserve {pad:6d} B: 4 conv GEMMs alone {a_:.3f} ms; chain || them {b_:.3f} ms (sum {one + a_:.3f})")
    print(f"one chain (128 steps, H=1024, B=64): {one:.3f} ms")
    print(f"two chains, one stream:               {seq:.3f} ms")
    print(f"two chains, two streams:              {par:.3f} ms")
    print(f"proj GEMM 8192x4096x1024 alone:       {gm:.3f} ms")
    print(f"chain || GEMM:                        {gpar:.3f} ms  (sum {one + gm:.3f})")
    print(f"4 GEMMs alone:                        {g4:.3f} ms")
    print(f"chain || 4 GEMMs:                     {g4par:.3f} ms  (sum {one + g4:.3f})")
    # correctness of the concurrent run: chain outputs equal to a solo run
    chain(B, T, H, *bufs[0], s1)
    torch.cuda.synchronize()
    ref = bufs[0][2].clone()
    chain(B, T, H, *bufs[0], s1)
    chain(B, T, H, *bufs[1], s2)
    torch.cuda.synchronize()
    print("concurrent run bit-exact:", bool(torch.equal(ref, bufs[0][2])))


if __name__ == "__main__":
    main()
