"""Probe (tools only): can the weight-gradient GEMMs and a latency-bound LSTM backward chain
stop slowing each other if they run on DIFFERENT XCDs (so that they share no L2)?
1. maps CU-mask bits to XCDs (a one-workgroup stamp kernel on a stream masked to one bit:
   autovc_stream_create_cu_mask + autovc_xcc_probe);
2. times the lstm1-shaped backward chain (decoder lstm1, H=512, B=64, T=128, fused steps) and
   three LSTM dW GEMMs (4096x1024x8192, fp32) alone and together: unmasked (today's side stream),
   and with the chain on XCD set A and the GEMMs on the complementary set B.
Chain times are from events on the chain's own stream.   python tools/xcd_split_probe.py"""
from __future__ import annotations

import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


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
    out = torch.full((1,), -1, dtype=torch.int32, device=dev)
    bit_xcd = []
    for i in range(ncu):
        st = masked_stream(dev, [i])
        _lib.call("autovc_xcc_probe", out.data_ptr(), st.cuda_stream)
        st.synchronize()
        bit_xcd.append(int(out.item()))
    by_x = {x: [i for i, v in enumerate(bit_xcd) if v == x] for x in sorted(set(bit_xcd))}
    print("CU-mask bit -> XCD: " + "; ".join(f"XCD {x}: {len(b)} bits, first {b[:4]}" for x, b in by_x.items()),
          flush=True)

    g = torch.Generator().manual_seed(0)
    B, T, H, S = 64, 128, 512, 8
    dh = (torch.randn(B, T, H, generator=g) * 0.1).to(dev)
    gates = torch.rand(B, T, 4 * H, generator=g).to(dev)
    cc = (torch.randn(B, T, H, generator=g) * 0.5).to(dev)
    WT = (torch.randn(H, 4 * H, generator=g) * 0.03).to(dev)
    dG = torch.empty(B, T, 4 * H, device=dev)
    ws = torch.empty(_lib.load().autovc_lstm_bwd_workspace_floats(B, H, S), device=dev)
    M, N, K = 4096, 1024, B * T
    A = torch.randn(K, M, device=dev)
    Bm = torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)

    def chain(st):
        _lib.call("autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates.data_ptr(), cc.data_ptr(),
                  WT.data_ptr(), dG.data_ptr(), 0, S, ws.data_ptr(), st.cuda_stream)

    def gemms(st, n=3):
        for _ in range(n):
            _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), M, 1, 0, 0, 0, Bm.data_ptr(), N, 1, 0, 0, 0,
                      C.data_ptr(), N, 0, 0, 0, 1, 0, st.cuda_stream)

    def run(sc, sg, together, reps=5):
        res = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            e0c, e1c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0g, e1g = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if together in ("both", "gemm"):
                e0g.record(sg)
                gemms(sg)
                e1g.record(sg)
            if together in ("both", "chain"):
                e0c.record(sc)
                chain(sc)
                e1c.record(sc)
            torch.cuda.synchronize()
            res.append((e0c.elapsed_time(e1c) if together != "gemm" else 0.0,
                        e0g.elapsed_time(e1g) if together != "chain" else 0.0))
        res = sorted(res[1:])
        return res[len(res) // 2]

    s_full_c, s_full_g = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    print(f"full chip: chain alone {run(s_full_c, s_full_g, 'chain')[0]:.3f} ms, 3 GEMMs alone "
          f"{run(s_full_c, s_full_g, 'gemm')[1]:.3f} ms", flush=True)
    _lib.call("autovc_gemm_set_lds_reserve", 38912)
    c, gm = run(s_full_c, s_full_g, "both")
    print(f"full chip, together (LDS reserve 38912 on the GEMMs): chain {c:.3f} ms, GEMMs {gm:.3f} ms", flush=True)
    _lib.call("autovc_gemm_set_lds_reserve", 0)
    xs = sorted(by_x)
    for na in (4, 5, 6):
        ca = [b for x in xs[:na] for b in by_x[x]]
        cb = [b for x in xs[na:] for b in by_x[x]]
        sa, sb = masked_stream(dev, ca), masked_stream(dev, cb)
        c_alone = run(sa, sb, "chain")[0]
        g_alone = run(sa, sb, "gemm")[1]
        c, gm = run(sa, sb, "both")
        print(f"chain on {na} XCDs / GEMMs on {8 - na}: chain alone {c_alone:.3f}, GEMMs alone {g_alone:.3f}; "
              f"together: chain {c:.3f}, GEMMs {gm:.3f} ms", flush=True)
    # the chain on all CUs, the GEMMs confined to some XCDs
    for nb in (2, 3, 4):
        cb = [b for x in xs[:nb] for b in by_x[x]]
        sb = masked_stream(dev, cb)
        _lib.call("autovc_gemm_set_lds_reserve", 38912)
        c, gm = run(s_full_c, sb, "both")
        _lib.call("autovc_gemm_set_lds_reserve", 0)
        print(f"chain on all CUs, GEMMs on {nb} XCDs (reserve on): chain {c:.3f}, GEMMs {gm:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
