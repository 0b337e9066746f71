"""Per-step time of the decoder lstm1 forward recurrence (B=64, T=128, H=512) as run by
the Generator: the per-step launches (autovc_lstm_fwd_f32), the chip-wide persistent launch
(autovc_lstm_fwd_persist_f32) and the XCD-local persistent launch (autovc_lstm_fwd_xcd_f32);
median of 7 events-timed calls, alternating (tools only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T, H = 64, 128, 512
    g = torch.Generator().manual_seed(1)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    W = ((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(dev)
    h, c = (torch.empty(B, T, H, device=dev) for _ in range(2))
    gt = torch.empty(B, T, 4 * H, device=dev)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    wsp = torch.empty(lib.autovc_lstm_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
    wsx = torch.empty(lib.autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=dev)
    base = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(), T * H, H, c.data_ptr(),
            gt.data_ptr()]
    runs = {"per-step launches": lambda: _lib.call("autovc_lstm_fwd_f32", *base, 0, st),
            "persistent (chip-wide barrier)": lambda: _lib.call("autovc_lstm_fwd_persist_f32", *base, wsp.data_ptr(), st),
            "persistent (XCD-local)": lambda: _lib.call("autovc_lstm_fwd_xcd_f32", *base, wsx.data_ptr(), st)}
    WT = W.t().contiguous()
    dh = torch.randn(B, T, H, generator=g).to(dev) * 0.1
    dG = torch.empty(B, T, 4 * H, device=dev)
    wsb = torch.empty(4 * lib.autovc_lstm_bwd_workspace_floats(B, H, 8), dtype=torch.uint8, device=dev)
    runs["backward: split-K launches"] = lambda: _lib.call(
        "autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gt.data_ptr(), c.data_ptr(), WT.data_ptr(),
        dG.data_ptr(), 0, 8, wsb.data_ptr(), st)
    runs["backward: persistent (XCD-local)"] = lambda: _lib.call(
        "autovc_lstm_bwd_xcd_f32", B, T, H, dh.data_ptr(), T * H, H, gt.data_ptr(), c.data_ptr(), W.data_ptr(),
        dG.data_ptr(), wsx.data_ptr(), st)
    Wb = W.bfloat16().contiguous()
    hb = torch.empty(B, T, H, device=dev, dtype=torch.bfloat16)
    runs["bf16: per-step launches"] = lambda: _lib.call(
        "autovc_lstm_fwd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(), h.data_ptr(), hb.data_ptr(),
        c.data_ptr(), gt.data_ptr(), 0, st)
    runs["bf16: persistent (XCD-local)"] = lambda: _lib.call(
        "autovc_lstm_fwd_xcd_bf16", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, Wb.data_ptr(), h.data_ptr(), T * H, H,
        c.data_ptr(), gt.data_ptr(), wsx.data_ptr(), st)
    ts = {k: [] for k in runs}
    for _ in range(7):
        for k, fn in runs.items():
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) * 1e3)
    for k, v in ts.items():
        m = sorted(v)[len(v) // 2]
        print(f"{k:32s} {m:8.1f} us per sequence = {m / T:6.2f} us per step")


if __name__ == "__main__":
    main()
