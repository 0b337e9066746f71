"""Isolated timing of the large-H LSTM backward recurrences (decoder lstm2 stacked pair and
lstm1) at the training shape, fused step (one launch per step) against the product +
pointwise launch pair.  Tools only.   python tools/lstm_bwd_time.py [fp32|bf16]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autovc_amd import _lib  # noqa: E402
from autovc_amd import functional as AF  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    dev = torch.device("cuda", 0)
    B, T = 64, 128
    g = torch.Generator(device=dev).manual_seed(0)
    bf = prec == "bf16"
    for name, H, S in (("lstm2", 1024, int(os.environ.get("LBT_S2", "4"))), ("lstm1", 512, int(os.environ.get("LBT_S1", "8")))):
        gates = [torch.rand(B, T, 4 * H, device=dev, generator=g) for _ in range(2)]
        cs = [torch.randn(B, T, H, device=dev, generator=g) * 0.5 for _ in range(2)]
        WT = [torch.randn(H, 4 * H, device=dev, generator=g) * H ** -0.5 for _ in range(3)]
        WTb = [w.to(torch.bfloat16) for w in WT]
        dh = torch.randn(B, T, H, device=dev, generator=g)
        dG = [torch.empty(B, T, 4 * H, device=dev) for _ in range(2)]
        dGb = [torch.empty(B, T, 4 * H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        if name == "lstm2":
            ws = torch.empty(_lib.load().autovc_lstm2_bwd_workspace_floats(B, H, S), device=dev)
        else:
            ws = torch.empty(_lib.load().autovc_lstm_bwd_workspace_floats(B, H, S), device=dev)

        def call():
            st = _lib.stream_ptr(dev)
            if name == "lstm2" and bf:
                _lib.call("autovc_lstm2_bwd_bf16", B, T, H, dh.data_ptr(), T * H, H, gates[1].data_ptr(), cs[1].data_ptr(),
                          gates[0].data_ptr(), cs[0].data_ptr(), WTb[0].data_ptr(), WTb[1].data_ptr(), WTb[2].data_ptr(),
                          dG[1].data_ptr(), dGb[1].data_ptr(), dG[0].data_ptr(), dGb[0].data_ptr(), S, ws.data_ptr(), st)
            elif name == "lstm2":
                _lib.call("autovc_lstm2_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates[1].data_ptr(), cs[1].data_ptr(),
                          gates[0].data_ptr(), cs[0].data_ptr(), WT[0].data_ptr(), WT[1].data_ptr(), WT[2].data_ptr(),
                          dG[1].data_ptr(), dG[0].data_ptr(), S, ws.data_ptr(), st)
            elif bf:
                _lib.call("autovc_lstm_bwd_bf16", B, T, H, dh.data_ptr(), T * H, H, gates[0].data_ptr(), cs[0].data_ptr(),
                          WTb[0].data_ptr(), dG[0].data_ptr(), dGb[0].data_ptr(), 0, S, ws.data_ptr(), st)
            else:
                _lib.call("autovc_lstm_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates[0].data_ptr(), cs[0].data_ptr(),
                          WT[0].data_ptr(), dG[0].data_ptr(), 0, S, ws.data_ptr(), st)

        res = {}
        for rep in range(3):
            for fused in (1, 0):
                _lib.call("autovc_lstm_bwd_set_fused", fused)
                for _ in range(2):
                    call()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    call()
                b.record()
                torch.cuda.synchronize()
                res.setdefault(fused, []).append(a.elapsed_time(b) / 5 * 1e3)
        _lib.call("autovc_lstm_bwd_set_fused", -1)
        for fused in (1, 0):
            v = res[fused]
            print(f"{prec} {name} {'fused' if fused else 'pair '}: {min(v):8.1f} us per call "
                  f"({min(v) / T:6.2f} us per step; runs {', '.join(f'{x:.0f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
