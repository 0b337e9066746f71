"""Diagnostic: the stacked lstm2 backward, fused step vs launch pair, through the C-ABI at
one shape; prints where dG1 / dG0 differ and whether repeated fused calls agree.  Tools only.
    python tools/fused_diag.py [B T H splits prec]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autovc_amd import _lib  # noqa: E402


def main():
    B, T, H, S = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 12, 1024, 4)))
    prec = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    bf = prec == "bf16"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    gates = [torch.rand(B, T, 4 * H, device=dev, generator=g) for _ in range(2)]
    cs = [torch.randn(B, T, H, device=dev, generator=g) * 0.5 for _ in range(2)]
    WT = [torch.randn(H, 4 * H, device=dev, generator=g) * H ** -0.5 for _ in range(3)]
    WTb = [w.to(torch.bfloat16) for w in WT]
    dh = torch.randn(B, T, H, device=dev, generator=g)
    ws = torch.empty(_lib.load().autovc_lstm2_bwd_workspace_floats(B, H, S), device=dev)

    def run(fused):
        _lib.call("autovc_lstm_bwd_set_fused", fused)
        dG = [torch.full((B, T, 4 * H), float("nan"), device=dev) for _ in range(2)]
        dGb = [torch.empty(B, T, 4 * H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        st = _lib.stream_ptr(dev)
        if bf:
            _lib.call("autovc_lstm2_bwd_bf16", B, T, H, dh.data_ptr(), T * H, H, gates[1].data_ptr(), cs[1].data_ptr(),
                      gates[0].data_ptr(), cs[0].data_ptr(), WTb[0].data_ptr(), WTb[1].data_ptr(), WTb[2].data_ptr(),
                      dG[1].data_ptr(), dGb[1].data_ptr(), dG[0].data_ptr(), dGb[0].data_ptr(), S, ws.data_ptr(), st)
        else:
            _lib.call("autovc_lstm2_bwd_f32", B, T, H, dh.data_ptr(), T * H, H, gates[1].data_ptr(), cs[1].data_ptr(),
                      gates[0].data_ptr(), cs[0].data_ptr(), WT[0].data_ptr(), WT[1].data_ptr(), WT[2].data_ptr(),
                      dG[1].data_ptr(), dG[0].data_ptr(), S, ws.data_ptr(), st)
        torch.cuda.synchronize()
        return dG

    pair = run(0)
    pair2 = run(0)
    fa = run(1)
    fb = run(1)
    _lib.call("autovc_lstm_bwd_set_fused", -1)
    for name, k in (("dG0", 0), ("dG1", 1)):
        for lab, x, y in (("pair vs pair", pair, pair2), ("fused vs fused", fa, fb), ("fused vs pair", fa, pair)):
            d = (x[k] - y[k]).abs()
            nan = int(torch.isnan(x[k]).sum())
            bad = (d > 0) | torch.isnan(d)
            n = int(bad.sum())
            msg = f"{name} {lab:15s}: {n} differing, max {float(torch.nan_to_num(d, nan=1e30).max()):.3e}, nan {nan}"
            if n:
                idx = bad.nonzero()
                ts = sorted(set(idx[:, 1].tolist()))
                bs = sorted(set(idx[:, 0].tolist()))
                js = idx[:, 2]
                msg += f"; steps {ts[:12]}; rows {bs[:12]}{'...' if len(bs) > 12 else ''}; cols {int(js.min())}..{int(js.max())}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()
