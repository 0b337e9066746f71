"""A/B of the decoder lstm2 forward (B=64, T=128, H=1024): per-step wavefront launches
(autovc_lstm2_fwd_f32) vs the persistent weight-stationary launch
(autovc_lstm2_fwd_persist_f32), alternating, events on the launch stream.  Not product code."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402

B, T, H = 64, 128, 1024
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(5)
W = [((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(dev) for _ in range(3)]
b1, b2 = ((torch.rand(4 * H, generator=g) * 0.2 - 0.1).to(dev) for _ in range(2))
gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
outs = [torch.empty(B, T, H, device=dev) for _ in range(4)] + [torch.empty(B, T, 4 * H, device=dev) for _ in range(2)]
ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
st = _lib.stream_ptr(dev)
base = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W[0].data_ptr(), b1.data_ptr(), b2.data_ptr(), W[1].data_ptr(),
        W[2].data_ptr(), outs[0].data_ptr(), outs[1].data_ptr(), outs[4].data_ptr(), outs[2].data_ptr(),
        outs[3].data_ptr(), outs[5].data_ptr()]
step = lambda: _lib.call("autovc_lstm2_fwd_f32", *base, st)  # noqa: E731
pers = lambda: _lib.call("autovc_lstm2_fwd_persist_f32", *base, ws.data_ptr(), st)  # noqa: E731


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


res = {"step": [], "persist": []}
for _ in range(3):
    res["step"].append(timed(step))
    res["persist"].append(timed(pers))
print("status", _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), st))
for k, v in res.items():
    m = sorted(v)[1]
    print(f"{k:8s} {m:9.1f} us per sequence = {m / (T + 1):6.2f} us per wavefront iteration  (runs {', '.join(f'{x:.0f}' for x in v)})")
