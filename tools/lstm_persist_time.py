"""A/B of a single large-H LSTM layer's forward (B=64, T=128; H from argv, default 512 =
decoder lstm1): per-step launches (autovc_lstm_fwd_f32) vs the persistent launch
(autovc_lstm_fwd_persist_f32), alternating, events on the launch stream.  Not product code."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402

B, T = 64, 128
H = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(5)
W = ((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(dev)
gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
h, c = torch.empty(B, T, H, device=dev), torch.empty(B, T, H, device=dev)
gates = torch.empty(B, T, 4 * H, device=dev)
ws = torch.empty(_lib.load().autovc_lstm_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
st = _lib.stream_ptr(dev)
base = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(), T * H, H, c.data_ptr(), gates.data_ptr()]
step = lambda: _lib.call("autovc_lstm_fwd_f32", *base, 0, st)  # noqa: E731
pers = lambda: _lib.call("autovc_lstm_fwd_persist_f32", *base, ws.data_ptr(), st)  # noqa: E731


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
print("H", H, "status", _lib.load().autovc_lstm2_persist_status(ws.data_ptr(), st))
for k, v in res.items():
    m = sorted(v)[1]
    print(f"{k:8s} {m:9.1f} us per sequence = {m / T:6.2f} us per step  (runs {', '.join(f'{x:.0f}' for x in v)})")
