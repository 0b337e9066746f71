"""Timeline of one WaveNet sample step from the WN_STAMP diagnostic library (tools/wn_stamps.sh):
per launch the first/last workgroup start and end, and the median per-workgroup phase
durations (entry -> start barrier -> operands in -> products done -> arrived -> stored).
Not part of the product."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

B = int(os.environ.get("WN_B", "8"))
STEP = int(os.environ.get("WN_STEP", "300"))
dev = torch.device("cuda:0")
lib = _lib.load()
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
c = torch.clamp(torch.randn(B, 80, 2, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
m.generate(c, seed=1, log_scale_min=hparams.log_scale_min)
torch.cuda.synchronize()
L, NWG, NS = 64, 512, 8
for rep in range(2):
    assert lib.autovc_wavenet_stamp_set(STEP + rep) == 0
    m.generate(c, seed=1, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (L * NWG * NS))()
    assert lib.autovc_wavenet_stamps(buf, ctypes.c_int64(L * NWG * NS)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(L, NWG, NS).astype(np.int64)
    nl = m.layers
    t0 = min(a[k][a[k][:, 0] > 0][:, 0].min() for k in range(2 * nl + 2) if (a[k][:, 0] > 0).any())
    us = lambda v: (v - 0) / 100.0  # 100 MHz ticks -> us
    print(f"== sample step {STEP + rep}, B={B}: times in us from the first workgroup start")
    print("launch            n  start[min,med,max]        end[min,med,max]      | med phases: barrier ops-in prod-done arrived end")
    prev_end = None
    for k in list(range(2 * nl)) + [2 * nl, 2 * nl + 1]:
        r = a[k]
        r = r[r[:, 0] > 0]
        if len(r) == 0:
            continue
        name = (f"L{k // 2:02d} {'resid' if k % 2 else 'gate '}" if k < 2 * nl else ("tail   " if k == 2 * nl else "head   "))
        s0, s6 = r[:, 0] - t0, r[:, 6] - t0
        ph = ""
        if k < 2 * nl:
            # stamps: 0 entry, 1 after the start barrier, 2 operands in, 3 products done,
            # 4 arrived / residual rows stored, 6 stores drained (5 unused)
            cols = [0, 1, 2, 3, 4, 6]
            d = np.diff(r[:, cols], axis=1)
            ph = " ".join(f"{us(np.median(d[:, i])):6.2f}" for i in range(len(cols) - 1))
        gap = "" if prev_end is None or k % 2 else f" gap {us(s0.min() - prev_end):5.2f}"
        print(f"{name}  {len(r):4d}  {us(s0.min()):7.2f} {us(np.median(s0)):7.2f} {us(s0.max()):7.2f}   "
              f"{us(s6.min()):7.2f} {us(np.median(s6)):7.2f} {us(s6.max()):7.2f} | {ph}{gap}")
        if k % 2 == 0 or k >= 2 * nl:
            prev_end = s6.max() if k >= 2 * nl else max(s6.max(), a[k + 1][a[k + 1][:, 0] > 0][:, 6].max() - t0
                                                       if (a[k + 1][:, 0] > 0).any() else 0)
