"""Phase timeline of wn_pipe_kernel from the trace build (tools/build_variant.sh wntrace
-DAVC_WN_PIPE_TRACE; AUTOVC_HIP_LIB=tools/pbin/libautovc_wntrace.so): s_memrealtime stamps (10 ns)
of wave 0 of every workgroup for utterance 0 of steps 64..67.  Prints, per step, each role's
events relative to layer 0's phase start.  Not part of the product."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
lib = _lib.load()
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
c = torch.clamp(torch.randn(B, 80, 1, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
_lib.call("autovc_wavenet_set_grid", 3)
m.generate(c, seed=17, log_scale_min=hparams.log_scale_min)
torch.cuda.synchronize()
N, E = 4, 8
buf = np.zeros(N * 256 * E, dtype=np.uint64)
fn = lib.autovc_wavenet_pipe_trace
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
tr = buf.reshape(N, 256, E).astype(np.int64)


def role(bid):   # csrc/wavenet.hip pipe_role
    xs, rk = bid & 7, bid >> 3
    if rk < 30:
        return f"L{(rk // 10) * 8 + xs:02d}.{rk % 10}"
    return {0: "tail", 1: "head"}.get(xs, "idle") + f".{rk - 30}"


names = ["start", "polled", "synced", "reduced", "published", "step_end", "past_end"]
for s in range(N):
    t0 = tr[s, 0, 0]
    print(f"=== step {64 + s} (B={B}); times in us after layer 0's phase start (workgroup 0)")
    rows = []
    for bid in range(256):
        r = role(bid)
        if r.startswith("idle") or not tr[s, bid].any():
            continue
        ev = tr[s, bid]
        rows.append((ev[0], r, ev))
    rows.sort()
    for _, r, ev in rows:
        cols = "  ".join(f"{names[k]} {(ev[k] - t0) / 100:7.2f}" if ev[k] else f"{names[k]}     -  " for k in range(7))
        print(f"{r:8s} {cols}")
