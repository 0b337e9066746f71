"""Phase timeline of the all-CU WaveNet generation (tools only; needs the trace build,
tools/build_wn_trace.sh): free-running generation at B = 8 and B = 1, then per phase of one
steady-state step the time (us) from the phase start to: inputs in, partials summed, past taps
in, published — for workgroups 0 and 137 (different XCDs)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AUTOVC_HIP_LIB", os.path.join(HERE, "tools", "pbin", "libautovc_hip_trace.so"))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from oracle import wavenet as ow  # noqa: E402
from test_wavenet_gpu import _model, _cond, LSM  # noqa: E402

dev = torch.device("cuda:0")
_lib.call("autovc_wavenet_set_grid", 1)
lib = _lib.load()
lib.autovc_wavenet_grid_trace.argtypes = [ctypes.c_void_p]   # a 64-bit pointer, not a C int
lib.autovc_wavenet_grid_trace.restype = ctypes.c_int
for B in (8, 1):
    hp = ow.small_hparams(layers=24, stacks=4)
    m, W = _model(hp, dev)
    c = _cond(B, 2).to(dev)
    m.generate(c, T=512, seed=3, log_scale_min=LSM, graph_steps=0)
    buf = (ctypes.c_int * (2 * 26 * 5))()
    lib.autovc_wavenet_grid_trace(ctypes.addressof(buf))
    tr = np.array(buf, dtype=np.int64).reshape(2, 26, 5)
    for w in range(2):
        base = tr[w, 0, 0]
        print(f"B={B} workgroup {(0, 137)[w]}: phase start / +inputs / +summed / +past taps / +published (us)")
        for p in range(26):
            st = tr[w, p, 0]
            rel = ["%6.2f" % ((tr[w, p, k] - st) / 100.0) if tr[w, p, k] else "     -" for k in range(1, 5)]
            print(f"  p{p:2d} {(st - base) / 100.0:8.2f}  " + " ".join(rel))
    sys.stdout.flush()
