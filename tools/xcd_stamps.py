"""Phase timeline of the XCD-local lstm1 forward (tools only): runs the kernel from a
stamp build (tools/build_variant.sh xstamp -DXCD_STAMP=1) and prints, per phase, the median
over workgroups and steps 2..16 of the time since the previous phase (s_memrealtime, 100 MHz).
  AUTOVC_HIP_LIB=tools/ubin/libautovc_xstamp.so python tools/xcd_stamps.py [bf16]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402

PH = ["step start", "barrier passed", "h staged", "products", "gates in LDS", "cell + h store issued",
      "h stores acked"]


def main():
    bf = len(sys.argv) > 1 and sys.argv[1] == "bf16"
    dev = torch.device("cuda", 0)
    B, T, H = 64, 128, 512
    g = torch.Generator().manual_seed(1)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    W = ((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(dev)
    Wb = W.bfloat16().contiguous()
    h, c = (torch.empty(B, T, H, device=dev) for _ in range(2))
    gt = torch.empty(B, T, 4 * H, device=dev)
    lib = _lib.load()
    ws = torch.empty(lib.autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=dev)
    name = "autovc_lstm_fwd_xcd_bf16" if bf else "autovc_lstm_fwd_xcd_f32"
    for _ in range(3):
        _lib.call(name, B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, (Wb if bf else W).data_ptr(), h.data_ptr(), T * H,
                  H, c.data_ptr(), gt.data_ptr(), ws.data_ptr(), _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    n = 8 * 32 * 16 * 8
    buf = (ctypes.c_ulonglong * n)()
    lib.autovc_xcd_stamps.argtypes = [ctypes.c_void_p]
    assert lib.autovc_xcd_stamps(buf) == 0
    st = np.array(buf, dtype=np.int64).reshape(256, 16, 8).astype(np.float64) * 0.01   # us
    step = st[:, 1:, 0] - st[:, :-1, 0]
    print(f"{name}: step period median {np.median(step):.3f} us (min {step.min():.3f}, max {step.max():.3f})")
    for p in range(1, 7):
        d = st[:, 1:, p] - st[:, 1:, p - 1]
        print(f"  {PH[p - 1]:>24s} -> {PH[p]:<24s} {np.median(d):7.3f} us  (p10 {np.percentile(d, 10):.3f}, "
              f"p90 {np.percentile(d, 90):.3f})")
    d = st[:, 2:, 0] - st[:, 1:-1, 6]
    print(f"  {'h stores acked':>24s} -> {'next step start':<24s} {np.median(d):7.3f} us")


if __name__ == "__main__":
    main()
