"""Time of the persistent lstm2 forward (B=64, T=128, H=1024) fp32 and bf16, median of 7
events-timed launches (tools only; pick the library with AUTOVC_HIP_LIB for A/B builds).
`--ab ENV` alternates ENV=0 / ENV=1 (read per launch by the library) over 3 rounds."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T, H = 64, 128, 1024
    g = torch.Generator().manual_seed(1)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    W = [((torch.rand(4 * H, H, generator=g) * 2 - 1) / H ** 0.5).to(dev) for _ in range(3)]
    Wb = [w.bfloat16().contiguous() for w in W]
    b1, b2 = ((torch.rand(4 * H, generator=g) * 0.2 - 0.1).to(dev) for _ in range(2))
    o = [torch.empty(B, T, H, device=dev) for _ in range(4)]
    gt = [torch.empty(B, T, 4 * H, device=dev) for _ in range(2)]
    lib = _lib.load()
    ws = torch.empty(lib.autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
    st = _lib.stream_ptr(dev)
    ab = sys.argv[sys.argv.index("--ab") + 1] if "--ab" in sys.argv else None
    for r in range(3 if ab else 1):
        for v in (("0", "1") if ab else (None,)):
            if ab:
                os.environ[ab] = v
            run(lib, st, B, T, H, gx, W, Wb, b1, b2, o, gt, ws, f"{ab}={v} " if ab else "")


def run(lib, st, B, T, H, gx, W, Wb, b1, b2, o, gt, ws, tag):
    for name, ww in (("autovc_lstm2_fwd_persist_f32", W), ("autovc_lstm2_fwd_persist_bf16", Wb)):
        args = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, ww[0].data_ptr(), b1.data_ptr(), b2.data_ptr(),
                ww[1].data_ptr(), ww[2].data_ptr(), o[0].data_ptr(), o[1].data_ptr(), gt[0].data_ptr(), o[2].data_ptr(),
                o[3].data_ptr(), gt[1].data_ptr(), ws.data_ptr(), st]
        ts = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.call(name, *args)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        assert lib.autovc_lstm2_persist_status(ws.data_ptr(), st) == 0
        m = sorted(ts[1:])[3]
        print(f"{tag}{name:32s} {m:8.1f} us per sequence = {m / (T + 1):6.2f} us per wavefront step", flush=True)


if __name__ == "__main__":
    main()
