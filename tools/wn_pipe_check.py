"""Layer-pipelined WaveNet generation (wn_pipe_kernel, AVC_WN_GRID mode 3) against the
per-layer launches (mode 0) and the all-CU kernel (mode 2 / 1), then alternating timings at
B = 1, 2, 8 (us per sample step).  Not part of the product; the GPU tests hold the parity
checks.  Usage: python tools/wn_pipe_check.py [check|time|both] [T_frames]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "both"
Tc = int(sys.argv[2]) if len(sys.argv) > 2 else 8
lib = _lib.load()
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
LSM = hparams.log_scale_min


def gen(mode, c, **kw):
    _lib.call("autovc_wavenet_set_grid", mode)
    out = m.generate(c, seed=17, log_scale_min=LSM, **kw)
    torch.cuda.synchronize()
    return out, lib.autovc_wavenet_last_path()


if what in ("check", "both"):
    _lib.call("autovc_wavenet_set_timeout_ticks", 50000000)    # 0.5 s per wait
    for B in (1, 2, 3, 8):
        c = torch.clamp(torch.randn(B, 80, 2, generator=torch.Generator().manual_seed(B)) * 0.18 + 0.43, 0, 1).to(dev)
        teacher = (torch.rand(B, 512, generator=torch.Generator().manual_seed(7)) * 1.8 - 0.9).to(dev)
        (y0, mol0), p0 = gen(0, c, teacher=teacher, return_mol=True)
        (y3, mol3), p3 = gen(3, c, teacher=teacher, return_mol=True)
        f = ctypes.c_int(0)
        _lib.call("autovc_wavenet_fault", 1, ctypes.addressof(f))
        rel = float((mol3 - mol0).abs().max() / mol0.abs().max())
        fr0, _ = gen(0, c)
        fr3, _ = gen(3, c)
        print(f"B={B} paths {p0}/{p3} fault={f.value} teacher-forced MoL rel {rel:.2e}  "
              f"free-running max|dy| {float((fr3 - fr0).abs().max()):.2e}  finite {bool(torch.isfinite(fr3).all())}",
              flush=True)
        if f.value:
            diag = (ctypes.c_int * 5)()
            _lib.call("autovc_wavenet_grid_diag", 1, ctypes.addressof(diag))
            print("  diag (kind, step, phase, wg, tag):", tuple(diag), flush=True)
            sys.exit(1)
    _lib.call("autovc_wavenet_set_timeout_ticks", 0)

if what in ("time", "both"):
    for B in (1, 2, 8):
        c = torch.clamp(torch.randn(B, 80, Tc, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
        res = {0: [], 2 if B <= 2 else 1: [], 3: []}
        for mode in res:
            gen(mode, c[:, :, :2])
        for rep in range(3):
            for mode in res:
                t0 = time.perf_counter()
                gen(mode, c)
                res[mode].append((time.perf_counter() - t0) / (Tc * 256) * 1e6)
        print(f"B={B} T={Tc * 256}: " + "  ".join(
            f"mode {k}: {sorted(v)[1]:.2f} us ({', '.join(f'{x:.1f}' for x in v)})" for k, v in res.items()), flush=True)
