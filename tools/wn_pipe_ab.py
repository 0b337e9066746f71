"""A/B of WaveNet generation paths / library builds, alternating in one process per library:
us per sample step at B = 1, 2, 8 for the given AVC_WN_GRID modes.  Usage:
python tools/wn_pipe_ab.py MODES [T_frames]   (MODES like 0,2,3; AUTOVC_HIP_LIB selects a build)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3").split(",")]
Tc = int(sys.argv[2]) if len(sys.argv) > 2 else 8
lib = _lib.load()
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
print("lib:", os.environ.get("AUTOVC_HIP_LIB", "autovc_amd/libautovc_hip.so"), flush=True)
for B in (1, 2, 8):
    c = torch.clamp(torch.randn(B, 80, Tc, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
    res = {}
    for mode in modes:
        if mode in (1, 2) and B > (8 if mode == 1 else 2):
            continue
        res[mode] = []
        _lib.call("autovc_wavenet_set_grid", mode)
        m.generate(c[:, :, :2], seed=1, log_scale_min=hparams.log_scale_min)
    for rep in range(3):
        for mode in res:
            _lib.call("autovc_wavenet_set_grid", mode)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.generate(c, seed=1, log_scale_min=hparams.log_scale_min)
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / (Tc * 256) * 1e6)
    print(f"B={B} T={Tc * 256}: " + "  ".join(
        f"mode {k}: {sorted(v)[1]:.2f} us ({', '.join(f'{x:.1f}' for x in v)})" for k, v in res.items()), flush=True)
