"""us per sample step of WaveNet generation, alternating the per-layer launch chain
(set_grid(0)), the all-CU dataflow generation with every workgroup polling the producers
(set_grid(1), mirror off) and with the per-XCD mirrored all-gather (set_grid(1) +
set_mirror(1, 1)), for B in WN_B (default 8 (BASELINE config 4's batch), 4, 2, 1 (the
reference's wavegen)); WN_TC conditioning frames (x 256 samples), 24 layers.  Prints the
largest difference of each form from the launches and whether grid and mirror agree bit for
bit.  Not part of the product."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

Tc = int(os.environ.get("WN_TC", "8"))
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
lib = _lib.load()
MODES = (("launches", 0, 0), ("grid", 1, 0), ("mirror", 1, 1))
for B in [int(b) for b in os.environ.get("WN_B", "8,4,2,1").split(",")]:
    c = torch.clamp(torch.randn(B, 80, Tc, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
    ys = {}
    for rnd in range(3):
        for name, grid, mir in MODES:
            _lib.call("autovc_wavenet_set_grid", grid)
            _lib.call("autovc_wavenet_set_mirror", mir, 1)
            m.generate(c[:, :, :1], seed=1, log_scale_min=hparams.log_scale_min)   # warm (graphs / code objects)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            y = m.generate(c, seed=1, log_scale_min=hparams.log_scale_min)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / (Tc * 256) * 1e6
            ys[name] = y
            print(f"B={B} {name:8s} {us:8.2f} us per sample step", flush=True)
    for name in ("grid", "mirror"):
        d = (ys[name] - ys["launches"]).abs().max().item()
        print(f"B={B} max |{name} - launches| over {Tc * 256} free-running samples: {d:.3g}", flush=True)
    print(f"B={B} mirror == grid bit for bit: {bool(torch.equal(ys['mirror'], ys['grid']))}", flush=True)
f = ctypes.c_int(0)
_lib.call("autovc_wavenet_fault", 1, ctypes.addressof(f))
print(f"fault word after the runs: {f.value}", flush=True)
_lib.call("autovc_wavenet_set_grid", 2)
_lib.call("autovc_wavenet_set_mirror", 0, 1)
