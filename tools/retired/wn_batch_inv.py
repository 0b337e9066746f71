"""Batch invariance probe (tools only): wavegen_batch of [mel, mel[:2]] vs mel[:2] alone, per
generation mode (launches / XCD-local / all-CU), printing max |diff| and the first differing
sample."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib, synthesis  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = synthesis.build_model().to(dev)
mel = np.clip(np.random.RandomState(3).normal(0.43, 0.18, (3, 80)), 0, 1).astype(np.float32)
for name, xcd, grid in (("launches", 0, 0), ("xcd", 1, 0), ("grid", 0, 1)):
    _lib.call("autovc_wavenet_set_xcd", xcd)
    _lib.call("autovc_wavenet_set_grid", grid)
    ys = synthesis.wavegen_batch(model, [mel, mel[:2]], seed=9)
    solo = synthesis.wavegen_batch(model, [mel[:2]], seed=9, utt_offset=1)[0]
    d = np.abs(solo - ys[1])
    nz = np.nonzero(d)[0]
    print(f"{name}: max {d.max():.3e} first nonzero {nz[0] if len(nz) else None} n_nonzero {len(nz)}", flush=True)
