"""Debug runs of the all-CU WaveNet generation (tools only): teacher-forced T=512 at B=3 with
the conditioning chunk = 512 (one call) and 128 (four calls), printing the timeout diagnostics."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from oracle import wavenet as ow  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_wavenet_gpu import _model, _cond, LSM  # noqa: E402

dev = torch.device("cuda:0")
_lib.call("autovc_wavenet_set_grid", 1)
for B in (8,):
    hp = ow.small_hparams(layers=24, stacks=4)
    m, W = _model(hp, dev)
    c = _cond(B, 2).to(dev)
    T = 512
    teacher = torch.from_numpy(np.random.RandomState(11).uniform(-0.9, 0.9, (B, T)).astype(np.float32)).to(dev)
    for chunk in (512,):
        try:
            ws_bytes = _lib.load().autovc_wavenet_workspace_bytes(B, T, 24, 6, 3, 512, 512, 256)
            print("workspace bytes", ws_bytes, flush=True)
            y = m.generate(c, T=T, seed=1234567, teacher=teacher, log_scale_min=LSM, chunk=chunk, graph_steps=0)
            print(f"B={B} chunk={chunk}: ok, finite={bool(torch.isfinite(y).all())}", flush=True)
        except RuntimeError as e:
            print(f"B={B} chunk={chunk}: {e}"[:300], flush=True)
