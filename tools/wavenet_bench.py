"""WaveNet generation timing sweep (not part of the product): python tools/wavenet_bench.py [Tc] [n_utt]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

Tc = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = torch.device("cuda:0")
print(json.dumps(bench.wavenet_bench(dev, n_utt=n, Tc=Tc, cpu=False)), flush=True)
from autovc_amd import synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
c = torch.rand(n, 80, Tc, device=dev)
for gs in (0, 8, 32, 128):
    m.generate(c[:, :, :2], seed=1, graph_steps=gs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.generate(c, seed=1, graph_steps=gs, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"graph_steps={gs:4d}: {dt / (Tc * 256) * 1e6:8.2f} us/step  {n * Tc * 256 / dt:10.0f} samples/s", flush=True)
