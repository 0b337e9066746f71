"""Host enqueue time vs device time of WaveNet generation (is the sample loop host-bound?).
Not part of the product.  python tools/wn_hostcost.py [Tc] [graph_steps,...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

Tc = int(sys.argv[1]) if len(sys.argv) > 1 else 8
gss = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "128,256,512").split(",")]
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
c = torch.clamp(torch.randn(8, 80, Tc, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
for gs in gss:
    m.generate(c, seed=1, log_scale_min=hparams.log_scale_min, graph_steps=gs)
    torch.cuda.synchronize()
    for _ in range(2):
        t0 = time.perf_counter()
        m.generate(c, seed=1, log_scale_min=hparams.log_scale_min, graph_steps=gs)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        n = Tc * 256
        print(f"graph_steps={gs}: enqueue {(t1 - t0) / n * 1e6:7.2f} us/step, total {(t2 - t0) / n * 1e6:7.2f} us/step",
              flush=True)
