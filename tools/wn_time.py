"""us per sample step of the WaveNet generation (8 utterances, graph replay), for A/B runs
of the step kernels (tools/wn_ab.sh, tools/wn_ab_libs.sh); WN_TC frames, WN_B utterances,
WN_GS graph steps.  Not part of the product."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("WN_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

Tc = int(os.environ.get("WN_TC", "8"))
n = int(os.environ.get("WN_B", "8"))
gs = int(os.environ.get("WN_GS", "32"))
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
c = torch.clamp(torch.randn(n, 80, Tc, generator=torch.Generator().manual_seed(1)) * 0.18 + 0.43, 0, 1).to(dev)
m.generate(c[:, :, :2], seed=1, log_scale_min=hparams.log_scale_min, graph_steps=gs)
torch.cuda.synchronize()
res = []
for _ in range(3):
    t0 = time.perf_counter()
    m.generate(c, seed=1, log_scale_min=hparams.log_scale_min, graph_steps=gs)
    torch.cuda.synchronize()
    res.append((time.perf_counter() - t0) / (Tc * 256) * 1e6)
print(f"  us/sample step: {sorted(res)[1]:.2f}  (runs {', '.join(f'{r:.2f}' for r in res)})", flush=True)
