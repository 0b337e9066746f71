"""Workload for the WaveNet PMC passes and kernel-trace stats (not part of the product):
BASELINE config 4's model (r9y9, 24 layers, 512 residual channels) on 8 utterances for
`Tc` conditioning frames (256 * Tc sample steps), as bench.wavenet_bench runs it.
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/wnpmc_f -o run --output-format csv -- python tools/wn_pmc.py 1
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/wnpmc_w -o run --output-format csv -- python tools/wn_pmc.py 1
  python tools/wn_pmc_summarize.py gpurun_out/wnpmc_f gpurun_out/wnpmc_w > profiles/r02/wavenet_pmc.json"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import synthesis  # noqa: E402
from autovc_amd.hparams import hparams  # noqa: E402

Tc = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = torch.device("cuda:0")
torch.manual_seed(4322)
m = synthesis.build_model()
m.make_generation_fast_()
m = m.to(dev).eval()
g = torch.Generator().manual_seed(4321)
c = torch.clamp(torch.randn(n, 80, Tc, generator=g) * 0.18 + 0.43, 0, 1).to(dev)
y = m.generate(c, seed=2, log_scale_min=hparams.log_scale_min)
torch.cuda.synchronize()
print("ok", tuple(y.shape), float(y.abs().mean()))
