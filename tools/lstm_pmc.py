"""Workload for the PMC passes of the roofline `traffic` field (not part of the product):
the decoder lstm2 layer-0 forward recurrence (B=64, T=128, H=1024), as bench.py times it.
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python tools/lstm_pmc.py
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run --output-format csv -- python tools/lstm_pmc.py
  python tools/pmc_summarize.py gpurun_out/pmc_f gpurun_out/pmc_w > profiles/lstm_step_pmc.json"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402

B, T, H = 64, 128, 1024
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(7)
W = (torch.rand(4 * H, H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev)
gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
h = torch.empty(B, T, H, device=dev)
c = torch.empty(B, T, H, device=dev)
gates = torch.empty(B, T, 4 * H, device=dev)
for _ in range(2):
    _lib.call("autovc_lstm_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(),
              T * H, H, c.data_ptr(), gates.data_ptr(), 0, _lib.stream_ptr(dev))
torch.cuda.synchronize()
print("ok", float(h[:, -1].abs().mean()))
