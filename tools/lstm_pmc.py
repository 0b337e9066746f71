"""Workload for the PMC passes of the roofline `traffic` field (not part of the product):
`single`: one H=1024 layer's forward recurrence (B=64, T=128) on lstm_fwd_step_kernel;
`stack`: decoder lstm2's two-layer wavefront (lstm2_fwd_step_kernel), as bench.py times it;
`stackbwd`: its backward wavefront (lstm2_bwd_rec_kernel, autovc_lstm2_bwd_f32, split-K 4);
`persist`: the persistent weight-stationary lstm2 forward (lstm2_persist_kernel, one launch
  per sequence, what the Generator runs at B=64);
`blstm`: the encoder BLSTM layer (H=32, both directions per launch), forward and backward
  kernels, as bench.py's blstm_roofline times them;
`xcd`: decoder lstm1's XCD-local persistent forward (H=512, B=64).
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python tools/lstm_pmc.py stack
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run --output-format csv -- python tools/lstm_pmc.py stack
  python tools/pmc_summarize.py gpurun_out/pmc_f gpurun_out/pmc_w stack > profiles/lstm2_step_pmc.json"""
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
MODE = sys.argv[1] if len(sys.argv) > 1 else "single"
if MODE in ("stack", "persist"):
    W1 = (torch.rand(4 * H, H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev)
    Wi1 = (torch.rand(4 * H, H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev)
    bi, bh = (torch.rand(4 * H, generator=g) * 0.2 - 0.1).to(dev), (torch.rand(4 * H, generator=g) * 0.2 - 0.1).to(dev)
    h1, c1, g1 = torch.empty_like(h), torch.empty_like(c), torch.empty_like(gates)
if MODE == "stackbwd":
    dh1 = torch.randn(B, T, H, generator=g).to(dev)
    c1, g1 = torch.randn(B, T, H, generator=g).to(dev), torch.randn(B, T, 4 * H, generator=g).to(dev)
    c0, g0 = torch.randn(B, T, H, generator=g).to(dev), torch.randn(B, T, 4 * H, generator=g).to(dev)
    WT1, WIT1, WT0 = ((torch.rand(H, 4 * H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev) for _ in range(3))
    dG1, dG0 = torch.empty(B, T, 4 * H, device=dev), torch.empty(B, T, 4 * H, device=dev)
    ws = torch.empty(_lib.load().autovc_lstm2_bwd_workspace_floats(B, H, 4), device=dev)
if MODE == "blstm":
    Hs = 32
    bgx = (torch.randn(B, T, 8 * Hs, generator=g) * 0.5).to(dev)
    Wf, Wb = ((torch.rand(4 * Hs, Hs, generator=g) * 2 - 1).div_(Hs ** 0.5).to(dev) for _ in range(2))
    bh, bc = torch.empty(B, T, 2 * Hs, device=dev), torch.empty(B, T, 2 * Hs, device=dev)
    bgates = torch.empty(B, T, 8 * Hs, device=dev)
    bdh = torch.randn(B, T, 2 * Hs, generator=g).to(dev)
    bdG = torch.empty(B, T, 8 * Hs, device=dev)
if MODE == "xcd":
    H = 512
    W = (torch.rand(4 * H, H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    h, c, gates = torch.empty(B, T, H, device=dev), torch.empty(B, T, H, device=dev), torch.empty(B, T, 4 * H, device=dev)
    ws = torch.empty(_lib.load().autovc_lstm_xcd_workspace_bytes(), dtype=torch.uint8, device=dev)
for _ in range(2):
    if MODE == "blstm":
        st = _lib.stream_ptr(dev)
        _lib.call("autovc_blstm_fwd_f32", B, T, 32, 2, bgx.data_ptr(), Wf.data_ptr(), Wb.data_ptr(), bh.data_ptr(),
                  bc.data_ptr(), bgates.data_ptr(), st)
        _lib.call("autovc_blstm_bwd_f32", B, T, 32, 2, bdh.data_ptr(), bgates.data_ptr(), bc.data_ptr(),
                  Wf.data_ptr(), Wb.data_ptr(), bdG.data_ptr(), st)
    elif MODE == "xcd":
        _lib.call("autovc_lstm_fwd_xcd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(),
                  T * H, H, c.data_ptr(), gates.data_ptr(), ws.data_ptr(), _lib.stream_ptr(dev))
    elif MODE == "stackbwd":
        _lib.call("autovc_lstm2_bwd_f32", B, T, H, dh1.data_ptr(), T * H, H, g1.data_ptr(), c1.data_ptr(),
                  g0.data_ptr(), c0.data_ptr(), WT1.data_ptr(), WIT1.data_ptr(), WT0.data_ptr(), dG1.data_ptr(),
                  dG0.data_ptr(), 4, ws.data_ptr(), _lib.stream_ptr(dev))
    elif MODE == "persist":
        if "ws" not in globals():
            ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
        _lib.call("autovc_lstm2_fwd_persist_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(),
                  bi.data_ptr(), bh.data_ptr(), Wi1.data_ptr(), W1.data_ptr(), h.data_ptr(), c.data_ptr(),
                  gates.data_ptr(), h1.data_ptr(), c1.data_ptr(), g1.data_ptr(), ws.data_ptr(), _lib.stream_ptr(dev))
    elif MODE == "stack":
        _lib.call("autovc_lstm2_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), bi.data_ptr(),
                  bh.data_ptr(), Wi1.data_ptr(), W1.data_ptr(), h.data_ptr(), c.data_ptr(), gates.data_ptr(),
                  h1.data_ptr(), c1.data_ptr(), g1.data_ptr(), _lib.stream_ptr(dev))
    else:
        _lib.call("autovc_lstm_fwd_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(), h.data_ptr(),
                  T * H, H, c.data_ptr(), gates.data_ptr(), 0, _lib.stream_ptr(dev))
torch.cuda.synchronize()
print("ok", float(dG0.abs().mean()) if MODE == "stackbwd" else
      float(bdG.abs().mean()) if MODE == "blstm" else float(h[:, -1].abs().mean()))
