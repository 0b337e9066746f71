"""Run-to-run determinism probe of the Solver step (graph replays under
AVC_GRAD_STREAM=0).  For each variant, two fresh solvers (same seed, same batch) run
`steps` steps; prints the loss trajectory's hex and whether the two runs agree bit for bit
and agree with the eager run of the same variant.

  python tools/det_probe.py B steps "graph=1,stream=0" "graph=1,stream=0,persist=0" ...
keys: graph (HIP graph replay), stream (weight-gradient side stream), persist (lstm2
persistent forward), wino (Winograd convs), keepxt (X~ reuse), prec (fp32|bf16)."""
import contextlib
import gc
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from autovc_amd import functional as AF  # noqa: E402
from autovc_amd.graph import StepGraphs  # noqa: E402


def run(B, steps, v):
    AF._GRAD_STREAM_ON = v.get("stream", "1") != "0"
    AF._PERSIST_ON = v.get("persist", "1") != "0"
    AF._WINOGRAD = v.get("wino", "1") != "0"
    AF._WINO_KEEP_XT = v.get("keepxt", "1") != "0"
    torch.manual_seed(0)
    with contextlib.redirect_stdout(sys.stderr):
        s = bench.make_solver(torch.device("cuda", 0), B)
    s.G.train()
    s.precision = v.get("prec", "fp32")
    x, e = bench.synthetic_batch(B, 128, torch.device("cuda", 0), 1234)
    graphs = StepGraphs(s._forward_backward, s.G) if v.get("graph", "1") == "1" else None
    out = []
    for _ in range(steps):
        if graphs is not None:
            g_loss, a, b, c, _ = graphs.run(s.precision, x, e)
        else:
            g_loss, a, b, c, _ = s._forward_backward(x, e)
        s._after_backward()
        s._optimizer_step()
        out.append(torch.stack([a.detach().reshape(()), b.detach().reshape(()), c.detach().reshape(())]).clone())
    torch.cuda.synchronize()
    AF.check_device_faults()
    traj = torch.stack(out).cpu()
    del graphs, s
    gc.collect()
    torch.cuda.empty_cache()
    return traj


def main():
    B, steps = int(sys.argv[1]), int(sys.argv[2])
    for spec in sys.argv[3:]:
        v = dict(kv.split("=") for kv in spec.split(",") if kv)
        r1 = run(B, steps, v)
        r2 = run(B, steps, v)
        re = run(B, steps, dict(v, graph="0"))
        h = lambda t: " ".join(f"{float(z):.9g}" for z in t[-1])  # noqa: E731
        first = next((i for i in range(steps) if not torch.equal(r1[i], r2[i])), None)
        firste = next((i for i in range(steps) if not torch.equal(r1[i], re[i])), None)
        print(f"{spec:40s} run1==run2: {torch.equal(r1, r2)} (first diff step {first}); "
              f"graph==eager: {torch.equal(r1, re)} (first diff step {firste}); last {h(r1)} | {h(r2)} | {h(re)}",
              flush=True)


if __name__ == "__main__":
    main()
