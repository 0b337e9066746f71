"""Pointer-lifetime audit of the captured step graph (diagnostic, never faults the GPU).

Every C-ABI call made while the Solver's step graph is captured is recorded with its device
pointer arguments (the c_void_p slots of autovc_amd._lib._SIGS, minus the trailing stream
handle and the host-side job arrays of autovc_conv_weights_batched_f32).  After the capture,
after replays, and after eager work that allocates and frees memory between replays, each
recorded pointer is located in torch.cuda.memory_snapshot():
  live     inside an allocated block;
  pool     inside a free block of the graph's private pool (memory the capture itself freed
           and that only this graph's replays reuse);
  DANGLING inside a free block of the ordinary pool (the caching allocator may hand it to
           another tensor while the graph still reads or writes it);
  FOREIGN  outside every torch segment.
Any DANGLING / FOREIGN pointer is a lifetime hazard of the replay.

    python tools/graph_ptr_audit.py [B] [stream_on(0|1)] [precision]
"""
import contextlib
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from autovc_amd import _lib, functional as AF  # noqa: E402
from autovc_amd import graph as G  # noqa: E402

HOST_ARGS = {"autovc_conv_weights_batched_f32": {1, 2, 3, 4, 5}}


class Recorder:
    def __init__(self):
        self.on = False
        self.rec = []
        self._orig = _lib.call

    def __call__(self, name, *args):
        if self.on:
            sig = _lib._SIGS.get(name, [])
            ptr_slots = [i for i, t in enumerate(sig) if t is ctypes.c_void_p]
            if ptr_slots and ptr_slots[-1] == len(sig) - 1:
                ptr_slots = ptr_slots[:-1]          # the stream handle
            skip = HOST_ARGS.get(name, set())
            for i in ptr_slots:
                if i < len(args) and i not in skip and isinstance(args[i], int) and args[i]:
                    self.rec.append((name, i, args[i]))
        return self._orig(name, *args)


def classify(ptrs, pool_id):
    snap = torch.cuda.memory_snapshot()
    segs = []
    for s in snap:
        blocks, addr = [], s["address"]
        for b in s["blocks"]:
            blocks.append((addr, addr + b["size"], b["state"]))
            addr += b["size"]
        segs.append((s["address"], s["address"] + s["total_size"], tuple(s.get("segment_pool_id", (0, 0))), blocks))
    out = {}
    for name, i, p in ptrs:
        kind = "FOREIGN"
        for lo, hi, pid, blocks in segs:
            if lo <= p < hi:
                for blo, bhi, st in blocks:
                    if blo <= p < bhi:
                        if st.startswith("active"):
                            kind = "live"
                        elif tuple(pid) == tuple(pool_id):
                            kind = "pool"
                        else:
                            kind = "DANGLING"
                        break
                break
        out.setdefault(kind, []).append((name, i, p))
    return out


def report(tag, res):
    counts = {k: len(v) for k, v in res.items()}
    print(f"[{tag}] {counts}", flush=True)
    bad = 0
    for k in ("DANGLING", "FOREIGN"):
        for name, i, p in res.get(k, [])[:20]:
            print(f"   {k}: {name} arg {i} = {p:#x}", flush=True)
            bad += 1
    return bad


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    stream_on = (sys.argv[2] if len(sys.argv) > 2 else "0") != "0"
    prec = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    AF._GRAD_STREAM_ON = stream_on
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with contextlib.redirect_stdout(sys.stderr):
        s = bench.make_solver(dev, B)
    s.G.train()
    s.precision = prec
    x, e = bench.synthetic_batch(B, 128, dev, 1234)
    rec = Recorder()
    _lib.call = rec
    dot = os.path.join(ROOT, "gpurun_out", f"step_graph_{prec}_side{int(stream_on)}.dot")
    os.makedirs(os.path.dirname(dot), exist_ok=True)
    graphs = G.StepGraphs(s._forward_backward, s.G, debug_dot=dot)
    orig_capture = graphs._capture

    def capture(inputs):
        # record only inside the capture proper (the warm-up's pointers are not in the graph)
        real_graph = torch.cuda.graph

        class _G(real_graph):
            def __enter__(self_inner):
                r = super().__enter__()
                rec.on = True
                return r

            def __exit__(self_inner, *a):
                rec.on = False
                return super().__exit__(*a)
        torch.cuda.graph = _G
        try:
            return orig_capture(inputs)
        finally:
            torch.cuda.graph = real_graph
    graphs._capture = capture
    graphs.run(prec, x, e)
    torch.cuda.synchronize()
    graph = next(iter(graphs._graphs.values()))[0]
    pool = graph.pool()
    uniq = sorted({(n, i, p) for n, i, p in rec.rec}, key=lambda t: t[2])
    print(f"B={B} side_stream={'on' if stream_on else 'off'} precision={prec}: {len(rec.rec)} pointer "
          f"arguments recorded in the capture ({len(uniq)} distinct), graph pool {pool}", flush=True)
    bad = report("after capture", classify(uniq, pool))
    if os.path.exists(dot):
        import re
        text = open(dot).read()
        counts = {k: len(re.findall(k, text, re.I)) for k in ("kernel", "memset", "memcpy", "event")}
        print(f"graph DOT ({os.path.basename(dot)}): mentions per node kind {counts}", flush=True)
        if counts["memset"] or counts["memcpy"]:
            print("   graph holds memset / memcpy nodes", flush=True)
            bad += 1
    for _ in range(3):
        graphs.run(prec, x, e)
        s._after_backward()
        s._optimizer_step()
    torch.cuda.synchronize()
    bad += report("after 3 replays + Adam", classify(uniq, pool))
    # eager work between replays: an eager forward/backward allocates and frees activations
    with AF.precision(prec), AF.weight_scope():
        g_loss = s.compute_losses(x, e)[0]
        g_loss.backward()
    AF.join_grad_stream()
    del g_loss
    import gc
    gc.collect()
    bad += report("after an eager step between replays", classify(uniq, pool))
    graphs.run(prec, x, e)
    torch.cuda.synchronize()
    bad += report("after one more replay", classify(uniq, pool))
    print("AUDIT", "FAIL" if bad else "CLEAN", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
