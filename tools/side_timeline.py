"""Where the weight-gradient side stream's batches land in an UNPROFILED step-graph replay
(rocprofv3 tracing serialises the side stream, so its timeline cannot be
used).  Tools only: time stamps are one-thread kernels (autovc_stamp, the chip's 100 MHz
clock) inserted on the main and side streams at every recurrence and side batch, captured
into the step graph with everything else.

    python tools/side_timeline.py [fp32|bf16] [replays]

Prints, per stamp, the mean / min / max time after the step's first stamp (us) over the
replays, then the side batches as intervals beside the main-stream recurrences."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from autovc_amd import _lib  # noqa: E402
from autovc_amd import functional as AF  # noqa: E402
from autovc_amd import solver_encoder as SE  # noqa: E402

NSLOT = 1024
_state = {"buf": None, "labels": [], "n": 0}


def stamp(label, stream):
    i = _state["n"]
    _state["n"] += 1
    if i >= NSLOT:
        raise RuntimeError("too many stamps")
    if i >= len(_state["labels"]):
        _state["labels"].append(label)
    else:
        _state["labels"][i] = label
    _lib.call("autovc_stamp", _state["buf"].data_ptr() + 8 * i, stream.cuda_stream)


def install():
    orig_fb = SE.Solver._forward_backward
    orig_cl = SE.Solver.compute_losses
    orig_mark = AF._grad_mark
    orig_join = AF.join_grad_stream
    nrec = [0]
    nfl = [0]

    def fb(self, x, e):
        _state["n"] = 0
        nrec[0] = 0
        nfl[0] = 0
        stamp("step_start", torch.cuda.current_stream())
        out = orig_fb(self, x, e)
        stamp("step_end", torch.cuda.current_stream())
        return out

    def cl(self, x, e):
        out = orig_cl(self, x, e)
        stamp("forward_done", torch.cuda.current_stream())
        return out

    def mark(dev):
        nrec[0] += 1
        stamp(f"rec{nrec[0]}_begin(q={len(AF._GRAD_QUEUE)})", torch.cuda.current_stream(dev))
        return orig_mark(dev)

    def flush(beside_recurrence=True, after=None, lds_reserve=None):
        # functional._flush_grad_queue with stamps: main when the recurrence is done, side
        # when its batch starts and ends
        nfl[0] += 1
        if beside_recurrence:
            stamp(f"rec{nrec[0]}_end.{nfl[0]}", torch.cuda.current_stream())
        if not AF._GRAD_QUEUE:
            return
        items = list(AF._GRAD_QUEUE)
        AF._GRAD_QUEUE.clear()
        dev = items[0][0]
        main = torch.cuda.current_stream(dev)
        side = AF._grad_stream(dev)
        if after is not None:
            side.wait_event(after)
        else:
            side.wait_stream(main)
        tag = f"side{nrec[0]}.{nfl[0]}" if beside_recurrence else "side_final"
        stamp(f"{tag}_begin(n={len(items)})", side)
        AF._GRAD_STREAM_ACTIVE[0] = True
        AF._GRAD_PENDING.add(side.device.index)
        prev = AF._PRECISION[0]
        if lds_reserve is None:
            lds_reserve = AF.GRAD_LDS_RESERVE[items[0][3]] if beside_recurrence else 0
        _lib.call("autovc_gemm_set_lds_reserve", lds_reserve)
        try:
            with torch.cuda.stream(side):
                for _, fn, inputs, prec, _outs in items:
                    for t in inputs:
                        if t is not None:
                            t.record_stream(side)
                    AF._PRECISION[0] = prec
                    fn()
        finally:
            AF._PRECISION[0] = prev
            _lib.call("autovc_gemm_set_lds_reserve", 0)
            AF._GRAD_STREAM_ACTIVE[0] = False
        stamp(f"{tag}_end", side)

    def join(dev=None):
        stamp("join_main", torch.cuda.current_stream())
        orig_join(dev)
        stamp("join_done", torch.cuda.current_stream())

    SE.Solver._forward_backward = fb
    SE.Solver.compute_losses = cl
    AF._grad_mark = mark
    AF._flush_grad_queue = flush
    AF.join_grad_stream = join
    SE.AF.join_grad_stream = join


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    _state["buf"] = torch.zeros(NSLOT, dtype=torch.int64, device=dev)
    install()
    torch.manual_seed(0)
    s = bench.make_solver(dev, 64)
    s.G.train()
    s.precision = prec
    s.hip_graph = True
    x, e = bench.synthetic_batch(64, 128, dev, 1234)
    for _ in range(4):
        s.train_step(x, e)
    torch.cuda.synchronize()
    n = _state["n"]
    labels = list(_state["labels"][:n])
    rows = []
    t0 = time.perf_counter()
    for _ in range(reps):
        s.train_step(x, e)
        torch.cuda.synchronize()
        v = _state["buf"][:n].cpu().tolist()
        rows.append([(a - v[0]) / 100.0 for a in v])     # 100 MHz ticks -> us
    wall = (time.perf_counter() - t0) / reps * 1e3
    print(f"# {prec}: {n} stamps, {reps} replays (host-synchronised per step: {wall:.2f} ms per step incl. sync)")
    for i, lab in enumerate(labels):
        col = [r[i] for r in rows]
        print(f"{lab:34s} {sum(col) / len(col):9.1f} {min(col):9.1f} {max(col):9.1f}")
    # side batches as intervals
    mean = {lab: sum(r[i] for r in rows) / len(rows) for i, lab in enumerate(labels)}
    print("# side batches (begin .. end us, busy) and the main-stream recurrences:")
    for lab in labels:
        if lab.startswith("side") and "_begin" in lab:
            tag = lab.split("_begin")[0]
            end = mean.get(f"{tag}_end")
            print(f"  {lab:30s} {mean[lab]:9.1f} .. {end:9.1f}  ({end - mean[lab]:8.1f} us)")
        if lab.startswith("rec") and "_begin" in lab:
            tag = lab.split("_begin")[0]
            ends = [v for k, v in mean.items() if k.startswith(f"{tag}_end")]
            end = max(ends) if ends else None
            if end is not None:
                print(f"  {lab:30s} {mean[lab]:9.1f} .. {end:9.1f}  ({end - mean[lab]:8.1f} us)")


if __name__ == "__main__":
    main()
