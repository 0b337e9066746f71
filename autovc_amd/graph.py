"""Whole-step HIP graphs for the Generator training step (not in the reference).

`Solver.train_step` is ~1,900 kernel launches per B=64 step (two Generator passes, the
LSTM/BLSTM recurrences one launch per time step, the backward with its side-stream weight
gradients).  Issued eagerly from Python, the host falls behind the GPU in the short-kernel
stretches (rocprof timeline: tools/trace_gaps.py).  `StepGraphs` captures the forward +
backward (losses, zero_grad, autograd backward, the gradient side stream's fork and join)
once per (input shapes, precision) into a `torch.cuda.CUDAGraph` (hipGraph) and replays it;
the data-parallel all-reduce and the FusedAdam step stay eager after the replay, so the
optimizer's host-side step count / lr schedule and RCCL are untouched.

Replays run the same kernels on the same buffers in the same order as the eager step, so
the losses and gradients are bit-identical to eager (tests/test_solver_gpu.py).  The
warm-up pass before the capture (lazy workspaces) would add one BatchNorm running-stat
update: those buffers are snapshotted and restored around it.
"""
from __future__ import annotations

import collections
import gc
import os

import torch

from . import functional as AF

# Replays the host may queue ahead of the GPU (0 = unbounded, the default).  Round 3 bounded
# it at 2 while looking for the cause of GPU memory faults in replays of step graphs without
# a side-stream branch; the cause was the memset nodes those single-stream graphs held
# (DESIGN.md section 9, round 4), not the queue depth, so the bound is off by default.
MAX_AHEAD = int(os.environ.get("AVC_GRAPH_MAX_AHEAD", "0"))
# AVC_CAPTURE_DEBUG=1: raise if device memory was returned to the HIP runtime (a hipFree:
# "segment.all.freed" of the caching allocator) while a step graph was being captured — the
# kind of free that aborted a capture in round 4 (an unreachable earlier Solver's graphs and
# private pool finalised by the cyclic collector inside the capture).
# Refcount-driven frees of ordinary tensors only return blocks to the caching allocator (no
# HIP call) and are allowed.
CAPTURE_DEBUG = os.environ.get("AVC_CAPTURE_DEBUG") == "1"


def _segments_freed(dev):
    return torch.cuda.memory_stats(dev).get("segment.all.freed", 0)


class CaptureFreeError(RuntimeError):
    """Device memory was released to the runtime during a step-graph capture (debug check)."""


class StepGraphs:
    def __init__(self, fn, module, debug_dot=None):
        self.fn = fn            # fn(*inputs) -> tuple of device tensors
        self.module = module    # holds the BatchNorm buffers the warm-up must not advance
        self.debug_dot = debug_dot   # path: write each captured graph as DOT (tools only)
        self._graphs = {}
        self._inflight = collections.deque()

    def _capture(self, inputs):
        dev = inputs[0].device
        static = [t.detach().clone() for t in inputs]
        saved = [b.detach().clone() for b in self.module.buffers()]
        cur = torch.cuda.current_stream(dev)
        warm = torch.cuda.Stream(dev)
        warm.wait_stream(cur)
        with torch.cuda.stream(warm):
            self.fn(*static)
        cur.wait_stream(warm)
        graph = torch.cuda.CUDAGraph()
        if self.debug_dot:
            graph.enable_debug_mode()
        # No garbage collection inside the capture: a collection there can finalise an
        # unreachable object that owns device state (an earlier Solver's captured graphs and
        # their private memory pool), and freeing it calls HIP APIs a capturing process must
        # not call — the process aborts (seen once: a previous test's Solver collected during
        # the next test's bf16 capture).  Collect first, then keep the collector off.
        gc.collect()
        gc.disable()
        # The counter is read inside the capture: torch.cuda.graph's entry empties the cache
        # (legitimate hipFree calls before capture begins), which must not count.
        freed = 0
        try:
            with torch.cuda.graph(graph):
                freed0 = _segments_freed(dev) if CAPTURE_DEBUG else 0
                out = self.fn(*static)
                freed = _segments_freed(dev) - freed0 if CAPTURE_DEBUG else 0
        finally:
            gc.enable()
        if CAPTURE_DEBUG:
            if freed:
                raise CaptureFreeError(f"{freed} device memory segment(s) were freed during a step-graph capture")
        if self.debug_dot:
            graph.debug_dump(self.debug_dot)
        with torch.no_grad():
            for b, s in zip(self.module.buffers(), saved):
                b.copy_(s)
        # the gradient-ready marks this graph records (data-parallel exchange): each cached
        # graph has its own mark structure, restored before each of its replays
        marks = AF.MARKS.snapshot() if AF.MARKS.active else None
        return graph, static, out, marks

    def run(self, key, *inputs):
        full_key = (key,) + tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)
        entry = self._graphs.get(full_key)
        if entry is None:
            entry = self._capture(inputs)
            self._graphs[full_key] = entry
        graph, static, out, marks = entry
        if marks is not None:
            AF.MARKS.restore(marks)
        for s, t in zip(static, inputs):
            if s.data_ptr() != t.data_ptr():
                s.copy_(t)
        if MAX_AHEAD > 0:
            while len(self._inflight) >= MAX_AHEAD:
                self._inflight.popleft().synchronize()
        graph.replay()
        if MAX_AHEAD > 0:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(inputs[0].device))
            self._inflight.append(ev)
        return out

    def reset(self):
        self._graphs.clear()
