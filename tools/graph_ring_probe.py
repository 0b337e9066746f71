"""Drive tools/graph_ring_probe.hip (diagnostic): replay a captured graph of `n` tiny kernel
nodes `r` times back to back (no host sync between replays) and check that every node ran
exactly r times, for a linear graph and for the same graph with a forked side node.

    python tools/graph_ring_probe.py N R1,R2,...      (e.g. 2000 1,2,4,8,16)

torch is imported first so that the probe binds to the same libamdhip64 as the product
library.  Build: hipcc --offload-arch=gfx950 -O2 -fPIC -shared tools/graph_ring_probe.hip
-o tools/pbin/libgraph_ring_probe.so"""
import ctypes
import os
import sys

import torch  # noqa: F401  (the runtime the product uses)

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    n = int(sys.argv[1])
    reps = [int(v) for v in sys.argv[2].split(",")]
    forks = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,0").split(",")]
    lib = ctypes.CDLL(os.path.join(HERE, "pbin", "libgraph_ring_probe.so"), mode=ctypes.RTLD_GLOBAL)
    fn = lib.probe_run
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
    print(f"HIP runtime: {torch.version.hip}; DEBUG_CLR_GRAPH_PACKET_CAPTURE="
          f"{os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '(unset)')}", flush=True)
    worst = 0
    for forked in forks:
        for r in reps:
            fb, fv, ms = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_double(0)
            bad = fn(n, r, forked, ctypes.byref(fb), ctypes.byref(fv), ctypes.byref(ms))
            shape = "forked" if forked else "linear"
            print(f"{shape:6s} n={n} replays={r:3d} packets_queued={n * r:7d}: "
                  f"{'OK' if bad == 0 else f'{bad} counters wrong (first node {fb.value}: {fv.value} runs)'}"
                  f"  {ms.value * 1e3:.1f} us/replay", flush=True)
            if bad < 0:
                print(f"  HIP error {-bad}", flush=True)
                return 2
            worst = max(worst, bad)
    return 1 if worst else 0


if __name__ == "__main__":
    sys.exit(main())
