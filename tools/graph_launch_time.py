"""Host time of one step-graph replay call (hipGraphLaunch of the captured forward+backward)
against the step's GPU time, to see whether the host's enqueue of the ~800 captured nodes
paces the side-stream branch (tools only).  python tools/graph_launch_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T = 64, 128
    torch.manual_seed(0)
    solver = bench.make_solver(dev, B)
    solver.G.train()
    solver.hip_graph = True
    x, e = bench.synthetic_batch(B, T, dev, 1234)
    for _ in range(3):
        solver.train_step(x, e)
    torch.cuda.synchronize()
    graphs = solver._graphs
    host, gpu = [], []
    for _ in range(5):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        graphs.run(solver.precision, x, e)
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        host.append((t1 - t0) * 1e3)
        gpu.append(e0.elapsed_time(e1))
    print("replay call (host) ms:", " ".join(f"{v:.2f}" for v in host))
    print("replay on the GPU  ms:", " ".join(f"{v:.2f}" for v in gpu))


if __name__ == "__main__":
    main()
