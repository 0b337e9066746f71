"""The ten-step Solver trajectory of tests/test_solver_gpu.py against the reference golden,
printed per step and loss (relative deviation), for the fp32 GEMM modes (fp32 MFMA, X6) and
a few seeds of the data order... (tools only).

    python tools/traj_dev.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from autovc_amd import _lib  # noqa: E402
import test_solver_gpu as T  # noqa: E402
from parity_tol import S, trajectory_tolerance  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    G = T.G
    tol = trajectory_tolerance()
    for mode in (0, 1):
        _lib.load().autovc_gemm_set_fp32_x6(mode)
        s = T._solver()
        x = torch.from_numpy(G["x"]).to(dev)
        e = torch.from_numpy(G["emb"]).to(dev)
        s.G.train()
        traj = []
        for _ in range(10):
            _, a, b, c = s.train_step(x, e)
            traj.append([a.item(), b.item(), c.item()])
        d = np.abs(np.array(traj) - G["solver_traj"]) / np.abs(G["solver_traj"])
        print(f"x6={mode}: max dev / tol per loss:", (d / tol).max(axis=0).round(3).tolist())
        print("  dev:", d.round(4).tolist(), flush=True)
        f64 = S["traj_f64"]
        own = np.abs(G["solver_traj"] - f64) / np.abs(f64)    # the reference's float32 vs its float64
        ours = np.abs(np.array(traj) - f64) / np.abs(f64)
        print("  vs float64 reference, ours:", ours.round(4).tolist())
        print("  vs float64 reference, the reference's float32:", own.round(4).tolist(), flush=True)


if __name__ == "__main__":
    main()
