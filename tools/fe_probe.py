"""Front-end kernel probe for rocprofv3 counter passes: 20 launches of the fused
STFT+mel kernel on the bench's 256-utterance synthetic batch (spmel mode)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    r = bench.frontend_roofline(dev)
    print(r)
