"""Generates tests/golden/dvector_golden.npz by running the REFERENCE speaker encoder itself
(/root/reference/model_bl.py D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256), the
configuration make_metadata.py:41 builds), in the build container only.  The reference never
travels: only the arrays written here do.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_dvector_golden.py

Inputs: the two bundled 128-frame spmel crops of generator_golden.npz["x"] and a 64-frame
crop of the first.  Weights: oracle.speaker.make_weights (the seeded numpy scheme of
oracle.generator.deterministic_state_dict), loaded with load_state_dict.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")
from oracle.speaker import make_weights  # noqa: E402
from model_bl import D_VECTOR  # noqa: E402  (the reference module)


def main():
    G = np.load(os.path.join(HERE, "generator_golden.npz"))
    x = torch.from_numpy(G["x"])
    C = D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256).eval()
    C.load_state_dict(make_weights())
    with torch.no_grad():
        out = C(x).numpy()
        out64 = C(x[:1, :64]).numpy()
    np.savez_compressed(os.path.join(HERE, "dvector_golden.npz"), out=out, out64=out64,
                        keys=np.array(list(C.state_dict().keys())))
    print("wrote dvector_golden.npz", out.shape, out64.shape)


if __name__ == "__main__":
    main()
