"""Oracle pinning for the D-VECTOR speaker encoder (model_bl.py): oracle/speaker.py against
tests/golden/dvector_golden.npz, made from the reference's own D_VECTOR
(tests/golden/make_dvector_golden.py).  Forward bar 1e-4 rel."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from oracle import speaker as sp

G = np.load(os.path.join(GOLDEN, "generator_golden.npz"))
D = np.load(os.path.join(GOLDEN, "dvector_golden.npz"))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / np.abs(b).max()


def test_keys_match_reference():
    assert [k for k, _ in sp.dvector_keys()] == list(D["keys"])


def test_oracle_matches_reference_golden():
    P = sp.make_weights()
    x = torch.from_numpy(G["x"])
    assert rel(sp.dvector(P, x), D["out"]) < 1e-4
    assert rel(sp.dvector(P, x[:1, :64]), D["out64"]) < 1e-4
    assert np.allclose(np.linalg.norm(D["out"], axis=1), 1.0, atol=1e-5)


def test_module_state_dict_layout():
    from autovc_amd.model_bl import D_VECTOR
    m = D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256)
    assert list(m.state_dict().keys()) == list(D["keys"])
    shapes = dict(sp.dvector_keys())
    assert all(tuple(v.shape) == shapes[k] for k, v in m.state_dict().items())
