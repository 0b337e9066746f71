"""D-VECTOR speaker encoder on the MI355X vs the reference golden (1e-4 rel), and
make_metadata's train.pkl / metadata.pkl generation end to end on a synthetic corpus."""
import os
import pickle
import types

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import speaker as sp

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(GOLDEN, "generator_golden.npz"))
D = np.load(os.path.join(GOLDEN, "dvector_golden.npz"))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / np.abs(b).max()


def _encoder(cuda):
    from autovc_amd.model_bl import D_VECTOR
    C = D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256).eval()
    C.load_state_dict(sp.make_weights())
    return C.to(cuda)


def test_dvector_vs_reference_golden(cuda):
    C = _encoder(cuda)
    x = torch.from_numpy(G["x"]).to(cuda)
    with torch.no_grad():
        out = C(x).cpu().numpy()
        out64 = C(x[:1, :64]).cpu().numpy()
    assert out.shape == (2, 256)
    assert rel(out, D["out"]) < 1e-4 and rel(out64, D["out64"]) < 1e-4


def test_make_metadata_end_to_end(cuda, tmp_path, monkeypatch):
    from autovc_amd.make_metadata import Metadata
    rs = np.random.RandomState(0)
    main = tmp_path / "corpus"
    for spk in ("p225", "p226"):
        d = main / "spmel" / spk
        d.mkdir(parents=True)
        for i in range(11):
            n = 100 if i == 3 else 150 + 7 * i        # one too-short file exercises the redraw loop
            np.save(d / f"{spk}_{i + 1:03d}.npy", rs.rand(n, 80).astype(np.float32))
    (main / "txt" / "p225").mkdir(parents=True)
    (main / "txt" / "p225" / "p225_001.txt").write_text("Please call Stella.\n")
    info = tmp_path / "speaker_info.txt"
    info.write_text("ID AGE GENDER ACCENTS REGION\np225 23 F English Southern\np226 22 M English Surrey\n")
    ckpt = tmp_path / "bl.ckpt"
    torch.save({"model_b": {"module." + k: v for k, v in sp.make_weights().items()}}, ckpt)
    cfg = types.SimpleNamespace(main_dir=str(main), model_type="spmel", speaker_embed=True,
                                speaker_info=str(info), speaker_checkpoint=str(ckpt))
    np.random.seed(0)
    Metadata(cfg).metadata()
    with open(main / "spmel" / "train.pkl", "rb") as f:   # written by this test's run
        train = pickle.load(f)
    assert [row[0] for row in train] == ["p225", "p226"]
    assert all(row[1].shape == (256,) and np.linalg.norm(row[1]) <= 1.0 + 1e-5 for row in train)
    assert train[0][2:] == [os.path.join("p225", f"p225_{i:03d}.npy") for i in range(1, 12)]
    with open(main / "spmel" / "metadata.pkl", "rb") as f:
        meta = pickle.load(f)
    assert meta[0][0] == 0 and meta[0][1][0] == "p225_001" and meta[0][2][0] == "p225"
    assert np.array_equal(meta[0][1][1], train[0][1])
    assert "Please call Stella." in (main / "spmel" / "metadata.log").read_text()


def test_metadata_missing_checkpoint_is_named(cuda, tmp_path):
    from autovc_amd.make_metadata import Metadata
    cfg = types.SimpleNamespace(main_dir=str(tmp_path), model_type="spmel", speaker_checkpoint=str(tmp_path / "x.ckpt"))
    with pytest.raises(FileNotFoundError, match="x.ckpt"):
        Metadata(cfg).speaker_encoder(cuda)
