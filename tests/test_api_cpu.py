"""Reference API surface (no GPU): module names, classes, signatures, hparams, data loader."""
import inspect
import os
import pickle
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT


def test_compat_shims_resolve_to_autovc_amd():
    sys.path.insert(0, os.path.join(ROOT, "compat"))
    try:
        import model_vc_mel
        import solver_encoder
        import hparams
        from autovc_amd import model_vc_mel as impl
        assert model_vc_mel is impl
        assert hasattr(solver_encoder, "Solver") and hasattr(hparams, "hparams")
    finally:
        sys.path.pop(0)


def test_generator_signature_and_state_dict_keys():
    from autovc_amd.model_vc_mel import Generator, Encoder, Decoder, Postnet, ConvNorm, LinearNorm  # noqa: F401
    from oracle.generator import generator_keys
    assert list(inspect.signature(Generator.__init__).parameters)[1:] == ["dim_neck", "dim_emb", "dim_pre", "freq"]
    g = Generator(32, 256, 512, 32)
    assert list(g.state_dict().keys()) == [k for k, _ in generator_keys()]
    assert sum(p.numel() for p in g.parameters()) == 28_422_464


def test_generator_stft_keys():
    from autovc_amd.model_vc_stft import GeneratorSTFT
    from oracle.generator import generator_keys
    g = GeneratorSTFT(32, 256, 512, 32)
    assert list(g.state_dict().keys()) == [k for k, _ in generator_keys(n_in=513, n_out=513, prefix="model.")]


def test_hparams_values():
    from autovc_amd.hparams import hparams
    assert hparams.layers == 24 and hparams.stacks == 4 and hparams.residual_channels == 512
    assert hparams.gate_channels == 512 and hparams.skip_out_channels == 256 and hparams.out_channels == 30
    assert hparams.upsample_scales == [4, 4, 4, 4] and hparams.hop_size == 256 and hparams.cin_channels == 80
    assert abs(hparams.log_scale_min - (-32.23619130191664)) < 1e-12
    hparams.foo = 3
    assert hparams["foo"] == 3


def test_data_loader_crop_pad_and_batches(tmp_path):
    from autovc_amd.data_loader import get_loader
    root = tmp_path / "spmel"
    meta = []
    rs = np.random.RandomState(0)
    for spk in ["p001", "p002", "p003"]:
        (root / spk).mkdir(parents=True)
        files = []
        for i, T in enumerate([100, 128, 300]):
            np.save(root / spk / f"{spk}_{i}.npy", rs.rand(T, 80).astype(np.float32))
            files.append(f"{spk}/{spk}_{i}.npy")
        meta.append([spk, rs.rand(256).astype(np.float32)] + files)
    with open(root / "train.pkl", "wb") as f:
        pickle.dump(meta, f)
    loader = get_loader(str(tmp_path), batch_size=2, len_crop=128, model_type="spmel")
    batches = list(loader)
    assert len(batches) == 1  # 3 speakers, drop_last
    x, e = batches[0]
    assert x.shape == (2, 128, 80) and e.shape == (2, 256) and x.dtype == torch.float32
    np.random.seed(0)
    ds = loader.dataset
    for _ in range(20):
        u, _ = ds[0]
        assert u.shape == (128, 80)


def test_metadata_refuses_cpu():
    import types
    from autovc_amd.make_metadata import Metadata
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="MI355X"):
        Metadata(types.SimpleNamespace(main_dir=".", model_type="spmel")).metadata()


def test_solver_refuses_cpu():
    import types
    from autovc_amd.solver_encoder import Solver
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cfg = types.SimpleNamespace(lambda_cd=1, dim_neck=32, dim_emb=256, dim_pre=512, freq=32, lr=1e-4, batch_size=2,
                                num_iters=1, ema=0.9999, run_name="x", model_type="spmel", log_step=1)
    with pytest.raises(RuntimeError, match="MI355X"):
        Solver(None, cfg)


def test_bench_rank_count_mismatch_exits_nonzero():
    """bench.py under a launcher that started fewer ranks than --gpus asks for refuses to
    report (exit 3) instead of labelling a 1-rank number as N GPUs."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1")     # a launcher's env: no self-spawn
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 3, out.stderr[-2000:]
    assert "process group has 1 rank" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
