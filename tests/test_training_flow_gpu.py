"""The training driver as the reference's callers use it, on the GPU:

  * main.py:14-40's sequence (spectrogram folder found -> train.pkl found -> get_loader ->
    Solver(loader, config) -> train()) through the compat/ modules, on a tiny on-disk corpus
    in the reference layout (<main_dir>/spmel/<spk>/*.npy + train.pkl), with main.py's
    argparse defaults (main.py:44-73);
  * checkpoint / resume (solver_encoder.py:92-93,147-153,330-346): an interrupted run
    resumed from its checkpoint reproduces the uninterrupted run's later losses, and the
    saved state_dict is the reference's (loads into the oracle Generator with
    torch.load(weights_only=True) and gives the same forward)."""
import os
import pickle
import sys
import types

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import generator as og

pytestmark = pytest.mark.gpu


def _main_config(main_dir, run_name, **over):
    """main.py:44-73 defaults (model_type passed explicitly: the default 'stft' is the
    reference's broken GeneratorSTFT.forward)."""
    cfg = dict(lambda_cd=1.0, lambda_SISNR=1.0, dim_neck=32, dim_emb=256, dim_pre=512, freq=32, main_dir=main_dir,
               batch_size=2, num_iters=10000000, len_crop=128, lr=0.0001, speaker_embed=True, model_type="spmel",
               run_name=run_name, lr_scheduler=None, depth=1, ema=0.9999, resume=False, run_id=None, log_step=100)
    cfg.update(over)
    return types.SimpleNamespace(**cfg)


def _corpus(root, n_spk=3, seed=0):
    rs = np.random.RandomState(seed)
    meta = []
    for s in range(n_spk):
        spk = f"p{225 + s}"
        os.makedirs(os.path.join(root, "spmel", spk))
        files = []
        for i, T in enumerate([96, 160, 230]):
            np.save(os.path.join(root, "spmel", spk, f"{spk}_{i:03d}.npy"),
                    np.clip(rs.normal(0.43, 0.18, (T, 80)), 0, 1).astype(np.float32))
            files.append(f"{spk}/{spk}_{i:03d}.npy")
        e = rs.normal(size=256)
        meta.append([spk, (0.8 * e / np.linalg.norm(e)).astype(np.float32)] + files)
    with open(os.path.join(root, "spmel", "train.pkl"), "wb") as f:
        pickle.dump(meta, f)


def test_main_py_sequence_through_compat(cuda, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    main_dir = str(tmp_path / "corpus")
    _corpus(main_dir)
    sys.path.insert(0, os.path.join(ROOT, "compat"))
    try:
        import data_loader
        import make_metadata  # noqa: F401  (main.py:6 imports it)
        import make_spect     # noqa: F401  (main.py:7)
        import solver_encoder
        cfg = _main_config(main_dir, "flowtest", num_iters=3, log_step=3)
        # main.py:19-24 / 27-33: both the spectrogram folder and train.pkl exist -> skipped
        assert os.path.exists(os.path.join(cfg.main_dir, cfg.model_type))
        assert os.path.exists(cfg.main_dir + "/" + cfg.model_type + "/train.pkl")
        loader = data_loader.get_loader(cfg.main_dir, cfg.batch_size, cfg.len_crop, cfg.model_type)
        np.random.seed(0)
        solver = solver_encoder.Solver(loader, cfg)
        seen = []
        step = solver.train_step
        solver.train_step = lambda x, e: seen.append((tuple(x.shape), tuple(e.shape))) or step(x, e)
        solver.train()
    finally:
        sys.path.pop(0)
    assert seen == [((2, 128, 80), (2, 256))] * 3
    ck = torch.load(tmp_path / "chkpnt_spmel_flowtest.ckpt", map_location="cpu", weights_only=True)
    assert set(ck) == {"epoch", "state_dict", "optimizer", "loss"} and ck["epoch"] == 3
    assert set(ck["loss"]) == {"G/loss_id", "G/loss_id_psnt", "G/loss_cd"}
    assert all(np.isfinite(v) for v in ck["loss"].values())


class _FixedLoader:
    """A loader yielding one fixed batch per epoch (the Solver re-creates its iterator
    every iteration), so an interrupted and an uninterrupted run see the same data."""

    def __init__(self, x, e):
        self.batch = (x, e)

    def __iter__(self):
        return iter([self.batch])


def _run(cfg, loader):
    from autovc_amd.solver_encoder import Solver
    s = Solver(loader, cfg)
    if not s.file_exists:
        s.G.load_state_dict(og.make_weights())
    losses = []
    step = s.train_step

    def rec(x, e):
        out = step(x, e)
        losses.append([float(v.item()) for v in out[1:]])
        return out
    s.train_step = rec
    s.train()
    return s, losses


def test_checkpoint_resume_reproduces_uninterrupted_run(cuda, tmp_path, monkeypatch):
    import bench
    x, e = bench.synthetic_batch(4, 128, "cpu", 77)
    loader = _FixedLoader(x, e)
    monkeypatch.chdir(tmp_path)
    # uninterrupted: 4 iterations, checkpoint (EMA applied first) every 2
    _, full = _run(_main_config(".", "full", num_iters=4, log_step=2), loader)
    # interrupted after 2, then a fresh Solver resumes from chkpnt_spmel_part.ckpt
    _, first = _run(_main_config(".", "part", num_iters=2, log_step=2), loader)
    assert os.path.exists("chkpnt_spmel_part.ckpt")
    resumed_solver, rest = _run(_main_config(".", "part", num_iters=4, log_step=2, resume=True), loader)
    assert resumed_solver.file_exists and resumed_solver.i == 2
    assert os.path.exists("chkpnt_spmel_part_resumed.ckpt")      # solver_encoder.py:341-344
    assert first == full[:2]
    assert rest == full[2:], (rest, full[2:])                      # bit-identical continuation
    # the saved state_dict is the reference's: keys, and the oracle's forward on it
    ck = torch.load("chkpnt_spmel_part_resumed.ckpt", map_location="cpu", weights_only=True)
    assert ck["epoch"] == 4 and ck["optimizer"]["state"][0]["step"] == 4
    sd = ck["state_dict"]
    assert list(sd.keys()) == [k for k, _ in og.generator_keys()]
    P = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        _, ref_psnt, ref_code = og.OracleGenerator(P, training=False).forward(x, e, e)
        resumed_solver.G.eval()
        _, psnt, code = resumed_solver.G(x.to(cuda), e.to(cuda), e.to(cuda))
    rel = (psnt.cpu().double() - ref_psnt.double()).abs().max() / ref_psnt.abs().max()
    assert rel.item() < 1e-4
    assert (code.cpu().double() - ref_code.double()).abs().max().item() < 1e-4 * ref_code.abs().max().item()


def test_model_ema_matches_reference_formula(cuda, tmp_path, monkeypatch):
    """solver_encoder.py:168-177: the EMA pass writes ema*p + (1-ema)*p (fp32) over the
    concatenation of G.parameters() back into every parameter, bit for bit."""
    import bench
    x, e = bench.synthetic_batch(4, 128, "cpu", 5)
    monkeypatch.chdir(tmp_path)
    from autovc_amd.solver_encoder import Solver
    s = Solver(_FixedLoader(x, e), _main_config(".", "ema", num_iters=1, log_step=1, ema=0.9999))
    s.G.load_state_dict(og.make_weights())
    with torch.no_grad():
        for p in s.G.parameters():             # non-trivial values everywhere
            p.mul_(1.37)
    flat = torch.cat([p.detach().reshape(-1) for p in s.G.parameters()])
    want = s.ema * flat + (1 - s.ema) * flat
    s.model_EMA()
    got = torch.cat([p.detach().reshape(-1) for p in s.G.parameters()])
    assert torch.equal(got, want)
    assert (got - flat).abs().max().item() <= 2e-7 * flat.abs().max().item()   # ~p, as in the reference


def test_main_py_under_torchrun_trains_data_parallel(cuda, tmp_path):
    """main.py unchanged under torchrun: two ranks sharing cuda:0 over
    gloo (AVC_DIST_BACKEND=gloo; the driver's nodes use RCCL, one GPU per rank) run
    main.py's get_loader + Solver(...).train() with no data-parallel code of their own.
    get_loader shards from RANK/WORLD_SIZE (each rank draws different crops), the Solver
    joins the process group and exchanges gradients, so the ranks' parameters stay
    bit-identical; only rank 0 writes the checkpoint."""
    import json
    import socket
    import subprocess
    main_dir = str(tmp_path / "corpus")
    _corpus(main_dir)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, AVC_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "ddp_main_worker.py"), main_dir,
           str(tmp_path)]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    p = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    info = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    for r in range(2):
        assert info[r]["sampler"] == "SpeakerCropSampler" and info[r]["rank"] == r and info[r]["world"] == 2
        assert info[r]["solver_world"] == 2
    assert info[0]["saves"] == ["chkpnt_spmel_ddpmain.ckpt"] * 2 and info[1]["saves"] == []
    for a, b in zip(*p):
        assert torch.equal(a, b)
    ck = torch.load(tmp_path / "chkpnt_spmel_ddpmain.ckpt", map_location="cpu", weights_only=True)
    assert ck["epoch"] == 4 and all(np.isfinite(v) for v in ck["loss"].values())
