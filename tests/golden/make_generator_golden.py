"""Generates tests/golden/generator_golden.npz by running the REFERENCE code itself
(/root/reference/model_vc_mel.py, model_vc_stft.py and solver_encoder.Solver.train), in the
build container only.  The reference never travels: only the arrays written here do.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_generator_golden.py [--spread | --b64]

Inputs: the bundled spmel crops spmel/p225/p225_003.npy[:128], spmel/p226/p226_003.npy[:128]
(also under tests/golden/frontend/) and the bundled embeddings emb_org_mel.npy (2, 256).
Weights: oracle.generator.deterministic_state_dict (seeded numpy scheme), loaded into the
reference Generator with load_state_dict.  `wandb` / `librosa` are replaced by inert stub
modules (they are only used for logging/plots, solver_encoder.py:10-15,88-98,203,348-421).
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
from oracle.generator import deterministic_state_dict  # noqa: E402

N_SLICE = 64


def _stub_modules():
    class _Any(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("__"):
                raise AttributeError(name)
            return lambda *a, **k: None

    for name in ["wandb", "librosa", "librosa.display", "librosa.feature", "librosa.filters"]:
        sys.modules[name] = _Any(name)
    sys.modules["librosa"].display = sys.modules["librosa.display"]
    sys.modules["librosa"].feature = sys.modules["librosa.feature"]
    sys.modules["librosa"].filters = sys.modules["librosa.filters"]


def main(out_path=os.path.join(HERE, "generator_golden.npz")):
    torch.set_num_threads(8)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _stub_modules()
    sys.path.insert(0, REF)
    import model_vc_mel as ref_mel  # reference
    import model_vc_stft as ref_stft  # reference

    x = np.stack([np.load(os.path.join(REF, "spmel/p225/p225_003.npy"))[:128],
                  np.load(os.path.join(REF, "spmel/p226/p226_003.npy"))[:128]]).astype(np.float32)
    emb = np.load(os.path.join(REF, "emb_org_mel.npy")).astype(np.float32)
    xt, et = torch.from_numpy(x), torch.from_numpy(emb)
    out = {"x": x, "emb": emb}

    # ---- reference Generator, train mode, one Solver-composed step
    G = ref_mel.Generator(32, 256, 512, 32)
    sd = deterministic_state_dict(G.state_dict())
    G.load_state_dict(sd)
    out["keys"] = np.array(list(sd.keys()))
    G.train()
    x_id, x_psnt, code_real = G(xt, et, et)
    l_id = torch.nn.functional.mse_loss(xt.squeeze(), x_id.squeeze())
    l_psnt = torch.nn.functional.mse_loss(xt, x_psnt.squeeze())
    code_rec = G(x_psnt, et, None)
    l_cd = torch.nn.functional.l1_loss(code_real, code_rec)
    g_loss = l_id + l_psnt + l_cd
    out.update(train_x_identic=x_id.detach().numpy(), train_x_psnt=x_psnt.detach().numpy(),
               train_code_real=code_real.detach().numpy(), train_code_reconst=code_rec.detach().numpy(),
               train_losses=np.array([l_id.item(), l_psnt.item(), l_cd.item()]))
    opt = torch.optim.Adam(G.parameters(), 1e-4)
    opt.zero_grad()
    g_loss.backward()
    names = [k for k, _ in G.named_parameters()]
    out["param_names"] = np.array(names)
    out["grad_norm"] = np.array([p.grad.norm().item() for _, p in G.named_parameters()])
    out["grad_slice"] = np.stack([p.grad.detach().flatten()[:N_SLICE].numpy() if p.numel() >= N_SLICE else
                                  np.pad(p.grad.detach().flatten().numpy(), (0, N_SLICE - p.numel()))
                                  for _, p in G.named_parameters()])
    opt.step()
    out["step1_param_slice"] = np.stack([p.detach().flatten()[:N_SLICE].numpy() for _, p in G.named_parameters()])
    bufs = {k: v for k, v in G.state_dict().items() if "running" in k or "num_batches" in k}
    out["step1_buffer_names"] = np.array(list(bufs))
    out["step1_buffers"] = np.concatenate([v.float().flatten().numpy() for v in bufs.values()])

    # ---- eval mode forward with fresh weights (running stats 0/1)
    G2 = ref_mel.Generator(32, 256, 512, 32)
    G2.load_state_dict(sd)
    G2.eval()
    with torch.no_grad():
        e_id, e_psnt, e_code = G2(xt, et, et)
    out.update(eval_x_identic=e_id.numpy(), eval_x_psnt=e_psnt.numpy(), eval_code_real=e_code.numpy())

    # ---- T=160 forward (code width 320), train mode, fresh weights
    G3 = ref_mel.Generator(32, 256, 512, 32)
    G3.load_state_dict(sd)
    x160 = np.stack([np.load(os.path.join(REF, "spmel/p225/p225_003.npy"))[:160],
                     np.load(os.path.join(REF, "spmel/p226/p226_003.npy"))[:160]]).astype(np.float32)
    with torch.no_grad():
        a, b, c = G3(torch.from_numpy(x160), et, et)
    out.update(x160=x160, t160_x_psnt=b.numpy(), t160_code_real=c.numpy())

    # ---- the reference Solver.train itself: 10 iterations on the fixed batch
    import solver_encoder as ref_solver  # reference (wandb/librosa stubbed)
    recorded = []
    orig_mse, orig_l1 = torch.nn.functional.mse_loss, torch.nn.functional.l1_loss

    def rec_mse(a, b, *k, **kw):
        v = orig_mse(a, b, *k, **kw)
        recorded.append(("mse", v.item()))
        return v

    def rec_l1(a, b, *k, **kw):
        v = orig_l1(a, b, *k, **kw)
        recorded.append(("l1", v.item()))
        return v

    cfg = types.SimpleNamespace(main_dir=tempfile.mkdtemp(), lambda_cd=1.0, lambda_SISNR=1.0, dim_neck=32,
                                dim_emb=256, dim_pre=512, freq=32, lr=1e-4, lr_scheduler=None, depth=1,
                                batch_size=2, num_iters=10, ema=0.9999, run_name="golden", resume=False,
                                run_id=None, model_type="spmel", speaker_embed=True, log_step=1000)
    cwd = os.getcwd()
    os.chdir(cfg.main_dir)
    try:
        with open("wandb.token", "w") as f:
            f.write("stub\n")
        solver = ref_solver.Solver([(xt.clone(), et.clone())], cfg)
        solver.G.load_state_dict(sd)
        torch.nn.functional.mse_loss, torch.nn.functional.l1_loss = rec_mse, rec_l1
        solver.train()
    finally:
        torch.nn.functional.mse_loss, torch.nn.functional.l1_loss = orig_mse, orig_l1
        os.chdir(cwd)
    traj = np.array([v for _, v in recorded]).reshape(10, 3)
    out["solver_traj"] = traj

    # ---- 513-bin variant: GeneratorSTFT(...).model arithmetic (model_vc_stft.py:16-29)
    GS = ref_stft.GeneratorSTFT(32, 256, 512, 32)
    sds = deterministic_state_dict(GS.state_dict())
    GS.load_state_dict(sds)
    out["stft_keys"] = np.array(list(sds.keys()))
    rs = np.random.RandomState(7)
    xs = np.clip(rs.normal(0.43, 0.18, (2, 64, 513)), 0, 1).astype(np.float32)
    GS.train()
    with torch.no_grad():
        s_id, s_psnt, s_code = GS.model(torch.from_numpy(xs), et, et)
        s_enc = GS(torch.from_numpy(xs), et, None)
    out.update(stft_x=xs, stft_x_identic=s_id.numpy(), stft_x_psnt=s_psnt.numpy(), stft_code_real=s_code.numpy(),
               stft_encoder_only=s_enc.numpy())
    try:
        GS(torch.from_numpy(xs), et, et)
        out["stft_forward_raises"] = np.array(False)
    except AttributeError:
        out["stft_forward_raises"] = np.array(True)   # F10: GeneratorSTFT.forward is broken

    np.savez_compressed(out_path, **out)
    print("wrote", out_path, {k: getattr(v, "shape", None) for k, v in out.items()})


def _reference_steps(ref_mel, sd, xt, et, dtype, threads, n_steps):
    """The reference Generator + the Solver's loss composition (solver_encoder.py:228-243,
    293-300) + torch Adam, in `dtype` on `threads` intra-op threads.  Returns (per-step
    losses (n,3), first-step gradient slices (n_params, N_SLICE) in float64)."""
    torch.set_num_threads(threads)
    G = ref_mel.Generator(32, 256, 512, 32)
    G.load_state_dict(sd)
    G = G.to(dtype).train()
    x, e = xt.to(dtype), et.to(dtype)
    opt = torch.optim.Adam(G.parameters(), 1e-4)
    hist, gslice = [], None
    for _ in range(n_steps):
        x_id, x_psnt, code = G(x, e, e)
        l_id = torch.nn.functional.mse_loss(x.squeeze(), x_id.squeeze())
        l_psnt = torch.nn.functional.mse_loss(x, x_psnt.squeeze())
        l_cd = torch.nn.functional.l1_loss(code, G(x_psnt, e, None))
        opt.zero_grad()
        (l_id + l_psnt + l_cd).backward()
        if gslice is None:
            gslice = np.stack([np.pad(p.grad.detach().double().flatten()[:N_SLICE].numpy(),
                                      (0, max(0, N_SLICE - p.numel()))) for p in G.parameters()])
        opt.step()
        hist.append([l_id.item(), l_psnt.item(), l_cd.item()])
    return np.array(hist), gslice


def main_spread(out_path=os.path.join(HERE, "generator_spread.npz")):
    """The reference's OWN numerical spread, used to set the trajectory and gradient-slice
    tolerances from evidence instead of by hand:
      traj_f64 / grad_slice_f64 — the reference Generator run in float64 (the closest thing
                                  to the exact answer the reference can give),
      traj_t1                   — the reference in float32 on ONE intra-op thread (the golden
                                  solver_traj ran on 8): same code, another reduction order."""
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _stub_modules()
    sys.path.insert(0, REF)
    import model_vc_mel as ref_mel  # reference
    g = np.load(os.path.join(HERE, "generator_golden.npz"))
    xt, et = torch.from_numpy(g["x"]), torch.from_numpy(g["emb"])
    sd = deterministic_state_dict(ref_mel.Generator(32, 256, 512, 32).state_dict())
    traj_f64, gs64 = _reference_steps(ref_mel, sd, xt, et, torch.float64, 8, 10)
    traj_t1, _ = _reference_steps(ref_mel, sd, xt, et, torch.float32, 1, 10)
    traj_t8, gs32 = _reference_steps(ref_mel, sd, xt, et, torch.float32, 8, 1)
    assert np.array_equal(traj_t8[0], g["solver_traj"][0]) or np.allclose(traj_t8[0], g["solver_traj"][0], rtol=1e-6)
    np.savez_compressed(out_path, traj_f64=traj_f64, traj_t1=traj_t1, grad_slice_f64=gs64,
                        grad_slice_f32_check=gs32)
    print("wrote", out_path)


def main_b64(out_path=os.path.join(HERE, "generator_b64_traj.npz")):
    """The reference at BASELINE config 2's shape (B=64, T=128): the Solver-composed step
    (+ torch Adam) for 10 steps on bench.py's synthetic batch (seed 1234, one
    batch reused every step, as bench.py times it), from the same deterministic weights —
    in float32 on 8 threads (the pin), float64 and float32 on 1 thread (the reference's own
    spread, which sets the tolerance as for the B=2 trajectory).  The batch itself is not
    stored (2.6 MB): its float64 sum and a hash pin that the GPU test regenerated the same
    one."""
    import hashlib
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _stub_modules()
    sys.path.insert(0, REF)
    import model_vc_mel as ref_mel  # reference
    sys.path.insert(0, ROOT)
    import bench
    xt, et = bench.synthetic_batch(64, 128, torch.device("cpu"), 1234)
    sd = deterministic_state_dict(ref_mel.Generator(32, 256, 512, 32).state_dict())
    traj32, _ = _reference_steps(ref_mel, sd, xt, et, torch.float32, 8, 10)
    traj64, _ = _reference_steps(ref_mel, sd, xt, et, torch.float64, 8, 10)
    traj_t1, _ = _reference_steps(ref_mel, sd, xt, et, torch.float32, 1, 10)
    digest = hashlib.sha256(xt.numpy().tobytes() + et.numpy().tobytes()).hexdigest()
    np.savez_compressed(out_path, traj=traj32, traj_f64=traj64, traj_t1=traj_t1, batch_sha256=np.array(digest),
                        x_sum=np.float64(xt.double().sum()), e_sum=np.float64(et.double().sum()))
    print("wrote", out_path, traj32.tolist())


if __name__ == "__main__":
    if "--spread" in sys.argv:
        main_spread()
    elif "--b64" in sys.argv:
        main_b64()
    else:
        main()
