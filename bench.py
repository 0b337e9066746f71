"""AutoVC hot-path benchmark (BASELINE.json metric: mel-frames/sec of the Generator
training step, fwd+bwd, at 1/2/4/8 GPUs).

One "step" = solver_encoder.py's iteration on a B=64 x T=128 x 80-mel synthetic batch
(BASELINE config 2): Generator forward, the second (encoder-only) pass, the three losses,
backward, fused Adam — all on libautovc_hip.so.  N>1: one process per GPU (torchrun),
B=64 per GPU ("weak" scaling), RCCL all-reduce of the flat gradient buffer per step.

Prints ONE JSON line (rank 0).  Extra objects: "roofline" for the recurrent kernel of the
decoder lstm2 (the north-star "LSTM kernel", HBM-bound weight-streaming accounting),
"cpu_baseline" = the oracle's CPU restatement of the same step timed on this host.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def synthetic_batch(B, T, dev, seed):
    """x = clamp(N(0.43, 0.18), 0, 1), emb = N(0,1) rows L2-normalised x 0.8."""
    g = torch.Generator().manual_seed(seed)
    x = torch.clamp(torch.randn(B, T, 80, generator=g) * 0.18 + 0.43, 0, 1)
    g2 = torch.Generator().manual_seed(seed + 1)
    e = torch.randn(B, 256, generator=g2)
    e = e / e.norm(dim=1, keepdim=True) * 0.8
    return x.to(dev), e.to(dev)


def make_solver(dev, B):
    from autovc_amd.solver_encoder import Solver
    cfg = types.SimpleNamespace(main_dir=".", lambda_cd=1.0, lambda_SISNR=1.0, dim_neck=32, dim_emb=256,
                                dim_pre=512, freq=32, lr=1e-4, lr_scheduler=None, depth=1, batch_size=B,
                                num_iters=0, ema=0.9999, run_name="bench", resume=False, run_id=None,
                                model_type="spmel", speaker_embed=True, log_step=100)
    with contextlib.redirect_stdout(sys.stderr):
        return Solver(None, cfg)


def lstm_roofline(solver, B, T, dev):
    """Time the decoder lstm2 layer-0 recurrence kernel per launch (dispatch events) and
    price it with SURVEY §8d's algorithmic bytes per step."""
    from autovc_amd import _lib
    import ctypes
    lstm = solver.G.decoder.lstm2
    H = lstm.hidden_size
    W = lstm.weight_hh_l0.detach()
    g = torch.Generator().manual_seed(7)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    h = torch.empty(B, T, H, device=dev)
    c = torch.empty(B, T, H, device=dev)
    gates = torch.empty(B, T, 4 * H, device=dev)
    avg = ctypes.c_float(0.0)
    samples = []
    for _ in range(3):
        _lib.call("autovc_lstm_fwd_timed_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, W.data_ptr(),
                  h.data_ptr(), T * H, H, c.data_ptr(), gates.data_ptr(), _lib.stream_ptr(dev), ctypes.byref(avg))
        samples.append(avg.value)
    us = sorted(samples)[len(samples) // 2]
    # per step: W_hh (4H x H fp32) + gates_x (B x 4H) + h read, c read+write, h write (B x H each)
    bytes_per_launch = 4 * H * H * 4 + B * 4 * H * 4 + 4 * B * H * 4
    achieved = bytes_per_launch / (us * 1e-6) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "lstm_step_pmc.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    return {"kernel": "lstm_fwd_step_kernel (decoder lstm2, H=1024, B=64)", "bound": "hbm",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": bytes_per_launch, "avg_launch_us": round(us, 3)}


def wavenet_bench(dev, n_utt=8, Tc=128, warmup_steps=256, seconds_cpu=10.0, cpu=True):
    """BASELINE config 4 / SURVEY §8d C4: r9y9 WaveNet (24 layers, 512 residual channels),
    8 utterances x 128 conditioning frames (32,768 samples = 2.048 s each) synthesised in one
    batch.  Timed: the whole job (upsample, per-chunk conditioning GEMM, every sample step
    incl. sampling).  Roofline: weight streaming — every sample step reads the packed
    per-step weights once (98.6 MB fp32)."""
    from autovc_amd import _lib, synthesis
    from autovc_amd.hparams import hparams
    torch.manual_seed(4322)
    model = synthesis.build_model()
    model.make_generation_fast_()
    model = model.to(dev).eval()
    g = torch.Generator().manual_seed(4321)
    c = torch.clamp(torch.randn(n_utt, 80, Tc, generator=g) * 0.18 + 0.43, 0, 1).to(dev)
    T = Tc * hparams.hop_size
    model.generate(c[:, :, : max(1, warmup_steps // hparams.hop_size)], seed=1, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    y = model.generate(c, seed=2, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert y.shape == (n_utt, T) and bool(torch.isfinite(y).all())
    packed = _lib.load().autovc_wavenet_packed_floats(model.layers, model.kernel_size, model.residual_channels,
                                                       model.gate_channels, model.skip_out_channels,
                                                       model.out_channels)
    step_bytes = 4 * packed
    achieved = step_bytes * T / dt / 1e9
    out = {"workload": f"r9y9 WaveNet incremental synthesis, {n_utt} utterances x {T} samples (16 kHz), fp32",
           "samples_per_s": round(n_utt * T / dt, 1), "rtf_aggregate": round(n_utt * T / dt / 16000.0, 3),
           "rtf_per_stream": round(T / 16000.0 / dt, 3), "wall_s": round(dt, 3),
           "us_per_sample_step": round(dt / T * 1e6, 2),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                        "bytes_per_step": step_bytes,
                        "note": "weight-streaming convention: packed per-step weights once per sample step"}}
    if cpu:
        out["cpu_baseline"] = wavenet_cpu_baseline(n_utt, seconds_cpu)
        out["vs_cpu_baseline"] = round(out["samples_per_s"] / out["cpu_baseline"]["value"], 1)
    return out


def wavenet_cpu_baseline(n_utt, seconds):
    """oracle/wavenet.py (fp32 torch CPU ops, the reference's own per-step structure) on a
    bounded number of sample steps of the same batch."""
    from oracle import wavenet as ow
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    hp = ow.HPARAMS
    o = ow.OracleWaveNet(ow.make_weights(hp), hp, dtype=torch.float32)
    g = torch.Generator().manual_seed(4321)
    c = torch.clamp(torch.randn(n_utt, 80, 4, generator=g) * 0.18 + 0.43, 0, 1)
    cu = o.upsample(c)          # 1024 samples: enough for the largest sample below
    steps = 16
    while True:
        u = ow.philox_uniforms(3, list(range(n_utt)), 0, steps)
        t0 = time.perf_counter()
        o.incremental(cu[:, :, :steps], steps, uniforms=u)
        dt = time.perf_counter() - t0
        if dt > seconds / 4 or steps >= 1024:
            break
        steps *= 2
    return {"value": round(n_utt * steps / dt, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{steps} incremental steps x {n_utt} utterances of oracle/wavenet.py (fp32, torch "
                      f"{torch.__version__} CPU, {threads} threads), {dt:.2f} s"}


def cpu_baseline(B, T, seconds=15.0):
    """The oracle's CPU restatement of the same training step (fused torch CPU LSTM, conv1d,
    batch_norm, Adam — the reference's own CPU ops), timed on this host."""
    from oracle import generator as og
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P = og.make_weights()
    params = [v for k, v in P.items() if v.dtype == torch.float32 and "running_" not in k]
    for v in params:
        v.requires_grad_(True)
    opt = torch.optim.Adam(params, 1e-4)
    G = og.OracleGenerator(P, fused_lstm=True)
    x, e = synthetic_batch(B, T, "cpu", 1234)
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        g_loss = og.solver_losses(G, x, e)[0]
        opt.zero_grad()
        g_loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > seconds or len(times) >= 20:
            break
    steady = times[1:] if len(times) > 1 else times
    s = sorted(steady)[len(steady) // 2]
    return {"value": round(B * T / s, 1), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle training steps at B={B}, T={T} (median of steps 2..n, "
                      f"{s:.2f} s/step), torch {torch.__version__} CPU, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-wavenet", action="store_true")
    args = ap.parse_args()

    from autovc_amd import ddp
    rank, world = ddp.init_from_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    B, T = args.batch, args.frames

    solver = make_solver(dev, B)
    if world > 1:
        ddp.make_data_parallel(solver)
    solver.G.train()
    x, e = synthetic_batch(B, T, dev, 1234 + 2 * rank)

    for _ in range(args.warmup):
        solver.train_step(x, e)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = solver.train_step(x, e)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    last_loss = float(losses[0].item())

    roof = None
    if not args.no_roofline and rank == 0:
        roof = lstm_roofline(solver, B, T, dev)
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(B, T)
    wn = None
    if not args.no_wavenet:
        # config 4 per GPU (vocoder batches shard with no collective): every rank synthesises
        # its own 8 utterances; rank 0 reports the per-GPU rate
        wn = wavenet_bench(dev, cpu=(not args.no_cpu_baseline and rank == 0 and world == 1))

    if rank == 0:
        value = world * B * T * args.steps / dt
        line = {
            "metric": "mel-frames/sec Generator fwd+bwd", "value": round(value, 1), "unit": "mel-frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (clamped N(0.43,0.18) mels, unit-norm*0.8 emb)",
            "config": {"workload": "AutoVC Generator training step (solver_encoder.py), fwd+bwd+Adam",
                       "global_batch": B * world, "seq_len": T, "n_mels": 80, "parallelism": f"dp{world}",
                       "dim_neck": 32, "dim_emb": 256, "dim_pre": 512, "freq": 32},
            "final_loss": round(last_loss, 6),
            "roofline": roof, "cpu_baseline": cpu,
            "wavenet": wn,
        }
        if cpu:
            line["vs_cpu_baseline"] = round(value / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
