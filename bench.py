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
MFMA_F32_PEAK_TF = 157.3   # dense fp32 MFMA (= vector) peak (MI355X_MICROARCH.md)


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
    """The dominant LSTM kernel of the forward — decoder lstm2's two-layer recurrence as the
    Generator runs it: the persistent weight-stationary launch (lstm2_persist_kernel, one
    launch per sequence) when functional.lstm2_persistent(B, H), else the per-step wavefront
    launch (lstm2_fwd_step_kernel).  Timed with events on the launch stream; FLOPs = the
    recurrent MACs of both layers (layer 1's input product included), x 2; SURVEY §8d's
    algorithmic bytes per layer-step are reported under 'hbm'.  The per-step launch and the
    single-layer step kernel are reported alongside."""
    from autovc_amd import _lib, functional as AF
    import ctypes
    lstm = solver.G.decoder.lstm2
    H = lstm.hidden_size
    P = {n: getattr(lstm, n).detach() for n in ("weight_hh_l0", "weight_ih_l1", "weight_hh_l1", "bias_ih_l1",
                                                "bias_hh_l1")}
    g = torch.Generator().manual_seed(7)
    gx = (torch.randn(B, T, 4 * H, generator=g) * 0.5).to(dev)
    h0, c0, h1, c1 = (torch.empty(B, T, H, device=dev) for _ in range(4))
    g0, g1 = (torch.empty(B, T, 4 * H, device=dev) for _ in range(2))
    avg = ctypes.c_float(0.0)

    def med(fn):
        xs = []
        for _ in range(3):
            fn()
            xs.append(avg.value)
        return sorted(xs)[1]

    st = _lib.stream_ptr(dev)
    args = [B, T, H, gx.data_ptr(), T * 4 * H, 4 * H, P["weight_hh_l0"].data_ptr(), P["bias_ih_l1"].data_ptr(),
            P["bias_hh_l1"].data_ptr(), P["weight_ih_l1"].data_ptr(), P["weight_hh_l1"].data_ptr(), h0.data_ptr(),
            c0.data_ptr(), g0.data_ptr(), h1.data_ptr(), c1.data_ptr(), g1.data_ptr()]
    us2 = med(lambda: _lib.call("autovc_lstm2_fwd_timed_f32", *args, st, ctypes.byref(avg)))
    us1 = med(lambda: _lib.call("autovc_lstm_fwd_timed_f32", B, T, H, gx.data_ptr(), T * 4 * H, 4 * H,
                                P["weight_hh_l0"].data_ptr(), h0.data_ptr(), T * H, H, c0.data_ptr(), g0.data_ptr(),
                                st, ctypes.byref(avg)))
    # per layer-step: W_hh (4H x H fp32) + gates_x (B x 4H) + h read, c read+write, h write (B x H each)
    per_layer_step = 4 * H * H * 4 + B * 4 * H * 4 + 4 * B * H * 4
    # per wavefront step: layer 0's recurrent product (B x 4H x H) and layer 1's input +
    # recurrent products (B x 4H x 2H), 2 FLOP per MAC
    flop2 = 2 * B * 4 * H * H * 3
    ridge = MFMA_F32_PEAK_TF * 1e12 / (HBM_PEAK_GBS * 1e9)
    step_launch = {"kernel": "lstm2_fwd_step_kernel (per-step wavefront launch)", "avg_launch_us": round(us2, 3),
                   "mfma_frac": round(flop2 / (us2 * 1e-6) / 1e12 / MFMA_F32_PEAK_TF, 4),
                   "hbm_frac": round(2 * per_layer_step / (us2 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    persistent = AF.lstm2_persistent(B, H)
    if persistent:
        ws = torch.empty(_lib.load().autovc_lstm2_persist_workspace_bytes(B, T, H), dtype=torch.uint8, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        xs = []
        for _ in range(4):
            e0.record()
            _lib.call("autovc_lstm2_fwd_persist_f32", *args, ws.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            xs.append(e0.elapsed_time(e1) * 1e3)
        launch_us = sorted(xs[1:])[1]
        flop_launch, bytes_launch = flop2 * T, 2 * per_layer_step * T
        # the default is the row-split kernel (AVC_LSTM2_RS=0: lstm_persist_kernel) in the two-step
        # wavefront form (layer 1 two steps behind layer 0: T + 2 iterations); AVC_LSTM2_LAG2=0
        # selects the one-step form (T + 1)
        lag2 = os.environ.get("AVC_LSTM2_LAG2", "") != "0"
        rs = os.environ.get("AVC_LSTM2_RS", "") != "0"
        iters = T + 2 if lag2 else T + 1
        kname = (f"lstm2_rs_kernel<1024, false, {'true' if lag2 else 'false'}>" if rs else
                 f"lstm_persist_kernel<1024, true, false, {'true' if lag2 else 'false'}>")
        kernel = (f"{kname} (decoder lstm2 forward, both layers, whole sequence per launch, H=1024, B=64"
                  + (", row split" if rs else "") + (", two-step wavefront)" if lag2 else ")"))
        pmc_file = "lstm2_persist_pmc.json"
    else:
        launch_us, flop_launch, bytes_launch = us2, flop2, 2 * per_layer_step
        kernel = "lstm2_fwd_step_kernel (decoder lstm2: both layers per launch, H=1024, B=64)"
        pmc_file = "lstm2_step_pmc.json"
    tf = flop_launch / (launch_us * 1e-6) / 1e12
    achieved = bytes_launch / (launch_us * 1e-6) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", pmc_file)
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    out = {"kernel": kernel, "bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F32_PEAK_TF, "unit": "TFLOP/s",
           "frac": round(tf / MFMA_F32_PEAK_TF, 4), "traffic": traffic,
           "flop_per_launch": flop_launch, "bytes_per_launch": bytes_launch, "avg_launch_us": round(launch_us, 3),
           "arithmetic_intensity": round(flop2 / (2 * per_layer_step), 1), "ridge_flop_per_byte": round(ridge, 1),
           "hbm": {"convention": "SURVEY 8d weight-streaming bytes (W_hh, gates_x, h/c per layer-step), x 2 layers",
                   "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(achieved / HBM_PEAK_GBS, 4)},
           "note": ("bound = mfma: the arithmetic intensity over the 8d algorithmic bytes is above the fp32 ridge "
                    "point (157.3 TF / 8 TB/s), so the fp32 MFMA peak is the roofline; the 8d HBM convention figure "
                    "is reported under 'hbm'.  traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per launch "
                    f"(profiles/{pmc_file})"),
           "step_launch": step_launch,
           "single_layer": {"kernel": "lstm_fwd_step_kernel (H=1024, B=64)", "bytes_per_launch": per_layer_step,
                            "avg_launch_us": round(us1, 3),
                            "hbm_achieved": round(per_layer_step / (us1 * 1e-6) / 1e9, 1),
                            "hbm_frac": round(per_layer_step / (us1 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                            "mfma_frac": round(2 * B * 4 * H * H / (us1 * 1e-6) / 1e12 / MFMA_F32_PEAK_TF, 4)}}
    if persistent:
        out["us_per_wavefront_step"] = round(launch_us / iters, 3)
    return out


def blstm_roofline(dev, B, T, H=32):
    """The encoder BLSTM recurrence (model_vc_mel.py:61,72-73; blstm_fwd/bwd_kernel: one
    launch per layer covers all T steps of both directions) priced with SURVEY §8d's
    formula: per step and direction W_hh (4H x H) + gates_x (B x 4H) + h read, c read+write,
    h write (B x H each) = 82 KB at H=32, B=64 -> x T x 2 directions per launch.  Timed with
    events on the launch stream (one kernel per call), median of 5."""
    from autovc_amd import _lib
    g = torch.Generator().manual_seed(11)
    gx = (torch.randn(B, T, 8 * H, generator=g) * 0.5).to(dev)
    Wf, Wb = ((torch.rand(4 * H, H, generator=g) * 2 - 1).div_(H ** 0.5).to(dev) for _ in range(2))
    h = torch.empty(B, T, 2 * H, device=dev)
    c = torch.empty(B, T, 2 * H, device=dev)
    gates = torch.empty(B, T, 8 * H, device=dev)
    dh = torch.randn(B, T, 2 * H, generator=g).to(dev)
    dG = torch.empty(B, T, 8 * H, device=dev)
    st = _lib.stream_ptr(dev)
    fwd = lambda: _lib.call("autovc_blstm_fwd_f32", B, T, H, 2, gx.data_ptr(), Wf.data_ptr(), Wb.data_ptr(),  # noqa: E731
                            h.data_ptr(), c.data_ptr(), gates.data_ptr(), st)
    bwd = lambda: _lib.call("autovc_blstm_bwd_f32", B, T, H, 2, dh.data_ptr(), gates.data_ptr(), c.data_ptr(),  # noqa: E731
                            Wf.data_ptr(), Wb.data_ptr(), dG.data_ptr(), st)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return sorted(ts)[2]

    per_step_dir = 4 * H * H * 4 + B * 4 * H * 4 + 4 * B * H * 4
    nbytes = per_step_dir * T * 2
    out = {"kernel": f"blstm_fwd_kernel (encoder BLSTM layer, H={H}, B={B}, T={T}, both directions per launch)",
           "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "bytes_per_launch": nbytes,
           "bytes_per_step_direction": per_step_dir, "traffic": None}
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        us = timed(fn)
        a = nbytes / (us * 1e-6) / 1e9
        out[name] = {"avg_launch_us": round(us, 2), "achieved": round(a, 1), "frac": round(a / HBM_PEAK_GBS, 4)}
        pmc = os.path.join(ROOT, "profiles", f"blstm_{name}_pmc.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                out[name]["traffic"] = json.load(f).get("hbm_bytes_per_launch")
    out["achieved"], out["frac"] = out["fwd"]["achieved"], out["fwd"]["frac"]
    out["traffic"] = out["fwd"].get("traffic")
    out["note"] = ("latency-bound: 128 dependent steps per launch; the 82 KB per step-direction the formula "
                   "counts fit in L2/LDS, so HBM never limits this kernel (SURVEY §8d expects << 40 %); "
                   "traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per launch (profiles/blstm_{fwd,bwd}_pmc.json): "
                   "the h/c/gates writes and the gx read, the formula's per-step W_hh/h re-reads stay on chip")
    return out


def gemm_x6_roofline(dev, M=4096, N=1024, K=8192, reps=20):
    """The step's largest GEMM shape (decoder lstm2's dW_hh: 4H x H over K = B*T, both operands
    K-strided, the library's split plan) under precision fp32 on its default X6 kernel and on
    the fp32 MFMA kernel, HIP events over `reps` launches on the launch stream.  X6 issues six
    v_mfma_f32_32x32x16_bf16 per fp32 product: its MFMA roofline is the bf16 dense peak / 6."""
    from autovc_amd import _lib
    st = _lib.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    A = torch.randn(K, M, device=dev, generator=g)
    Bm = torch.randn(K, N, device=dev, generator=g)
    C = torch.zeros(M, N, device=dev)
    out = {}
    prev = _lib.load().autovc_gemm_fp32_x6()
    try:
        for mode in (1, 0):
            _lib.load().autovc_gemm_set_fp32_x6(mode)
            splits = _lib.load().autovc_gemm_f32_splits(M, N, K, 1)
            ws = torch.empty(4 * max(1, _lib.load().autovc_gemm_workspace_floats(M, N, splits)), dtype=torch.uint8,
                             device=dev)

            def launch():
                _lib.call("autovc_gemm_f32", M, N, K, A.data_ptr(), M, 1, 0, 0, 0, Bm.data_ptr(), N, 1, 0, 0, 0,
                          C.data_ptr(), N, 0, 0, 0, splits, ws.data_ptr(), st)
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                launch()
            e1.record()
            torch.cuda.synchronize()
            out[mode] = e0.elapsed_time(e1) / reps * 1e3
    finally:
        _lib.load().autovc_gemm_set_fp32_x6(prev)
    flop = 2.0 * M * N * K
    tf = flop / (out[1] * 1e-6) / 1e12
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "r06", "x6_pmc_dw_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_dispatch")
    return {"kernel": f"gemm_bf16_kernel<256, 128, 16, 64, 64, false, false, true, 0, 0, true> (X6: fp32 GEMM on "
                      f"bf16 planes), LSTM dW {M}x{N}x{K}, both operands K-strided",
            "bound": "mfma", "achieved": round(tf, 1), "unit": "TFLOP/s (fp32-equivalent)",
            "peak": round(2500.0 / 6, 1), "frac": round(tf / (2500.0 / 6), 4), "traffic": traffic,
            "algorithmic_bytes": 4 * (M * K + N * K) + 4 * M * N,
            "traffic_note": "PMC FETCH_SIZE x2 + WRITE_SIZE of the kernel dispatch (2 K splits: its writes are the "
                            "two partial slabs; profiles/r06/x6_pmc_dw_traffic.json, L2 hit 74 %)",
            "avg_launch_us": round(out[1], 1), "fp32_mfma_kernel_us": round(out[0], 1),
            "fp32_mfma_kernel_tf": round(flop / (out[0] * 1e-6) / 1e12, 1),
            "note": "peak = bf16 dense MFMA 2.5 PF / 6 products per fp32 product; MFMA busy 46 % by PMC "
                    "(profiles/r06/x6_pmc_dw_v2.json); the fp32 MFMA kernel's peak is 157.3 TF"}


def step_roofline(B, ms_per_step, precision="fp32"):
    """Whole-step MFMA fraction: algorithmic FLOPs (convs, LSTMs, linear
    fwd + bwd, the second encoder pass; 24.60 GFLOP per sample) / step time / peak."""
    flop = 24.60e9 * B
    peak = MFMA_F32_PEAK_TF if precision == "fp32" else 2500.0
    tf = flop / (ms_per_step * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(tf / peak, 4), "flop_per_step": flop,
            "note": f"{precision} dense MFMA peak (MI355X_MICROARCH.md); FLOPs = 2 x MACs of convs/LSTMs/linear, "
                    "fwd+bwd, both encoder passes (SURVEY §8d C2)" +
                    ("; under fp32 the GEMMs run on the bf16 MFMA units (X6, 'gemm_roofline'), so this "
                     "fp32-equivalent fraction is not bounded by 1" if precision == "fp32" else "")}


def cpu_share():
    """(threads this process may run on, physical cores of the host).  On the GPU box the
    process is given a share of the host (16 CPUs per GPU); os.cpu_count() shows the whole
    machine."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:     # the box's per-job CPU share (16 per GPU)
        allowed = min(allowed, int(env))
    phys = set()
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                phys.add((pid, core))
    except OSError:
        pass
    return allowed, len(phys) or (os.cpu_count() or 1)


def wavenet_bench(dev, n_utt=8, Tc=128, warmup_steps=256, seconds_cpu=20.0, cpu=True):
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
    wn_path_b8 = _wn_path_name(_lib.load().autovc_wavenet_last_path())
    assert y.shape == (n_utt, T) and bool(torch.isfinite(y).all())
    packed = _lib.load().autovc_wavenet_packed_floats(model.layers, model.kernel_size, model.residual_channels,
                                                       model.gate_channels, model.skip_out_channels,
                                                       model.out_channels)
    step_bytes = 4 * packed
    achieved = step_bytes * T / dt / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "wavenet_pmc.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_sample_step")
    out = {"workload": f"r9y9 WaveNet incremental synthesis, {n_utt} utterances x {T} samples (16 kHz), fp32",
           "samples_per_s": round(n_utt * T / dt, 1), "rtf_aggregate": round(n_utt * T / dt / 16000.0, 3),
           "rtf_per_stream": round(T / 16000.0 / dt, 3), "wall_s": round(dt, 3),
           "us_per_sample_step": round(dt / T * 1e6, 2),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "bytes_per_step": step_bytes,
                        "note": "weight-streaming convention: packed per-step weights once per sample step "
                                "(SURVEY 8d); traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per sample step of the "
                                "generation kernel (profiles/wavenet_pmc.json, tools/gpu_r06_prof.sh wnpmc): the "
                                "layer-pipelined kernel keeps the current-tap and residual rows on chip and moves "
                                "the past-tap weights once per 4 utterances, so the step is bound by its 26 "
                                "dependent hand-offs, not by HBM"}}
    # the reference's own call shape: wavegen synthesises ONE utterance at a time
    # (synthesis.py:58-69); 32 conditioning frames = 8,192 samples of one stream
    c1 = c[:1, :, :32].contiguous()
    model.generate(c1[:, :, :1], seed=1, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    y1 = model.generate(c1, seed=5, log_scale_min=hparams.log_scale_min)
    torch.cuda.synchronize()
    d1 = time.perf_counter() - t0
    n1 = c1.shape[2] * hparams.hop_size
    assert y1.shape == (1, n1) and bool(torch.isfinite(y1).all())
    out["b1"] = {"workload": f"1 utterance x {n1} samples (wavegen's batch of one)",
                 "us_per_sample_step": round(d1 / n1 * 1e6, 2), "samples_per_s": round(n1 / d1, 1),
                 "rtf": round(n1 / 16000.0 / d1, 3),
                 "path": _wn_path_name(_lib.load().autovc_wavenet_last_path())}
    out["path"] = wn_path_b8
    if cpu:
        out["cpu_baseline"] = wavenet_cpu_baseline(n_utt, seconds_cpu)
        out["vs_cpu_baseline"] = round(out["samples_per_s"] / out["cpu_baseline"]["value"], 1)
    return out


def _wn_path_name(p):
    return {0: "per-layer launches (hipGraph replay)",
            1: "wn_grid_kernel (all-CU weight-resident dataflow, one launch per call)",
            2: "wn_pipe_kernel (layer-pipelined weight-resident chain, one launch per call)"}.get(p, str(p))


def wavenet_cpu_baseline(n_utt, seconds, steps=512, min_passes=7):
    """oracle/wavenet.py (fp32 torch CPU ops, the reference's own per-step structure): after a
    short warm-up pass, passes of `steps` incremental sample steps of the same batch are timed
    until `seconds` have elapsed (at least `min_passes`); the value is the MEDIAN pass's rate
    (a single pass swung 1.1k-1.5k samples/s between identical runs; with 3-5
    passes over 12 s three round-6 runs on different boxes read 1,367-1,539, hence >= 7 passes
    over >= 20 s)."""
    from oracle import wavenet as ow
    threads, _ = cpu_share()
    torch.set_num_threads(threads)
    hp = ow.HPARAMS
    o = ow.OracleWaveNet(ow.make_weights(hp), hp, dtype=torch.float32)
    g = torch.Generator().manual_seed(4321)
    c = torch.clamp(torch.randn(n_utt, 80, 4, generator=g) * 0.18 + 0.43, 0, 1)
    cu = o.upsample(c)          # 1024 samples: enough for the passes below
    u = ow.philox_uniforms(3, list(range(n_utt)), 0, steps)
    o.incremental(cu[:, :, :32], 32, uniforms=ow.philox_uniforms(3, list(range(n_utt)), 0, 32))   # warm-up
    rates = []
    t_start = time.perf_counter()
    while len(rates) < min_passes or time.perf_counter() - t_start < seconds:
        t0 = time.perf_counter()
        o.incremental(cu[:, :, :steps], steps, uniforms=u)
        rates.append(n_utt * steps / (time.perf_counter() - t0))
    rates.sort()
    med = rates[len(rates) // 2]
    return {"value": round(med, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"median of {len(rates)} passes of {steps} incremental steps x {n_utt} utterances of "
                      f"oracle/wavenet.py (fp32, torch {torch.__version__} CPU, {threads} threads), "
                      f"{time.perf_counter() - t_start:.1f} s; pass rates {rates[0]:.0f}-{rates[-1]:.0f} samples/s"}


def synthetic_wavs(n, base_index, seed=5000):
    """per utterance a seeded sum of 3 sinusoids (100-4000 Hz, amplitude
    <= 0.3 each) + N(0, 0.01), clipped to +-0.99; 2-4 s long, cut so that the frame count
    (L//256 + 1) is a multiple of 32 (no conversion padding)."""
    import numpy as np
    out = []
    for i in range(n):
        rs = np.random.RandomState(seed + base_index + i)
        frames = 32 * rs.randint(4, 8)                     # 128..224 frames = 2.0..3.6 s
        L = (frames - 1) * 256 + int(rs.randint(0, 256))
        t = np.arange(L) / 16000.0
        w = sum(rs.uniform(0.05, 0.3) * np.sin(2 * np.pi * rs.uniform(100, 4000) * t + rs.uniform(0, 6.3))
                for _ in range(3))
        w = w + rs.normal(0, 0.01, L)
        out.append(np.clip(w, -0.99, 0.99))
    return out


def frontend_roofline(dev, n_utt=256):
    """The fused STFT+mel kernel on a large batch (n_utt synthetic utterances, spmel and
    513-bin stft modes), one launch each, timed with events on the launch stream.
    Algorithmic bytes per frame: 256 new float64 samples in (the reference's filtfilt/dither
    output is float64, make_spect.py:74-76) + the float32 row out (80 or 513 values)."""
    from autovc_amd import _lib, dsp
    import numpy as np
    wavs = synthetic_wavs(n_utt, 100000)
    lens = [len(w) for w in wavs]
    fr_each = [dsp.n_frames(n) for n in lens]
    fr = int(sum(fr_each))
    wav = torch.from_numpy(np.concatenate(wavs).astype(np.float64)).to(dev)
    woff = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int64, device=dev)
    foff = torch.tensor(np.concatenate([[0], np.cumsum(fr_each)]), dtype=torch.int64, device=dev)
    lo, ln, off, w = dsp._DeviceMel.get(dev, 80)
    res = {}
    for mode, width in (("spmel", 80), ("stft", 513)):
        out = torch.empty((fr, width), dtype=torch.float32, device=dev)
        args = (_lib.ptr(wav), _lib.ptr(woff), _lib.ptr(foff), n_utt, fr,
                *((_lib.ptr(lo), _lib.ptr(ln), _lib.ptr(off), _lib.ptr(w), 80, 0) if mode == "spmel"
                  else (0, 0, 0, 0, 0, 1)), _lib.ptr(out), _lib.stream_ptr(dev))
        _lib.call("autovc_stft_mel_f32", *args)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):   # one launch per sample, events on the launch stream
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.call("autovc_stft_mel_f32", *args)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        dt = sorted(ts)[2]
        bpf = 256 * 8 + width * 4
        res[mode] = {"frames": fr, "kernel_ms": round(dt * 1e3, 3), "frames_per_s": round(fr / dt, 1),
                     "bytes_per_frame": bpf, "achieved": round(fr * bpf / dt / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(fr * bpf / dt / 1e9 / HBM_PEAK_GBS, 4)}
    # filtfilt + dither (make_spect.py:74-76) of the same batch, one RandomState per
    # utterance: latency-bound (a sequential IIR per utterance, bit-exact with scipy), so
    # the figure is samples/s with all utterances in flight, not a bandwidth fraction.
    ns = int(sum(lens))
    seeds = list(range(n_utt))
    dsp.preprocess_gpu(wavs, seeds=seeds, device=dev)          # the API path (incl. host->device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dsp.preprocess_gpu(wavs, seeds=seeds, device=dev)
    torch.cuda.synchronize()
    dwall = time.perf_counter() - t0
    # the two kernels alone on device-resident input, events on the launch stream
    b, a, zi = dsp._filter_consts()
    soff = woff
    sd = torch.arange(n_utt, dtype=torch.int32, device=dev)
    pre = torch.empty(ns, dtype=torch.float64, device=dev)
    pargs = (_lib.ptr(wav), 1, _lib.ptr(woff), n_utt, b.ctypes.data, a.ctypes.data, zi.ctypes.data, dsp.ORDER,
             _lib.ptr(soff), _lib.ptr(sd), n_utt, _lib.ptr(pre), _lib.stream_ptr(dev))
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("autovc_preprocess_f64", *pargs)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    dt = sorted(ts)[1]
    n_cpu = 16
    t0 = time.perf_counter()
    for i in range(n_cpu):
        fe_oracle_preprocess(wavs[i], np.random.RandomState(i))
    dcpu = time.perf_counter() - t0
    ns_cpu = int(sum(lens[:n_cpu]))
    res["preprocess"] = {"utterances": n_utt, "samples": ns, "kernel_ms": round(dt * 1e3, 3),
                         "samples_per_s": round(ns / dt, 1), "wall_ms_incl_h2d": round(dwall * 1e3, 3),
                         "bound": "latency (sequential IIR per utterance)",
                         "cpu_baseline": {"value": round(ns_cpu / dcpu, 1), "unit": "samples/s", "cores": 1,
                                          "kind": "reference",
                                          "sample": f"scipy.signal.filtfilt + RandomState.rand on {n_cpu} "
                                                    f"utterances ({ns_cpu} samples), the reference's own host code"}}
    return res


def fe_oracle_preprocess(w, prng):
    from oracle import frontend as fe
    return fe.preprocess(w, prng)


def e2e_bench(dev, rank, world, per_rank=8):
    """BASELINE config 5 / SURVEY §8d C5: 64 synthetic utterances sharded 8 per GPU; GPU
    filtfilt + dither -> GPU 513-bin STFT -> GeneratorSTFT conversion (eval) -> projection
    to 80 mels (conversion.py:102) -> batched WaveNet synthesis.  Random-init weights (the
    reference checkpoints are absent).  The spectrogram stage includes the GPU filtfilt +
    dither (autovc_preprocess_f64).  Timed per stage with the device synchronised."""
    import numpy as np
    from autovc_amd import pipeline, synthesis
    from autovc_amd.model_vc_stft import GeneratorSTFT
    torch.manual_seed(77)
    G = GeneratorSTFT(32, 256, 512, 32).to(dev).eval()
    voc = synthesis.build_model()
    voc.make_generation_fast_()
    voc = voc.to(dev).eval()
    base = rank * per_rank
    wavs = synthetic_wavs(per_rank, base)
    g = torch.Generator().manual_seed(6000 + base)
    e = torch.randn(2 * per_rank, 256, generator=g)
    e = (e / e.norm(dim=1, keepdim=True) * 0.8).to(dev)
    e_org, e_trg = e[:per_rank], e[per_rank:]
    # warm-up on a short utterance pair (kernels loaded, graphs captured)
    w0 = [wavs[0][: 127 * 256 + 10]]
    m0 = pipeline.convert(G, pipeline.spectrograms(w0, "stft", device=dev, seeds=[base]), e_org[:1], e_trg[:1])
    synthesis.wavegen_batch(voc, [m0[0][:4].cpu().numpy()], seed=1, utt_offset=base)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    specs = pipeline.spectrograms(wavs, "stft", device=dev, seeds=[base + i for i in range(per_rank)])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    mels = pipeline.convert(G, specs, e_org, e_trg)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    waves = synthesis.wavegen_batch(voc, [m.cpu().numpy() for m in mels], seed=3, utt_offset=base)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    stages = torch.tensor([t1 - t0, t2 - t1, t3 - t2, t3 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.all_reduce(stages, op=torch.distributed.ReduceOp.MAX)
    s = [float(v) for v in stages.cpu()]
    audio_s = sum(len(w) for w in waves) / 16000.0
    assert all(len(w) == m.shape[0] * 256 and np.isfinite(w).all() for w, m in zip(waves, mels))
    n_total = per_rank * world
    return {"workload": f"C5: {n_total} synthetic utterances ({per_rank} per GPU, 2.0-3.6 s), HIP filtfilt+dither "
                        "-> HIP 513-bin STFT -> GeneratorSTFT conversion -> mel projection -> WaveNet",
            "utterances_per_s": round(n_total / s[3], 3), "rtf_node": round(audio_s * world / s[3], 3),
            "rank0_audio_s": round(audio_s, 2),
            "stage_s_max_over_ranks": {"spectrograms": round(s[0], 4), "convert": round(s[1], 4),
                                       "vocode": round(s[2], 3), "total": round(s[3], 3)}}


def cpu_baseline(B, T, seconds=15.0):
    """The oracle's CPU restatement of the same training step (fused torch CPU LSTM, conv1d,
    batch_norm, Adam — the reference's own CPU ops), timed on this host on every CPU this
    process may use (the GPU box gives a job a 16-CPU share of the host; the host's
    physical core count is stated beside it).  Also the BASELINE config-1 shape (B=2)."""
    threads, phys = cpu_share()
    torch.set_num_threads(threads)
    out = _cpu_step(B, T, threads, seconds)
    out["host_physical_cores"] = phys
    c1 = _cpu_step(2, T, threads, seconds / 3)
    out["c1"] = {"value": c1["value"], "unit": "mel-frames/s", "cores": threads, "kind": "port",
                 "sample": c1["sample"].replace("oracle training steps", "oracle training steps (BASELINE config 1 "
                                                "shape: batch 2)")}
    return out


def _cpu_step(B, T, threads, seconds):
    from oracle import generator as og
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


def spawn_ranks(n):
    """Run this script as n ranks of one node (torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1) and return the worst exit status.  Called before anything
    initialises HIP in this process (importing torch does not)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


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
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="issue the step eagerly instead of replaying the captured HIP graph")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32",
                    help="precision of the headline measurement (default fp32 = BASELINE config 2)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` outside torchrun: start the N ranks here, before this
        # process touches the GPU, and exit with their status (rank 0 prints the line)
        sys.exit(spawn_ranks(args.gpus))

    # test hook (tests/test_bench_multirank, 1-GPU boxes): every rank on cuda:0 over gloo, to
    # exercise the N > 1 flow (sharding, barriers, max-over-ranks timing) without 2 GPUs.
    # Every persistent kernel (lstm2 forward, XCD-local lstm1 forward / backward, the opt-in
    # single-layer persistent forward) needs every CU to itself (all 256 workgroups
    # co-resident, INTEGRATION.md "Co-residency"): two processes' grids on one device could
    # each hold part of the chip, so ranks sharing a device use the per-step launches.
    share = os.environ.get("AVC_BENCH_SHARE_DEVICE") == "1"
    if share:
        for k in ("AVC_LSTM2_PERSIST", "AVC_LSTM_XCD", "AVC_LSTM_PERSIST", "AVC_WN_GRID"):
            os.environ[k] = "0"
    from autovc_amd import ddp
    rank, world = ddp.init_from_env(backend="gloo" if share else None)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s)", file=sys.stderr)
        sys.exit(3)
    local = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    B, T = args.batch, args.frames

    # world > 1: the Solver joins the process group and attaches the gradient exchange
    # itself (ddp.make_data_parallel, grad_dtype "auto": fp32 for the fp32 headline = config 2
    # numerics, bf16 with fp32 accumulation while the bf16 object runs = config 3)
    solver = make_solver(dev, B)
    assert world == 1 or solver.world == world
    solver.G.train()
    solver.precision = args.precision
    solver.hip_graph = not args.no_graph
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
    from autovc_amd import functional as AF
    AF.check_device_faults(dev)      # a co-residency failure of a persistent launch raises here
    rank_ms = [round(dt / args.steps * 1000, 3)]
    if world > 1:
        # every rank's own time (the line reports them) and the max over ranks (the value)
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        ts = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(ts, t)
        rank_ms = [round(float(x.item()) / args.steps * 1000, 3) for x in ts]
        dt = max(float(x.item()) for x in ts)
    last_loss = float(losses[0].item())

    def timed_steps(n):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t_0 = time.perf_counter()
        for _ in range(n):
            out = solver.train_step(x, e)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        d = time.perf_counter() - t_0
        if world > 1:
            tt = torch.tensor([d], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            d = float(tt.item())
        return d, out

    bf = None
    if not args.no_bf16 and args.precision == "fp32":
        # BASELINE config 3 numerics (bf16 matmul operands, fp32 master/optimizer/BN/loss),
        # same solver and batch, after the fp32 measurement
        solver.precision = "bf16"
        timed_steps(max(2, args.warmup // 2))
        dtb, lb = timed_steps(args.steps)
        AF.check_device_faults(dev)
        solver.precision = args.precision
        bf = {"value": round(world * B * T * args.steps / dtb, 1), "unit": "mel-frames/s",
              "ms_per_step": round(dtb / args.steps * 1000, 3), "dtype": "bf16 MFMA operands, fp32 accumulate",
              "final_loss": round(float(lb[0].item()), 6),
              "grad_exchange": None if world == 1 else "bf16 all-to-all + fp32 shard sums + bf16 all-gather",
              "note": "BASELINE config 3 precision; the headline value above is config 2 (fp32)"}

    f32m = None
    if not args.no_bf16 and args.precision == "fp32":
        # the same fp32 step with the GEMMs on fp32 MFMA instead of the default three-plane bf16
        # split (both fp32-accurate: tests/test_gemm_x6_gpu.py), for comparison
        prev = AF.set_fp32_gemm("mfma")
        try:
            timed_steps(max(2, args.warmup // 2))
            dtm, lm = timed_steps(args.steps)
            AF.check_device_faults(dev)
        finally:
            AF.set_fp32_gemm(prev)
        f32m = {"value": round(world * B * T * args.steps / dtm, 1), "unit": "mel-frames/s",
                "ms_per_step": round(dtm / args.steps * 1000, 3), "final_loss": round(float(lm[0].item()), 6),
                "note": "precision fp32 with every GEMM on v_mfma_f32_32x32x2_f32 (AVC_FP32_X6=0)"}

    roof = blstm = groof = None
    if not args.no_roofline and rank == 0:
        roof = lstm_roofline(solver, B, T, dev)
        blstm = blstm_roofline(dev, B, T)
        groof = gemm_x6_roofline(dev)
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(B, T)
    wn = None
    if not args.no_wavenet:
        # config 4 per GPU (vocoder batches shard with no collective): every rank synthesises
        # its own 8 utterances; rank 0 reports the per-GPU rate
        wn = wavenet_bench(dev, cpu=(not args.no_cpu_baseline and rank == 0 and world == 1))
    e2e = fe = None
    if not args.no_e2e:
        e2e = e2e_bench(dev, rank, world)
        if rank == 0:
            fe = frontend_roofline(dev)

    if rank == 0:
        value = world * B * T * args.steps / dt
        line = {
            "metric": "mel-frames/sec Generator fwd+bwd", "value": round(value, 1), "unit": "mel-frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else "bf16", "data": "synthetic (clamped N(0.43,0.18) mels, unit-norm*0.8 emb)",
            "fp32_gemm": (AF.fp32_gemm_mode() + (": fp32 operands split exactly into three bf16 planes, six bf16 MFMA "
                          "products per pair in two fp32 accumulators (error vs fp64 <= the fp32-MFMA kernel's)"
                          if AF.fp32_gemm_mode() == "x6" else ": v_mfma_f32_32x32x2_f32"))
            if args.precision == "fp32" else None,
            "dist_backend": torch.distributed.get_backend() if world > 1 else None,
            "world_size": torch.distributed.get_world_size() if world > 1 else 1,
            "rank_ms_per_step": rank_ms,
            "config": {"workload": "AutoVC Generator training step (solver_encoder.py), fwd+bwd+Adam",
                       "global_batch": B * world, "seq_len": T, "n_mels": 80, "parallelism": f"dp{world}",
                       "hip_graph": not args.no_graph,
                       "dim_neck": 32, "dim_emb": 256, "dim_pre": 512, "freq": 32},
            "final_loss": round(last_loss, 6),
            "roofline": roof, "blstm_roofline": blstm, "gemm_roofline": groof,
            "step_roofline": step_roofline(B, dt / args.steps * 1000, args.precision),
            "cpu_baseline": cpu, "bf16": bf, "fp32_mfma": f32m,
            "wavenet": wn,
            "e2e": e2e, "frontend": fe,
        }
        if cpu:
            line["vs_cpu_baseline"] = round(value / cpu["value"], 2)
            line["vs_cpu_baseline_c1"] = round(value / cpu["c1"]["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
