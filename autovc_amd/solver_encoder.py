"""Solver — reference solver_encoder.py's training driver on MI355X.

Same class, constructor (vcc_loader, config), attributes (G, g_optimizer, lr_scheduler,
device, ...), methods (build_model, reset_grad, model_EMA, train) and checkpoint dict
({'epoch', 'state_dict', 'optimizer', 'loss'}, file chkpnt_<model_type>_<run_name>.ckpt)
as solver_encoder.py:52-421, so main.py runs unchanged.  The step itself
(solver_encoder.py:226-300) is `train_step`, which runs entirely on the GPU: Generator
fwd/bwd on the HIP kernels, losses on device (no .item() sync per iteration: loss values
are read only when they are logged), fused flat-buffer Adam.

Deliberate differences (DESIGN.md "Reference quirks"):
  * no CPU fallback: the product path needs the GPU (the reference trains on CPU when
    CUDA is absent, solver_encoder.py:101-109);
  * wandb is optional (logging only, solver_encoder.py:88-98,203,415-421): used when the
    module is importable and a 'wandb.token' file exists, otherwise skipped;
  * the lr-scheduler branch steps the scheduler that was built ('Cosine' -> .step(),
    'Plateau' -> .step(loss)); the reference compares the scheduler object to the string
    'Cosine' (solver_encoder.py:304) and so always takes the Plateau call;
  * model_type 'stft' trains GeneratorSTFT (whose reference forward raises, F10) and
    'wav' (ConvTasNet generator) is out of scope.
"""
from __future__ import annotations

import datetime
import os
import time

import torch

from . import functional as AF
from .model_vc_mel import Generator
from .model_vc_stft import GeneratorSTFT
from .optim import FusedAdam


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


class _NoLogger:
    def log(self, *a, **k):
        pass

    def watch(self, *a, **k):
        pass


def _make_logger(config, resume_exists):
    if not os.path.exists("wandb.token"):
        return _NoLogger()
    try:
        import wandb
    except ImportError:
        return _NoLogger()
    with open("wandb.token") as f:
        wandb.login(key=f.readline())
    if resume_exists:
        wandb.init(project="DNS autovc", entity="macaroni", config=config, reinit=True, id=config.run_id, resume=True)
    else:
        wandb.init(project="DNS autovc", entity="macaroni", config=config, reinit=True, name=config.run_name)
    return wandb


class Solver(object):

    def __init__(self, vcc_loader, config):
        self.main_dir = getattr(config, "main_dir", ".")
        self.vcc_loader = vcc_loader
        self.lambda_cd = config.lambda_cd
        self.lambda_SISNR = getattr(config, "lambda_SISNR", 1.0)
        self.dim_neck = config.dim_neck
        self.dim_emb = config.dim_emb
        self.dim_pre = config.dim_pre
        self.freq = config.freq
        self.lr = config.lr
        self.lr_scheduler = getattr(config, "lr_scheduler", None)
        self.depth = getattr(config, "depth", 1)
        self.batch_size = config.batch_size
        self.num_iters = config.num_iters
        self.ema = config.ema
        self.run_name = config.run_name
        self.resume = getattr(config, "resume", False)
        self.run_id = getattr(config, "run_id", None)
        self.model_type = config.model_type
        self.speaker_embed = getattr(config, "speaker_embed", True)
        self.log_step = config.log_step
        # matmul precision of the step: "fp32" (BASELINE config 2) or "bf16" (config 3:
        # bf16 MFMA operands, fp32 master weights / Adam / BN / losses); not in the reference
        self.precision = getattr(config, "precision", "fp32")
        # replay the forward+backward as a captured HIP graph (autovc_amd.graph); not in the
        # reference.  Inputs of a new shape or precision capture a new graph.
        self.hip_graph = bool(getattr(config, "hip_graph", False))
        self._graphs = None

        self.path = "chkpnt_" + self.model_type + "_" + self.run_name + ".ckpt"
        self.file_exists = os.path.exists(self.path)

        if not torch.cuda.is_available():
            raise RuntimeError("autovc_amd.Solver trains on the MI355X only (no CPU fallback)")
        # data parallel under a launcher (torchrun: WORLD_SIZE > 1): one process per GPU, the
        # process group is created here (RCCL, device = LOCAL_RANK) so that main.py's
        # unchanged `Solver(vcc_loader, config).train()` (main.py:39-40) trains on every rank
        # with the gradient exchange of autovc_amd.ddp; get_loader shards from the same env
        from . import ddp
        self.world = ddp.init_from_env()[1]
        self.logger = _make_logger(config, self.file_exists) if _rank() == 0 else _NoLogger()
        self.device = torch.device("cuda", torch.cuda.current_device())
        print("Training on GPU.")
        self.build_model()
        if self.world > 1:
            ddp.make_data_parallel(self)      # rank 0's weights everywhere, then bucketed exchange

    def build_model(self):
        if self.model_type == "spmel":
            self.G = Generator(self.dim_neck, self.dim_emb, self.dim_pre, self.freq)
        elif self.model_type == "stft":
            self.G = GeneratorSTFT(self.dim_neck, self.dim_emb, self.dim_pre, self.freq)
        elif self.model_type == "wav":
            raise NotImplementedError("model_type 'wav' (ConvTasNet generator) is out of scope (DESIGN.md)")
        else:
            raise ValueError("Model type not recognized")
        self.G.to(self.device)
        if self.file_exists:
            print("Loading checkpoint: " + self.path)
            checkpoint = torch.load(self.path, map_location=self.device, weights_only=True)
            self.G.load_state_dict(checkpoint["state_dict"])
        self.g_optimizer = FusedAdam(filter(lambda p: p.requires_grad, self.G.parameters()), self.lr)
        if self.lr_scheduler == "Cosine":
            self.lr_scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(self.g_optimizer, T_max=10000, eta_min=0)
        elif self.lr_scheduler == "Plateau":
            self.lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.g_optimizer, "min")
        else:
            print("No learning rate scheduler used.")
            self.lr_scheduler = None
        if self.file_exists:
            self.g_optimizer.load_state_dict(checkpoint["optimizer"])
            self.i = checkpoint["epoch"]
            self.loss = checkpoint["loss"]

    def reset_grad(self):
        self.g_optimizer.zero_grad()

    def model_EMA(self):
        """solver_encoder.py:168-177 (ema*p + (1-ema)*p: numerically ~p, kept as is)."""
        with torch.no_grad():
            for flat in self.g_optimizer.flat_params():
                flat.copy_(self.ema * flat + (1 - self.ema) * flat)

    # ------------------------------------------------------------------ one iteration
    def compute_losses(self, x_real, emb_org):
        """solver_encoder.py:226-243 (spmel / stft branch) -> (g_loss, id, id_psnt, cd)."""
        x_identic, x_identic_psnt, code_real = self.G(x_real, emb_org, emb_org)
        g_loss_id = AF.mse_loss(x_real.squeeze(), x_identic.squeeze())
        g_loss_id_psnt = AF.mse_loss(x_real, x_identic_psnt.squeeze())
        code_reconst = self.G(x_identic_psnt, emb_org, None)
        g_loss_cd = AF.l1_loss(code_real, code_reconst)
        g_loss = g_loss_id + g_loss_id_psnt + self.lambda_cd * g_loss_cd
        return g_loss, g_loss_id, g_loss_id_psnt, g_loss_cd, x_identic_psnt

    def _forward_backward(self, x_real, emb_org):
        # the weights do not change until the optimizer step: each conv weight transform is
        # computed once per step (AF.weight_scope)
        if AF.MARKS.active:     # data parallel: gradient-ready marks for the exchange (ddp)
            AF.MARKS.begin()
        with AF.precision(self.precision), AF.weight_scope():
            g_loss, l_id, l_psnt, l_cd, x_psnt = self.compute_losses(x_real, emb_org)
            self.reset_grad()
            g_loss.backward()
        AF.join_grad_stream()   # weight gradients (side stream) complete before they are read
        if AF.MARKS.active:
            AF.MARKS.final(x_real.device)
        return g_loss, l_id, l_psnt, l_cd, x_psnt

    def train_step(self, x_real, emb_org):
        """Losses, zero_grad, backward, Adam (solver_encoder.py:226-300).  Returns device
        scalars (g_loss, loss_id, loss_id_psnt, loss_cd); nothing synchronises.  With
        `hip_graph` the forward+backward is a graph replay (its outputs are the graph's
        static tensors, overwritten by the next step)."""
        # the captured step replays bit-identically to eager with the weight-gradient side
        # stream on and off (tests/test_solver_gpu.py::test_hip_graph_replays_without_host_sync)
        if self.hip_graph:
            if self._graphs is None:
                from .graph import StepGraphs
                self._graphs = StepGraphs(self._forward_backward, self.G)
            # the fp32 GEMM mode (X6 / fp32 MFMA) selects other kernels: a graph of its own
            key = (self.precision, AF.fp32_gemm_mode())
            g_loss, l_id, l_psnt, l_cd, x_psnt = self._graphs.run(key, x_real, emb_org)
        else:
            g_loss, l_id, l_psnt, l_cd, x_psnt = self._forward_backward(x_real, emb_org)
        self._after_backward()
        self._optimizer_step()
        self._last_psnt = x_psnt
        return g_loss, l_id, l_psnt, l_cd

    def _after_backward(self):
        """Hook for data-parallel gradient reduction (autovc_amd.ddp)."""
        return None

    def _optimizer_step(self):
        """Adam (solver_encoder.py:300); autovc_amd.ddp replaces it by the bucketed
        all-reduce interleaved with per-bucket updates."""
        self.g_optimizer.step()

    # ------------------------------------------------------------------ loop
    def train(self):
        data_loader = self.vcc_loader
        lr = self.lr
        keys = ["G/loss_id", "G/loss_id_psnt", "G/loss_cd"]
        if self.file_exists:
            i_start = self.i
            print("Continue from iteration: ", i_start)
        else:
            i_start = 0
        print("Starting training...")
        start_time = time.time()
        self.G.train()
        self.logger.watch(self.G, log=None)
        data_iter = None
        epoch = 0
        for i in range(i_start, self.num_iters):
            try:
                x_real, emb_org = next(data_iter)
            except Exception:  # reference: bare except re-creates the iterator (:212-216)
                sampler = getattr(data_loader, "sampler", None)
                if hasattr(sampler, "set_epoch"):   # data-parallel sampler: reshuffle per epoch
                    sampler.set_epoch(epoch)
                epoch += 1
                data_iter = iter(data_loader)
                x_real, emb_org = next(data_iter)
            x_real = x_real.to(self.device, non_blocking=True)
            emb_org = emb_org.to(self.device, non_blocking=True)

            if self.model_type not in ("spmel", "stft"):
                raise ValueError("Model type not recognized")
            g_loss, g_loss_id, g_loss_id_psnt, g_loss_cd = self.train_step(x_real, emb_org)

            if self.lr_scheduler is not None:
                if isinstance(self.lr_scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                    self.lr_scheduler.step(g_loss.item())
                else:
                    self.lr_scheduler.step()
                lr = self.g_optimizer.param_groups[0]["lr"]
                print("The current convtas learning rate:", lr)

            if (i + 1) % self.log_step == 0:
                AF.check_device_faults(self.device)   # raises if a persistent launch failed
                loss = {"G/loss_id": g_loss_id.item(), "G/loss_id_psnt": g_loss_id_psnt.item(),
                        "G/loss_cd": g_loss_cd.item()}
                self.loss = loss
                et = time.time() - start_time
                et = str(datetime.timedelta(seconds=et))[:-7]
                log = "Elapsed [{}], Iteration [{}/{}]".format(et, i + 1, self.num_iters)
                for tag in keys:
                    log += ", {}: {:.4f}".format(tag, loss[tag])
                self.model_EMA()
                state = {"epoch": i + 1, "state_dict": self.G.state_dict(),
                         "optimizer": self.g_optimizer.state_dict(), "loss": loss}
                if self.file_exists:
                    save_name = "chkpnt_" + self.model_type + "_" + self.run_name + "_resumed.ckpt"
                else:
                    save_name = "chkpnt_" + self.model_type + "_" + self.run_name + ".ckpt"
                # data-parallel: the ranks hold identical weights; only rank 0 writes the file
                # and logs, and every rank waits until it is complete (a resume reads it)
                rank0 = _rank() == 0
                if rank0:
                    torch.save(state, save_name)
                    self.logger.log({"i": i, "lr": lr, "g_loss": g_loss.item(), "g_loss_id": loss["G/loss_id"],
                                     "g_loss_id_psnt": loss["G/loss_id_psnt"], "g_loss_cd": loss["G/loss_cd"],
                                     "g_loss_SISNR": float("nan")})
                _barrier()
        AF.check_device_faults(self.device)
        return self
