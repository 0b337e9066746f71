"""One rank of tests/test_training_flow_gpu.py::test_main_py_under_torchrun_trains_data_parallel
(not a test module): main.py:36-40's calls through compat/ with NO data-parallel code of
its own — `get_loader(main_dir, batch_size, len_crop, model_type)` and
`Solver(loader, config).train()` — started by torch.distributed.run.  Writes this rank's
parameters, its torch.save count and its sampler's (rank, world) to out_dir."""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compat"))

import data_loader  # noqa: E402
import solver_encoder  # noqa: E402


def main(main_dir, out_dir):
    rank = int(os.environ["RANK"])
    cfg = types.SimpleNamespace(lambda_cd=1.0, lambda_SISNR=1.0, dim_neck=32, dim_emb=256, dim_pre=512, freq=32,
                                main_dir=main_dir, batch_size=2, num_iters=4, len_crop=128, lr=0.0001,
                                speaker_embed=True, model_type="spmel", run_name="ddpmain", lr_scheduler=None,
                                depth=1, ema=0.9999, resume=False, run_id=None, log_step=2)
    vcc_loader = data_loader.get_loader(cfg.main_dir, cfg.batch_size, cfg.len_crop, cfg.model_type)   # main.py:36
    saves = []
    real_save = torch.save
    torch.save = lambda obj, f, *a, **k: saves.append(str(f)) or real_save(obj, f, *a, **k)
    solver = solver_encoder.Solver(vcc_loader, cfg)                                                   # main.py:39
    solver.train()                                                                                    # main.py:40
    torch.save = real_save
    torch.cuda.synchronize()
    sampler = vcc_loader.sampler
    torch.save([f.cpu() for f in solver.g_optimizer.flat_params()], os.path.join(out_dir, f"rank{rank}.pt"))
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"saves": saves, "sampler": type(sampler).__name__, "rank": getattr(sampler, "rank", None),
                   "world": getattr(sampler, "world", None), "solver_world": solver.world}, f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
