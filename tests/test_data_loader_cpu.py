"""Rank-aware data pipeline: get_loader(rank=, world=) on the reference's
layout (7 speakers like the bundled spmel/, data_loader.py:83-85) must feed B=64 crops per
rank at 8 ranks — the reference loader (speaker-indexed, drop_last) yields zero batches
there — with independent per-rank streams and a reshuffle every epoch (set_epoch)."""
import os
import pickle
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from autovc_amd.data_loader import SpeakerCropSampler, get_loader

N_SPK = 7


def _corpus(root):
    rs = np.random.RandomState(1)
    meta = []
    for s in range(N_SPK):
        spk = f"p{225 + s}"
        os.makedirs(os.path.join(root, "spmel", spk), exist_ok=True)
        files = []
        for i, T in enumerate([90, 128, 200]):
            # frame value = speaker index: the batch tells which speaker each crop came from
            np.save(os.path.join(root, "spmel", spk, f"{spk}_{i}.npy"), np.full((T, 80), s + 1, np.float32))
            files.append(f"{spk}/{spk}_{i}.npy")
        meta.append([spk, np.full(256, s, np.float32)] + files)
    with open(os.path.join(root, "spmel", "train.pkl"), "wb") as f:
        pickle.dump(meta, f)
    return root


def test_reference_semantics_without_world(tmp_path):
    root = _corpus(str(tmp_path))
    assert len(list(get_loader(root, batch_size=64))) == 0        # reference: B > speakers -> no batch
    assert len(list(get_loader(root, batch_size=2))) == 3         # 7 // 2, drop_last


def test_sampler_draws_full_batches_per_rank():
    s = SpeakerCropSampler(N_SPK, 64, rank=3, world=8, seed=5)
    idx = list(s)
    assert len(idx) == len(s) == 64 and set(idx) <= set(range(N_SPK))
    assert idx == list(SpeakerCropSampler(N_SPK, 64, rank=3, world=8, seed=5))      # reproducible
    assert idx != list(SpeakerCropSampler(N_SPK, 64, rank=4, world=8, seed=5))      # ranks differ
    s.set_epoch(1)
    assert list(s) != idx                                                            # epochs reshuffle
    assert len(set(idx)) == N_SPK                                                    # all speakers drawn


def _worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    np.random.seed(100 + rank)
    loader = get_loader(root, batch_size=64, rank=dist.get_rank(), world=dist.get_world_size(), seed=9)
    out = []
    for epoch in range(2):
        loader.sampler.set_epoch(epoch)
        batches = list(loader)
        x, e = batches[0]
        out.append((len(batches), tuple(x.shape), tuple(e.shape), x[:, 0, 0].tolist(), e[:, 0].tolist()))
    # ranks agree on nothing but the shape: gather every rank's speaker sequence
    seq = torch.tensor(out[0][3])
    allseq = [torch.zeros_like(seq) for _ in range(world)]
    dist.all_gather(allseq, seq)
    q.put((rank, out, [a.tolist() for a in allseq]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rank_aware_loader_gloo_world2(tmp_path):
    root = _corpus(str(tmp_path))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out, allseq in res:
        for n_batches, xs, es, spk_from_x, spk_from_e in out:
            assert n_batches == 1 and xs == (64, 128, 80) and es == (64, 256)
            # every crop comes from the speaker whose embedding it is paired with; crops
            # shorter than 128 frames are zero-padded at the end, never at the start
            assert [int(v) - 1 for v in spk_from_x] == [int(v) for v in spk_from_e]
        assert out[0][3] != out[1][3]                       # set_epoch reshuffles
        assert allseq[0] != allseq[1]                       # the two ranks draw different speakers
