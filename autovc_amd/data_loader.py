"""Utterance crops for Generator training — reference data_loader.py:11-102, same contract.

`get_loader(root_dir, batch_size, len_crop, model_type, num_workers)` returns a torch
DataLoader over speakers: each item is a random utterance of that speaker (never index 0/1,
which hold the speaker id and embedding, data_loader.py:68), randomly cropped to len_crop
frames or zero-padded at the end (:70-78), plus the speaker embedding.  `train.pkl` is the
user's metadata file in the reference layout [spk, emb, 'spk/file.npy', ...].

Differences: spectrograms are loaded in-process (no multiprocessing.Manager),
items stay on the host (the Solver moves each batch to the GPU with one non-blocking copy
instead of a per-item .to(device), :69), and data-parallel training (rank/world) uses
`SpeakerCropSampler`: every rank draws its batch from ALL speakers, with replacement, from
a stream seeded by (seed, rank, epoch).  The reference's loader indexes speakers without
replacement with drop_last (:96-101), so with the 7 bundled speakers any batch larger than
7 yields zero batches; sharding those speakers over 8 ranks would leave each rank none.
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch
from torch.utils import data


class Utterances(data.Dataset):
    def __init__(self, data_dir, len_crop, model_type):
        self.root_dir = os.path.join(data_dir, model_type)
        self.len_crop = len_crop
        with open(os.path.join(self.root_dir, "train.pkl"), "rb") as f:
            meta = pickle.load(f)  # user-provided metadata, as the reference does
        self.train_dataset = []
        for sbmt in meta:
            uttrs = [sbmt[0], np.asarray(sbmt[1], dtype=np.float32)]
            for rel in sbmt[2:]:
                uttrs.append(np.load(os.path.join(self.root_dir, rel)).astype(np.float32, copy=False))
            self.train_dataset.append(uttrs)
        self.num_tokens = len(self.train_dataset)

    def __getitem__(self, index):
        list_uttrs = self.train_dataset[index]
        emb_org = torch.from_numpy(list_uttrs[1])
        a = np.random.randint(2, len(list_uttrs))
        tmp = list_uttrs[a]
        if tmp.shape[0] < self.len_crop:
            uttr = np.pad(tmp, ((0, self.len_crop - tmp.shape[0]), (0, 0)), "constant")
        elif tmp.shape[0] > self.len_crop:
            left = np.random.randint(tmp.shape[0] - self.len_crop)
            uttr = tmp[left:left + self.len_crop, :]
        else:
            uttr = tmp
        return torch.from_numpy(np.ascontiguousarray(uttr, dtype=np.float32)), emb_org

    def __len__(self):
        return self.num_tokens


class SpeakerCropSampler(data.Sampler):
    """Speaker indices for one data-parallel rank: `batches` batches of `batch_size`
    speakers per epoch, drawn uniformly WITH replacement from all `n_speakers`, from
    RandomState(seed + 1_000_003 * rank + 7_919 * epoch).  Ranks draw independent streams
    (different crops of the same speakers), every epoch reshuffles (`set_epoch`, called by
    Solver.train each time it re-creates the data iterator), and the stream is reproducible.
    Default `batches` = max(1, n_speakers // (batch_size * world)): the reference's epoch
    length (len // batch_size, drop_last) spread over the ranks, but never zero."""

    def __init__(self, n_speakers, batch_size, rank=0, world=1, seed=0, batches=None):
        if n_speakers <= 0 or batch_size <= 0 or world <= 0 or not 0 <= rank < world:
            raise ValueError(f"SpeakerCropSampler: n_speakers={n_speakers} batch_size={batch_size} "
                             f"rank={rank} world={world}")
        self.n, self.bs, self.rank, self.world, self.seed = n_speakers, batch_size, rank, world, seed
        self.batches = batches if batches is not None else max(1, n_speakers // (batch_size * world))
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def __iter__(self):
        rs = np.random.RandomState((self.seed + 1_000_003 * self.rank + 7_919 * self.epoch) % (2 ** 32))
        return iter(rs.randint(0, self.n, self.batches * self.bs).tolist())

    def __len__(self):
        return self.batches * self.bs


def get_loader(root_dir, batch_size=16, len_crop=128, model_type="spmel", num_workers=0, rank=None, world=None,
               seed=0):
    """data_loader.py:90-102 (shuffle, drop_last, seeded workers).  With rank/world (and
    world > 1) the batches come from a per-rank `SpeakerCropSampler` instead.  rank/world
    not given: taken from a launcher's environment (torchrun's RANK / WORLD_SIZE), so
    main.py's unchanged call `get_loader(main_dir, batch_size, len_crop, model_type)`
    (main.py:36) shards under torchrun."""
    if world is None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
    dataset = Utterances(root_dir, len_crop, model_type)
    sampler = None
    if world is not None and world > 1:
        sampler = SpeakerCropSampler(len(dataset), batch_size, rank or 0, world, seed)
    worker_init_fn = lambda x: np.random.seed((torch.initial_seed()) % (2 ** 32))  # noqa: E731
    return data.DataLoader(dataset=dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                           num_workers=num_workers, drop_last=True, worker_init_fn=worker_init_fn)
