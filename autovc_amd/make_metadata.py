"""Metadata — reference make_metadata.py:12-134: D-VECTOR speaker embeddings -> train.pkl,
and the conversion list -> metadata.pkl / metadata.log.

The speaker encoder runs on the GPU (autovc_amd.model_bl.D_VECTOR: the HIP LSTM step
kernels, last-frame GEMM, L2-normalisation kernel); the 10 random crops of a speaker go
through it as one batch.  The random draws (np.random.choice / randint) are made in the
reference's order, so a seeded run picks the same crops.  Differences: the checkpoint path
is a parameter (default '3000000-BL.ckpt' in the working directory, as the reference) and it
is read with torch.load(weights_only=True); the file is absent from the reference tree, so
callers without it get a FileNotFoundError naming it.
"""
from __future__ import annotations

import os
import pickle
from collections import OrderedDict

import numpy as np
import torch

from .model_bl import D_VECTOR


class Metadata(object):

    def __init__(self, config):
        self.speaker_embed = getattr(config, "speaker_embed", True)
        self.main_dir = config.main_dir
        self.model_type = config.model_type
        self.root_dir = self.main_dir + "/" + self.model_type
        self.num_uttrs = 10
        self.len_crop = 128
        self.subject_conversions = [(("p225", "001"), "p225")]
        self.speaker_info_path = getattr(config, "speaker_info", "speaker_info.txt")
        self.checkpoint = getattr(config, "speaker_checkpoint", "3000000-BL.ckpt")

    def speaker_encoder(self, device):
        C = D_VECTOR(dim_input=80, dim_cell=768, dim_emb=256).eval().to(device)
        if not os.path.exists(self.checkpoint):
            raise FileNotFoundError(f"speaker encoder checkpoint {self.checkpoint!r} not found "
                                    "(make_metadata.py:42 loads '3000000-BL.ckpt'; it is not in the reference tree)")
        ckpt = torch.load(self.checkpoint, map_location=device, weights_only=True)
        state = OrderedDict((k[7:], v) for k, v in ckpt["model_b"].items())   # drop 'module.'
        C.load_state_dict(state)
        return C

    def speaker_embeddings(self, C, device):
        """train.pkl rows [speaker, mean embedding (256,), 'spk/file.npy', ...] (make_metadata.py:50-85)."""
        mel_dir = self.main_dir + "/spmel"
        dirName, subdirList, _ = next(os.walk(mel_dir))
        print("Found directory: %s" % dirName)
        speakers = []
        for speaker in sorted(subdirList):
            print("Processing speaker: %s" % speaker)
            utterances = [speaker]
            _, _, fileList = next(os.walk(os.path.join(dirName, speaker)))
            assert len(fileList) >= self.num_uttrs
            idx_uttrs = np.random.choice(len(fileList), size=self.num_uttrs, replace=False)
            crops = []
            for i in range(self.num_uttrs):
                tmp = np.load(os.path.join(dirName, speaker, fileList[idx_uttrs[i]]))
                candidates = np.delete(np.arange(len(fileList)), idx_uttrs)
                while tmp.shape[0] < self.len_crop:
                    idx_alt = np.random.choice(candidates)
                    tmp = np.load(os.path.join(dirName, speaker, fileList[idx_alt]))
                    candidates = np.delete(candidates, np.argwhere(candidates == idx_alt))
                left = np.random.randint(0, tmp.shape[0] - self.len_crop)
                crops.append(tmp[left:left + self.len_crop, :])
            with torch.no_grad():
                embs = C(torch.from_numpy(np.stack(crops).astype(np.float32)).to(device)).cpu().numpy()
            utterances.append(np.mean(embs, axis=0))
            for fileName in sorted(fileList):
                utterances.append(os.path.join(speaker, fileName))
            speakers.append(utterances)
        return speakers

    def metadata(self):
        if not torch.cuda.is_available():
            raise RuntimeError("make_metadata runs the speaker encoder on the MI355X (no CPU path)")
        device = torch.device("cuda")
        C = self.speaker_encoder(device)
        speakers = self.speaker_embeddings(C, device)
        os.makedirs(self.root_dir, exist_ok=True)
        with open(os.path.join(self.root_dir, "train.pkl"), "wb") as handle:
            pickle.dump(speakers, handle)
        subject_speaker_embedding = {row[0]: row[1] for row in speakers}
        import pandas as pd
        speaker_info = pd.read_csv(self.speaker_info_path, sep=r"\s+")
        with open(os.path.join(self.root_dir, "metadata.log"), "w") as log:
            log_ref_int = 0
            metadata = []
            for conversion in self.subject_conversions:
                log.write("CONVERSION FILENAME: " + str(log_ref_int) + " " + "#" * 40 + "\n\n")
                with open(os.path.join(self.main_dir, "txt", conversion[0][0],
                                       conversion[0][0] + "_" + conversion[0][1] + ".txt"), "r") as sentence_file:
                    sentence = "\"" + sentence_file.readline().rstrip("\n").rstrip() + "\""
                    log.write(f"Converting from sentence no. {conversion[0][1]} : {sentence} \n")
                log.write("Uttered by the speaker:\n")
                log.write(speaker_info[speaker_info["ID"] == conversion[0][0]].to_string(index=False))
                log.write("\n")
                log.write("To the speaker:\n")
                log.write(speaker_info[speaker_info["ID"] == conversion[1]].to_string(index=False))
                log.write("\n\n")
                base = self.root_dir + "/" + conversion[0][0] + "/" + conversion[0][0] + "_" + conversion[0][1]
                sound_input = np.load(base + "_mic2.npy") if os.path.exists(base + "_mic2.npy") else np.load(base + ".npy")
                metadata.append([log_ref_int,
                                 [conversion[0][0] + "_" + conversion[0][1], subject_speaker_embedding[conversion[0][0]],
                                  sound_input],
                                 [conversion[1], subject_speaker_embedding[conversion[1]]]])
                log_ref_int = log_ref_int + 1
            with open(os.path.join(self.root_dir, "metadata.pkl"), "wb") as handle:
                pickle.dump(metadata, handle)
        print("Finished generating metadata")
