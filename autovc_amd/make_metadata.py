"""Metadata — reference make_metadata.py:12-134 (D-VECTOR speaker embeddings -> train.pkl).

OUT OF SCOPE this round: it needs the absent 3000000-BL.ckpt speaker
encoder checkpoint.  The class exists so that main.py imports unchanged; metadata()
raises with an explanation.  main.py only calls it when <main_dir>/<model_type>/train.pkl
is missing (main.py:27-33).
"""


class Metadata(object):
    def __init__(self, config):
        self.main_dir = config.main_dir
        self.model_type = config.model_type

    def metadata(self):
        raise NotImplementedError(
            "make_metadata (D-VECTOR embeddings) is not on the autovc_amd GPU path: provide "
            f"{self.main_dir}/{self.model_type}/train.pkl (reference layout [spk, emb(256,), 'spk/f.npy', ...])")
