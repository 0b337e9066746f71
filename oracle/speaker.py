"""ORACLE (test infrastructure only) — CPU restatement of the D-VECTOR speaker encoder,
reference model_bl.py:5-20 (nn.LSTM(dim_input, dim_cell, 3 layers, batch_first) ->
Linear(dim_cell, dim_emb) on the last frame -> embeds / ||embeds||_2), on a flat
{state_dict key: tensor} map.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (autovc_amd/) never does.  Pinned against
tests/golden/dvector_golden.npz, produced by tests/golden/make_dvector_golden.py from the
reference's own model_bl.D_VECTOR (imported from /root/reference in the build container).
"""
from __future__ import annotations

import torch

from .generator import OracleGenerator, deterministic_state_dict


def dvector_keys(num_layers=3, dim_input=80, dim_cell=768, dim_emb=256):
    """Ordered (key, shape) list of model_bl.D_VECTOR's state_dict."""
    keys = []
    for l in range(num_layers):
        isz = dim_input if l == 0 else dim_cell
        keys += [(f"lstm.weight_ih_l{l}", (4 * dim_cell, isz)), (f"lstm.weight_hh_l{l}", (4 * dim_cell, dim_cell)),
                 (f"lstm.bias_ih_l{l}", (4 * dim_cell,)), (f"lstm.bias_hh_l{l}", (4 * dim_cell,))]
    keys += [("embedding.weight", (dim_emb, dim_cell)), ("embedding.bias", (dim_emb,))]
    return keys


def make_weights(**kw):
    return deterministic_state_dict({k: torch.empty(s) for k, s in dvector_keys(**kw)})


@torch.no_grad()
def dvector(P, x, num_layers=3):
    """x (B, T, dim_input) -> (B, dim_emb) unit-norm embeddings."""
    h = x.to(torch.float64)
    for l in range(num_layers):
        a = [P[f"lstm.{n}_l{l}"].to(torch.float64) for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        h = OracleGenerator._lstm_dir(h, *a, reverse=False)
    e = h[:, -1, :] @ P["embedding.weight"].to(torch.float64).t() + P["embedding.bias"].to(torch.float64)
    return e / e.norm(p=2, dim=-1, keepdim=True)
