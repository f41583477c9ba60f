"""Shared test helpers: reference params, synthetic batches, oracle/product pairing."""
from __future__ import annotations

from argparse import Namespace

import torch

from gnn.data import collate
from gnn.synthetic import SyntheticLattices


def params(message_passes: int = 2, lmax: int = 4, max_edge_radius: float = 0.05, **kw) -> Namespace:
    """``scripts/train_main.py:25-52`` (network part)."""
    hidden = "+".join(f"32x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    readout = "+".join(f"16x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    p = Namespace(lmax=lmax, hidden_irreps=hidden, readout_irreps=readout, num_edge_bases=6,
                  interaction_reduction="sum", interaction_bias=True, agg_norm_const=4.0,
                  inter_MLP_dim=64, inter_MLP_layers=3, correlation=3, global_reduction="mean",
                  message_passes=message_passes, positive_function="matrix_power_2",
                  max_edge_radius=max_edge_radius)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def batch(num_graphs: int = 4, num_nodes: int = 50, num_edges: int = 200, seed: int = 1234):
    ds = SyntheticLattices(num_graphs, num_nodes, num_edges, seed)
    return collate([ds[g] for g in range(num_graphs)]), ds.max_edge_radius


def copy_params(src: torch.nn.Module, dst: torch.nn.Module) -> None:
    sp = dict(src.named_parameters())
    with torch.no_grad():
        for name, p in dst.named_parameters():
            p.copy_(sp[name].to(p.dtype))


def batch_to(b, device, dtype=None):
    out = b.to(device)
    if dtype is not None:
        for k in ("positions", "node_attrs", "shifts", "edge_attr", "stiffness"):
            setattr(out, k, getattr(out, k).to(dtype))
    return out


def record_parity(key: str, **vals) -> None:
    """Append measured parity errors to the JSON file named by EELG_PARITY_OUT (if set):
    the GPU runs keep the achieved error next to each stated tolerance."""
    import json
    import os
    out = os.environ.get("EELG_PARITY_OUT")
    if not out:
        return
    data = {}
    if os.path.exists(out):
        with open(out) as f:
            data = json.load(f)
    data[key] = vals
    with open(out, "w") as f:
        json.dump(data, f, indent=1)
