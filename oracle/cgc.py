"""CPU restatement of the CGC / mCGC benchmark models (TEST INFRASTRUCTURE ONLY).

Follows scripts/benchmark_models/cgc_modified.py:11-88 (mCGC: node embedding from
node_attrs, no residual on the first layer, 21-vector -> symmetric 6x6 -> square) and
scripts/benchmark_models/cgc_vanilla.py:11-74 (CGC: node embedding from positions,
residual on every layer, 21-vector output).  torch_scatter's scatter(sum|mean) is an
index_add over the receivers divided by the in-degree for 'mean'.
"""
from __future__ import annotations

from argparse import Namespace
from typing import Dict

import torch

from .mace import get_edge_vectors_and_lengths

# cgc_modified.py:28-33: Mandel 6x6 from the 21 upper-triangular entries
INDS_VAL = [[0, 1, 2, 3, 4, 5],
            [1, 6, 7, 8, 9, 10],
            [2, 7, 11, 12, 13, 14],
            [3, 8, 12, 15, 16, 17],
            [4, 9, 13, 16, 18, 19],
            [5, 10, 14, 17, 19, 20]]


def scatter_reduce(src, index, n, reduce):
    out = torch.zeros(n, src.shape[1], dtype=src.dtype).index_add_(0, index, src)
    if reduce == "sum":
        return out
    if reduce == "mean":
        cnt = torch.bincount(index, minlength=n).clamp_min(1).to(src.dtype)
        return out / cnt[:, None]
    raise ValueError(reduce)


class CGCLayer(torch.nn.Module):
    """cgc_modified.py:11-25 (identical in cgc_vanilla.py:11-25 and gnn/blocks.py:949-966)."""

    def __init__(self, node_dim: int, edge_dim: int, reduction: str = "sum"):
        super().__init__()
        self.num_hid_dim = 2 * node_dim + edge_dim
        self.fc_values = torch.nn.Linear(self.num_hid_dim, node_dim)
        self.fc_multip = torch.nn.Linear(self.num_hid_dim, node_dim)
        self.reduction = reduction

    def forward(self, x, edge_index, edge_ft):
        snd, rcv = edge_index
        cat = torch.cat([x[snd], x[rcv], edge_ft], dim=1)
        msg = torch.nn.functional.softplus(self.fc_values(cat)) * torch.sigmoid(self.fc_multip(cat))
        return scatter_reduce(msg, rcv, x.shape[0], self.reduction)


def _head(hidden: int) -> torch.nn.Sequential:
    return torch.nn.Sequential(torch.nn.Linear(hidden, 128), torch.nn.Softplus(),
                               torch.nn.Linear(128, 64), torch.nn.Softplus(),
                               torch.nn.Linear(64, 32), torch.nn.Softplus(),
                               torch.nn.Linear(32, 21))


def _edge_features(batch):
    vec, ln = get_edge_vectors_and_lengths(batch.positions, batch.edge_index, batch.shifts,
                                           normalize=True)
    return torch.cat([vec, ln, batch.edge_attr], dim=1)                 # [E, 5]


class CrystGraphConv(torch.nn.Module):
    """mCGC, cgc_modified.py:27-88."""

    def __init__(self, params: Namespace):
        super().__init__()
        self.params = params
        hid = params.hidden_irreps
        self.node_ft_embedding = torch.nn.Linear(1, hid)
        self.edge_ft_embedding = torch.nn.Linear(5, hid)
        self.cgc_layers = torch.nn.ModuleList(
            [CGCLayer(hid, hid, params.interaction_reduction) for _ in range(params.message_passes)])
        self.global_reduction = params.global_reduction
        self.mlp = _head(hid)

    def forward(self, batch) -> Dict:
        h = self.node_ft_embedding(batch.node_attrs)
        ef = self.edge_ft_embedding(_edge_features(batch))
        h = self.cgc_layers[0](h, batch.edge_index, ef)
        for layer in self.cgc_layers[1:]:
            h = h + layer(h, batch.edge_index, ef)
        g = scatter_reduce(h, batch.batch, batch.num_graphs, self.global_reduction)
        a = self.mlp(g)[:, INDS_VAL]
        if self.params.positive == "square":
            return {"stiffness": torch.linalg.matrix_power(a, 2)}
        if self.params.positive == "none":
            return {"stiffness": a}
        raise NotImplementedError(self.params.positive)


class CrystGraphConvVanilla(torch.nn.Module):
    """CGC, cgc_vanilla.py:27-74."""

    def __init__(self, params: Namespace):
        super().__init__()
        self.params = params
        hid = params.hidden_irreps
        self.node_ft_embedding = torch.nn.Linear(3, hid)
        self.edge_ft_embedding = torch.nn.Linear(5, hid)
        self.cgc_layers = torch.nn.ModuleList(
            [CGCLayer(hid, hid, params.interaction_reduction) for _ in range(params.message_passes)])
        self.global_reduction = params.global_reduction
        self.mlp = _head(hid)

    def forward(self, batch) -> Dict:
        h = self.node_ft_embedding(batch.positions)
        ef = self.edge_ft_embedding(_edge_features(batch))
        for layer in self.cgc_layers:
            h = h + layer(h, batch.edge_index, ef)
        g = scatter_reduce(h, batch.batch, batch.num_graphs, self.global_reduction)
        return {"stiffness": self.mlp(g)}
