"""Restatement of ``gnn/model.py`` (``GNN_Head``, ``EnergyEquivGNN``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
from __future__ import annotations

from argparse import Namespace

import torch

from . import o3
from .blocks import (Cart_4_to_Mandel, GeneralNonLinearReadoutBlock, MACELayer, PositiveLayer,
                     Spherical_to_Cartesian, scatter_mean, scatter_reduce_order, scatter_sum)
from .mace import get_edge_vectors_and_lengths


class GNN_Head(torch.nn.Module):  # noqa: N801
    """``gnn/model.py:26-112``."""

    def __init__(self, params: Namespace):
        super().__init__()
        self.params = params
        hidden = o3.Irreps(params.hidden_irreps)
        node_ft_irreps = o3.Irreps([(hidden.count((0, 1)), (0, 1))])
        edge_feats_irreps = o3.Irreps(f"{params.num_edge_bases * 2}x0e")
        edge_attr_irreps = o3.Irreps.spherical_harmonics(params.lmax)
        num_features = hidden.count((0, 1))
        interaction_irreps = (edge_attr_irreps * num_features).sort()[0].simplify()
        readout_irreps = o3.Irreps(params.readout_irreps)
        self.num_interactions = params.message_passes
        mk = lambda inp: MACELayer(inp, edge_attr_irreps, edge_feats_irreps, interaction_irreps,  # noqa: E731
                                   hidden, params.agg_norm_const, params.interaction_reduction,
                                   True, params.correlation, params.inter_MLP_dim,
                                   params.inter_MLP_layers)
        self.layers = torch.nn.ModuleList([mk(node_ft_irreps)])
        for _ in range(self.num_interactions - 1):
            self.layers.append(mk(hidden))
        self.nonlin_readout = GeneralNonLinearReadoutBlock(hidden, hidden, readout_irreps)
        self.global_reduction = params.global_reduction
        self.linear = o3.Linear(readout_irreps, o3.Irreps("2x0e+2x2e+1x4e"), biases=True)
        self.sph_to_cart = Spherical_to_Cartesian()
        self.cart_to_Mandel = Cart_4_to_Mandel()
        self.positive_layer = PositiveLayer(params)

    def forward(self, edge_index, node_ft, edge_sh, edge_feats, batch_idx, num_graphs):
        node_ft = self.layers[0](node_ft, edge_index, edge_sh, edge_feats)
        for i in range(1, self.num_interactions):
            node_ft = node_ft + self.layers[i](node_ft, edge_index, edge_sh, edge_feats)
        out = self.nonlin_readout(node_ft)
        if self.global_reduction == "mean":
            g = scatter_mean(out, batch_idx, num_graphs)
        elif self.global_reduction in ("sum", "add"):
            g = scatter_sum(out, batch_idx, num_graphs)
        elif self.global_reduction in ("max", "min", "mul"):
            g = scatter_reduce_order(out, batch_idx, num_graphs, self.global_reduction)
        else:
            raise ValueError(self.global_reduction)
        stiff = self.sph_to_cart(self.linear(g))
        return self.positive_layer(self.cart_to_Mandel(stiff))


class EnergyEquivGNN(torch.nn.Module):
    """``gnn/model.py:115-161``."""

    def __init__(self, params: Namespace):
        super().__init__()
        self.params = params
        hidden = o3.Irreps(params.hidden_irreps)
        self.node_ft_embedding = torch.nn.Linear(1, hidden.count((0, 1)))
        self.number_of_edge_basis = params.num_edge_bases
        self.max_edge_radius = params.max_edge_radius
        self.lmax = params.lmax
        self.stiffness_head = GNN_Head(params)

    def embed(self, batch):
        """Edge geometry + embeddings, ``gnn/model.py:139-157``."""
        vectors, lengths = get_edge_vectors_and_lengths(batch.positions, batch.edge_index, batch.shifts)
        el = o3.soft_one_hot_linspace(lengths.squeeze(-1), 0, 0.6, self.number_of_edge_basis)
        er = o3.soft_one_hot_linspace(batch.edge_attr.squeeze(-1), 0, self.max_edge_radius,
                                      self.number_of_edge_basis)
        edge_feats = torch.cat((el, er), dim=1)
        edge_sh = o3.spherical_harmonics(self.lmax, vectors)
        return edge_sh, edge_feats

    def forward(self, batch):
        node_ft = self.node_ft_embedding(batch.node_attrs)
        edge_sh, edge_feats = self.embed(batch)
        c = self.stiffness_head(batch.edge_index, node_ft, edge_sh, edge_feats, batch.batch,
                                batch.num_graphs)
        return {"stiffness": c}
