"""Restatement of the hot-path blocks in ``gnn/blocks.py``.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
from __future__ import annotations

import math
from argparse import Namespace

import numpy as np
import torch

from . import o3
from .mace import SymmetricContraction, reshape_irreps, tp_out_irreps_with_instructions


def scatter_sum(src, index, dim_size):
    """torch_scatter ~2.0.9 ``scatter(reduce='sum')`` = zeros().scatter_add_()."""
    out = src.new_zeros((dim_size,) + src.shape[1:])
    return out.index_add(0, index, src)


def scatter_mean(src, index, dim_size):
    """torch_scatter ``scatter(reduce='mean')``: sum / clamp(count, 1)."""
    s = scatter_sum(src, index, dim_size)
    cnt = scatter_sum(torch.ones_like(index, dtype=src.dtype), index, dim_size).clamp_min(1)
    return s / cnt.view(-1, *([1] * (src.dim() - 1)))


def scatter_reduce_order(src, index, n, reduce):
    """torch_scatter ~2.0.9 ``scatter(reduce='max'|'min'|'mul')`` (the reference passes
    ``global_reduction`` straight through, ``gnn/model.py:100-106``): rows that receive
    nothing are 0 for max / min and 1 for mul.  Restated from torch_scatter's documented
    semantics (the package is absent here: parity unpinned); a per-row loop, small cases only."""
    rows = []
    for g in range(n):
        sel = src[index == g]
        if sel.shape[0] == 0:
            rows.append(torch.full((src.shape[1],), 1.0 if reduce == "mul" else 0.0, dtype=src.dtype))
        elif reduce == "max":
            rows.append(sel.max(0).values)
        elif reduce == "min":
            rows.append(sel.min(0).values)
        elif reduce == "mul":
            rows.append(sel.prod(0))
        else:
            raise ValueError(reduce)
    return torch.stack(rows)


class PositiveLayer(torch.nn.Module):
    """``gnn/blocks.py:185-229``."""

    def __init__(self, params: Namespace):
        super().__init__()
        f = params.positive_function
        funcs = {
            "matrix_power_2": lambda c: torch.linalg.matrix_power(c, 2),
            "matrix_power_4": lambda c: torch.linalg.matrix_power(c, 4),
            "matrix_exp": torch.linalg.matrix_exp,
            "matrix_trunc_exp_2": lambda c: torch.linalg.matrix_power(
                torch.eye(6, dtype=c.dtype) + c / 2, 2),
            "matrix_trunc_exp_4": lambda c: torch.linalg.matrix_power(
                torch.eye(6, dtype=c.dtype) + c / 4, 4),
            "none": lambda c: c,
        }
        if f not in funcs:
            raise ValueError(f"Unknown positive function: {f}")
        self.func = funcs[f]

    def forward(self, c):
        return self.func(c)


class GeneralNonLinearReadoutBlock(torch.nn.Module):
    """``gnn/blocks.py:250-283``."""

    def __init__(self, irreps_in, hidden_irreps, irreps_out):
        super().__init__()
        hidden_irreps, irreps_out = o3.Irreps(hidden_irreps), o3.Irreps(irreps_out)
        scal = o3.Irreps([(m, ir) for m, ir in hidden_irreps if ir.l == 0 and ir in irreps_out])
        gated = o3.Irreps([(m, ir) for m, ir in hidden_irreps if ir.l > 0 and ir in irreps_out])
        gates = o3.Irreps([(m, "0e") for m, _ in gated])
        self.equivariant_nonlin = o3.Gate(scal, gates, gated)
        self.irreps_nonlin = self.equivariant_nonlin.irreps_in.simplify()
        self.linear_1 = o3.Linear(irreps_in, self.irreps_nonlin)
        self.linear_2 = o3.Linear(self.equivariant_nonlin.irreps_out, irreps_out)

    def forward(self, x):
        return self.linear_2(self.equivariant_nonlin(self.linear_1(x)))


class Cart_4_to_Mandel(torch.nn.Module):  # noqa: N801
    """``gnn/blocks.py:392-425``."""

    a = [0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 1, 1, 1, 0, 0, 0]
    b = [0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1]
    c = [0, 1, 2, 1, 0, 0, 1, 2, 1, 0, 0, 2, 1, 0, 0, 1, 0, 0, 0, 0, 0]
    d = [0, 1, 2, 2, 2, 1, 1, 2, 2, 2, 1, 2, 2, 2, 1, 2, 2, 1, 2, 1, 1]

    def __init__(self):
        super().__init__()
        s2 = np.sqrt(2)
        self.register_buffer("mask", torch.tensor(
            [[1, 1, 1, s2, s2, s2]] * 3 + [[s2, s2, s2, 2, 2, 2]] * 3,
            dtype=torch.get_default_dtype()))
        rows, cols = torch.triu_indices(6, 6)
        self.register_buffer("rows", rows)
        self.register_buffer("cols", cols)

    def forward(self, c):
        c2 = c.new_zeros((c.shape[0], 6, 6))
        v = c[:, self.a, self.b, self.c, self.d]
        c2[:, self.rows, self.cols] = v
        c2[:, self.cols, self.rows] = v
        return c2 * self.mask.to(c.dtype).view(1, 6, 6)


class Spherical_to_Cartesian(torch.nn.Module):  # noqa: N801
    """``gnn/blocks.py:427-442``."""

    def __init__(self):
        super().__init__()
        q = o3.stiffness_change_of_basis(torch.get_default_dtype())
        self.register_buffer("Q_flat", q.flatten(-4))

    def forward(self, x):
        return (x @ self.Q_flat.to(x.dtype)).view(*x.shape[:-1], 3, 3, 3, 3)


class EquivariantProductBlock(torch.nn.Module):
    """``gnn/blocks.py:447-490`` (use_sc=False path used by MACELayer)."""

    def __init__(self, node_feats_irreps, target_irreps, correlation: int, use_sc: bool = True):
        super().__init__()
        self.node_feats_irreps = o3.Irreps(node_feats_irreps)
        self.use_sc = use_sc
        mul = self.node_feats_irreps.count((0, 1))
        sc_out = o3.Irreps([(mul, ir) for _, ir in o3.Irreps(target_irreps)])
        self.symmetric_contractions = SymmetricContraction(self.node_feats_irreps, sc_out, correlation)
        self.linear = o3.Linear(sc_out, target_irreps)

    def forward(self, node_feats, sc):
        x = reshape_irreps(self.node_feats_irreps, node_feats)
        x = self.symmetric_contractions(x)
        if self.use_sc:
            return self.linear(x) + sc
        return self.linear(x)


class TensorProductInteractionBlock(torch.nn.Module):
    """``gnn/blocks.py:495-604``; ``reduce`` is any torch_scatter reduce (``:595-597``)."""

    def __init__(self, node_feats_irreps, edge_attrs_irreps, edge_feats_irreps, irreps_out,
                 agg_norm_const, reduce="sum", bias=False, MLP_dim=64, MLP_layers=3):
        super().__init__()
        self._node_feats_irreps = o3.Irreps(node_feats_irreps)
        self.edge_attrs_irreps = o3.Irreps(edge_attrs_irreps)
        self.edge_feats_irreps = o3.Irreps(edge_feats_irreps)
        self._irreps_out = o3.Irreps(irreps_out)
        self.agg_norm_const = agg_norm_const
        self.reduce = reduce.lower()
        assert self.reduce in ("sum", "add", "mean", "max", "min", "mul"), self.reduce
        self.linear_up = o3.Linear(self._node_feats_irreps, self._node_feats_irreps)
        irreps_mid, instructions = tp_out_irreps_with_instructions(
            self._node_feats_irreps, self.edge_attrs_irreps, self._irreps_out)
        self.conv_tp = o3.TensorProduct(self._node_feats_irreps, self.edge_attrs_irreps,
                                        irreps_mid, instructions)
        input_dim = self.edge_feats_irreps.num_irreps
        layer = torch.nn.Linear(MLP_dim, self.conv_tp.weight_numel, bias=False)
        torch.nn.init.xavier_uniform_(layer.weight, gain=10)
        self.conv_tp_weights = torch.nn.Sequential(torch.nn.Linear(input_dim, MLP_dim), torch.nn.SiLU())
        for _ in range(MLP_layers - 2):
            self.conv_tp_weights.append(torch.nn.Linear(MLP_dim, MLP_dim))
            self.conv_tp_weights.append(torch.nn.SiLU())
        self.conv_tp_weights.append(layer)
        self.irreps_mid = irreps_mid.simplify()
        self.linear = o3.Linear(self.irreps_mid, self._irreps_out, biases=bias)

    @property
    def irreps_out(self):
        return self._irreps_out

    def forward(self, node_feats, edge_attrs, edge_feats, edge_index):
        sender, receiver = edge_index
        n = node_feats.shape[0]
        node_feats = self.linear_up(node_feats)
        tp_weights = self.conv_tp_weights(edge_feats)
        mji = self.conv_tp(node_feats[sender], edge_attrs, tp_weights)
        if self.reduce in ("sum", "add"):
            message = scatter_sum(mji, receiver, n)
        elif self.reduce == "mean":
            message = scatter_mean(mji, receiver, n)
        else:
            message = scatter_reduce_order(mji, receiver, n, self.reduce)
        message = message / self.agg_norm_const
        return self.linear(message), None


class MACELayer(torch.nn.Module):
    """``gnn/blocks.py:902-947``."""

    def __init__(self, input_irreps, edge_sh_irreps, edge_scalars_irreps, interaction_irreps,
                 output_irreps, agg_norm_const, reduction, bias, correlation,
                 MLP_dim=64, MLP_layers=3):
        super().__init__()
        self.interaction = TensorProductInteractionBlock(
            input_irreps, edge_sh_irreps, edge_scalars_irreps, interaction_irreps,
            agg_norm_const, reduction, bias, MLP_dim, MLP_layers)
        self.product = EquivariantProductBlock(self.interaction.irreps_out, output_irreps,
                                               correlation, use_sc=False)

    def forward(self, node_ft, edge_index, edge_sh, edge_scalars):
        node_ft, sc = self.interaction(node_ft, edge_sh, edge_scalars, edge_index)
        return self.product(node_ft, sc)
