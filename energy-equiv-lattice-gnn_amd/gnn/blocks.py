"""Hot-path blocks of the reference ``gnn/blocks.py``, MI355X-native.

Constructors, module names, parameter names, persistent buffers and ``forward``
signatures follow the reference, so ``state_dict``s round-trip strictly both ways:
the reference's large ``U_matrix_*`` buffers are derived data, emitted by
``state_dict()`` and verified / adopted on load (``mace.SymmetricContraction``)
rather than held on the device; ``Q_flat`` is a real buffer, so a loaded change
of basis is used as is.

``edge_index`` arguments accept either the reference's ``[2, E]`` tensor (the
edge tensors are then in the caller's order and get permuted once) or an
``ops.EdgeCSR`` (edge tensors already in receiver-sorted order, the fast path
used by ``EnergyEquivGNN``).
"""
from __future__ import annotations

import os
from argparse import Namespace
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _lib, cg, kernel_sets, ops
from .irreps import Irreps
from .mace import SymmetricContraction, reshape_irreps
from .o3 import Gate, GradMailbox, Linear, TensorProduct

# the layer residual's gradient summed in linear_up's grad-x epilogue (1) or by autograd (0)
RESIDUAL_GRAD_FUSED = os.environ.get("EELG_RESIDUAL_GRAD_FUSED", "1") != "0"
# when a layer computes its own radial weights (in line, EELG_OVERLAP=0): run the radial MLP
# before linear_up (1), so that tp_fwd directly follows the kernel that wrote its x, or after (0)
RADIAL_FIRST = os.environ.get("EELG_RADIAL_FIRST", "1") != "0"

EdgeIndex = Union[torch.Tensor, ops.EdgeCSR]

# torch_scatter reduces accepted for interaction_reduction (gnn/blocks.py:595-597): 'sum' is
# the fused kernel (the path scripts/train_main.py:32 uses); 'mean' scales its rows by the
# clamped in-degree; max / min / mul reduce the per-edge messages (ops.per_edge_csr)
REDUCTIONS = ("sum", "add", "mean", "max", "min", "mul")


def as_csr(edge_index: EdgeIndex, num_nodes: int, *edge_tensors):
    """Returns (csr, edge tensors in csr order)."""
    if isinstance(edge_index, ops.EdgeCSR):
        return (edge_index,) + tuple(edge_tensors)
    csr = ops.EdgeCSR.build(edge_index, num_nodes)
    return (csr,) + tuple(t[csr.perm] for t in edge_tensors)


def mat_square(c: torch.Tensor) -> torch.Tensor:
    """``c @ c`` for a batch of small (6 x 6) matrices as broadcast products and a sum: the
    library batched GEMM launches several 16x16-tile kernels (and two more in the backward) for
    what is 216 multiply-adds per matrix"""
    return (c.unsqueeze(-1) * c.unsqueeze(-3)).sum(-2)


def mat_power(c: torch.Tensor, k: int) -> torch.Tensor:
    """``torch.linalg.matrix_power(c, k)`` for k in {2, 4} by repeated ``mat_square``"""
    if k == 2:
        return mat_square(c)
    if k == 4:
        return mat_square(mat_square(c))
    return torch.linalg.matrix_power(c, k)


class PositiveLayer(torch.nn.Module):
    """``gnn/blocks.py:185-229``; the matrix powers as ``mat_power`` (same products, elementwise
    kernels instead of library GEMMs)."""

    def __init__(self, params: Namespace):
        super().__init__()
        f = params.positive_function
        eye = lambda c: torch.eye(6, device=c.device, dtype=c.dtype)  # noqa: E731
        funcs = {
            "matrix_power_2": lambda c: mat_power(c, 2),
            "matrix_power_4": lambda c: mat_power(c, 4),
            "matrix_exp": torch.linalg.matrix_exp,
            "matrix_trunc_exp_2": lambda c: mat_power(eye(c) + c / 2, 2),
            "matrix_trunc_exp_4": lambda c: mat_power(eye(c) + c / 4, 4),
            "none": lambda c: c,
        }
        if f not in funcs:
            raise ValueError(f"Unknown positive function: {f}")
        self.func = funcs[f]

    def forward(self, c):
        return self.func(c)


def _is_silu(gate) -> bool:
    return (gate is None or gate is torch.nn.functional.silu or isinstance(gate, torch.nn.SiLU)
            or gate is torch.nn.SiLU)


class GeneralNonLinearReadoutBlock(torch.nn.Module):
    """``gnn/blocks.py:250-283``.  ``gate`` is the activation of the scalars and the gates; the
    reference model passes ``torch.nn.functional.silu`` (``gnn/model.py:78-83``), which the
    fused Gate kernels implement (with e3nn's normalize2mom constant).  Any other activation
    raises instead of being silently replaced by SiLU."""

    def __init__(self, irreps_in, hidden_irreps, irreps_out, gate=torch.nn.functional.silu):
        super().__init__()
        if not _is_silu(gate):
            raise NotImplementedError(
                f"GeneralNonLinearReadoutBlock(gate={gate!r}): the Gate kernels are built for "
                "SiLU (torch.nn.functional.silu, as gnn/model.py:78-83 passes)")
        hidden_irreps, irreps_out = Irreps(hidden_irreps), Irreps(irreps_out)
        self.hidden_irreps, self.irreps_out = hidden_irreps, irreps_out
        scal = Irreps([(m, ir) for m, ir in hidden_irreps if ir.l == 0 and ir in irreps_out])
        gated = Irreps([(m, ir) for m, ir in hidden_irreps if ir.l > 0 and ir in irreps_out])
        gates = Irreps([(m, "0e") for m, _ in gated])
        self.equivariant_nonlin = Gate(scal, gates, gated)
        self.irreps_nonlin = self.equivariant_nonlin.irreps_in.simplify()
        self.linear_1 = Linear(irreps_in, self.irreps_nonlin)
        self.linear_2 = Linear(self.equivariant_nonlin.irreps_out, irreps_out)

    def forward(self, x):
        return self.linear_2(self.equivariant_nonlin(self.linear_1(x)))


class Cart_4_to_Mandel(torch.nn.Module):  # noqa: N801
    """``gnn/blocks.py:392-425``: a fixed linear map 81 -> 36 applied as one GEMM."""

    a = [0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 1, 1, 1, 0, 0, 0]
    b = [0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1]
    c = [0, 1, 2, 1, 0, 0, 1, 2, 1, 0, 0, 2, 1, 0, 0, 1, 0, 0, 0, 0, 0]
    d = [0, 1, 2, 2, 2, 1, 1, 2, 2, 2, 1, 2, 2, 2, 1, 2, 2, 1, 2, 1, 1]

    def __init__(self):
        super().__init__()
        s2 = np.sqrt(2)
        mask = np.array([[1, 1, 1, s2, s2, s2]] * 3 + [[s2, s2, s2, 2, 2, 2]] * 3)
        rows, cols = np.triu_indices(6)
        m = np.zeros((81, 36))
        for t, (r, q) in enumerate(zip(rows, cols)):
            src = ((self.a[t] * 3 + self.b[t]) * 3 + self.c[t]) * 3 + self.d[t]
            m[src, r * 6 + q] = mask[r, q]
            m[src, q * 6 + r] = mask[q, r]
        self.register_buffer("map", torch.tensor(m, dtype=torch.float32), persistent=False)
        # the reference's persistent buffers (same names, shapes and values), so checkpoints
        # round-trip strictly; they are verified on load, the GEMM above is what runs
        self.register_buffer("mask", torch.tensor(mask, dtype=torch.get_default_dtype()))
        rows_t, cols_t = torch.triu_indices(6, 6)
        self.register_buffer("rows", rows_t)
        self.register_buffer("cols", cols_t)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        absent = []
        for name in ("mask", "rows", "cols"):
            t = state_dict.get(prefix + name)
            mine = getattr(self, name)
            if t is None:
                absent.append(prefix + name)
            elif t.shape != mine.shape or not torch.allclose(
                    t.detach().cpu().double(), mine.cpu().double(), rtol=1e-6, atol=0):
                error_msgs.append(f"{prefix}{name}: differs from the reference's Cart_4_to_Mandel "
                                  "tables (gnn/blocks.py:395-417); refusing to load")
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)
        # derived tables: a checkpoint without them (written by this package before they were
        # registered) keeps the derived values instead of failing a strict load
        for k in absent:
            if k in missing_keys:
                missing_keys.remove(k)

    def forward(self, c):
        return (c.reshape(c.shape[0], 81) @ self.map).view(c.shape[0], 6, 6)


class Spherical_to_Cartesian(torch.nn.Module):  # noqa: N801
    """``gnn/blocks.py:427-442`` with the change of basis of ``cg.stiffness_change_of_basis``."""

    def __init__(self):
        super().__init__()
        q = torch.tensor(cg.stiffness_change_of_basis(), dtype=torch.float32)
        self.register_buffer("Q_flat", q.reshape(21, 81))

    def forward(self, x):
        return (x @ self.Q_flat).view(*x.shape[:-1], 3, 3, 3, 3)


class EquivariantProductBlock(torch.nn.Module):
    """``gnn/blocks.py:447-490``."""

    def __init__(self, node_feats_irreps, target_irreps, correlation: int, use_sc: bool = True):
        super().__init__()
        node_feats_irreps = Irreps(node_feats_irreps)
        self.reshape = reshape_irreps(node_feats_irreps)   # reference API; the path reads rows
        self.use_sc = use_sc
        mul = node_feats_irreps.count("0e")
        sc_out = Irreps([(mul, ir) for _, ir in Irreps(target_irreps)])
        self.symmetric_contractions = SymmetricContraction(node_feats_irreps, sc_out, correlation)
        self.linear = Linear(sc_out, target_irreps)

    def forward(self, node_feats, sc, residual: Optional[torch.Tensor] = None, grad_mailbox=None):
        """``residual``: the model's layer residual (``gnn/model.py:95``), added in the linear's
        epilogue instead of by a separate pass."""
        x = self.linear(self.symmetric_contractions(node_feats), residual=residual,
                        grad_mailbox=grad_mailbox)
        return x + sc if self.use_sc else x


class TensorProductInteractionBlock(torch.nn.Module):
    """``gnn/blocks.py:495-604`` with ``conv_tp`` + ``scatter / agg_norm_const`` fused
    into one HIP kernel (``eelg_tp_fwd``)."""

    def __init__(self, node_feats_irreps, edge_attrs_irreps, edge_feats_irreps, irreps_out,
                 agg_norm_const, reduce: str = "sum", bias: bool = False, MLP_dim: int = 64,
                 MLP_layers: int = 3, storage_dtype: torch.dtype = torch.float32):
        super().__init__()
        # bf16: the edge-sized tensors (TP weights, their gradient, per-edge grad of x)
        # are stored in bf16; all arithmetic stays fp32 (BASELINE config 5)
        self.storage_dtype = storage_dtype
        self._node_feats_irreps = Irreps(node_feats_irreps)
        self.edge_attrs_irreps = Irreps(edge_attrs_irreps)
        self.edge_feats_irreps = Irreps(edge_feats_irreps)
        self._irreps_out = Irreps(irreps_out)
        self.agg_norm_const = float(agg_norm_const)
        self.reduce = reduce.lower()
        if self.reduce not in REDUCTIONS:
            raise NotImplementedError(
                f"interaction_reduction {reduce!r}: the torch_scatter reduces {sorted(REDUCTIONS)} "
                "are built ('pna' is out of scope, SURVEY.md section 2)")
        # fail at construction, with the supported list, for structures without generated kernels
        kernel_sets.check_tp(self._node_feats_irreps, self.edge_attrs_irreps, self._irreps_out)
        if storage_dtype != torch.float32 and kernel_sets.mul_of(self._node_feats_irreps) != kernel_sets.MUL:
            raise NotImplementedError(
                f"{storage_dtype} storage of the edge tensors is generated for {kernel_sets.MUL} "
                f"channels only, not {self._node_feats_irreps}")
        self.linear_up = Linear(self._node_feats_irreps, self._node_feats_irreps)
        irreps_mid, instructions = cg.tp_out_irreps_with_instructions(
            self._node_feats_irreps, self.edge_attrs_irreps, self._irreps_out)
        self.conv_tp = TensorProduct(self._node_feats_irreps, self.edge_attrs_irreps, irreps_mid,
                                     instructions)
        # the fused radial-MLP kernels (csrc/eelg_radial.hip) are built for inter_MLP_dim 32 / 64,
        # inter_MLP_layers 2..4 and <= 32 edge features (the reference default: 12 -> 64 -> 64);
        # other shapes run the same torch.nn.Sequential on the device (library GEMMs + SiLU), the
        # reference's own formulation of conv_tp_weights
        n_feat = self.edge_feats_irreps.num_irreps
        if MLP_layers < 2:
            raise ValueError(f"inter_MLP_layers {MLP_layers}: the radial MLP needs at least one hidden layer")
        self._radial_hip = MLP_dim in (32, 64) and MLP_layers <= 4 and 1 <= n_feat <= 32
        layer = torch.nn.Linear(MLP_dim, self.conv_tp.weight_numel, bias=False)
        torch.nn.init.xavier_uniform_(layer.weight, gain=10)
        self.conv_tp_weights = torch.nn.Sequential(
            torch.nn.Linear(self.edge_feats_irreps.num_irreps, MLP_dim), torch.nn.SiLU())
        for _ in range(MLP_layers - 2):
            self.conv_tp_weights.append(torch.nn.Linear(MLP_dim, MLP_dim))
            self.conv_tp_weights.append(torch.nn.SiLU())
        self.conv_tp_weights.append(layer)
        self.irreps_mid = irreps_mid.simplify()
        self.linear = Linear(self.irreps_mid, self._irreps_out, biases=bias)
        # the generated kernel set serving this block is found by its structure hash
        self._sig = cg.fnv1a64(cg.tp_signature(self._node_feats_irreps, self.edge_attrs_irreps,
                                               self._irreps_out))
        self._cfg = None

    @property
    def irreps_in(self):
        return self._node_feats_irreps

    @property
    def irreps_out(self):
        return self._irreps_out

    def _config(self):
        if self._cfg is None:
            self._cfg = _lib.tp_config_by_sig(self._sig)
        return self._cfg

    def _bwf(self, cfg: int) -> bool:
        """the fused linear + TP backward serves this block (generated, same linear layout)"""
        if not hasattr(self, "_tp_paths"):
            self._tp_paths = cg.tp_paths(self._node_feats_irreps, self.edge_attrs_irreps, self._irreps_out)
        return ops.tp_linear_fusable(cfg, self.linear, self._tp_paths)

    def radial_weights(self, edge_feats: torch.Tensor) -> torch.Tensor:
        """``conv_tp_weights(edge_feats)`` (``gnn/blocks.py:590``): the per-edge TP weights."""
        if self._radial_hip:
            return ops.radial_mlp(edge_feats, self.conv_tp_weights, self.storage_dtype)
        ops._require_device(edge_feats)
        return self.conv_tp_weights(edge_feats).to(self.storage_dtype)

    def forward(self, node_feats, edge_attrs, edge_feats, edge_index: EdgeIndex,
                node_attrs: Optional[torch.Tensor] = None,
                tp_weights: Optional[torch.Tensor] = None, grad_mailbox=None) -> Tuple[torch.Tensor, None]:
        """``tp_weights``: ``radial_weights(edge_feats)`` computed ahead (possibly on another
        stream, see ``GNN_Head``); computed here when not given."""
        csr, edge_attrs, edge_feats = as_csr(edge_index, node_feats.shape[0], edge_attrs, edge_feats)
        idx, info = self._config()
        w = tp_weights
        if w is None and RADIAL_FIRST:
            w = self.radial_weights(edge_feats)
        x = self.linear_up(node_feats, grad_mailbox=grad_mailbox)
        if w is None:
            w = self.radial_weights(edge_feats)
        inv = 1.0 / self.agg_norm_const
        if self.reduce in ("sum", "add"):
            if ops.TP_BWF and self._bwf(idx):
                # output linear + TP with one fused backward kernel (eelg_tp_bwd_fused)
                return ops.tp_interaction_linear(x, edge_attrs, w, csr, idx, info, inv, self.linear), None
            if ops.TP_BWC > 1 and x.requires_grad:
                # the linear's grad-x and tp_bwd interleaved per receiver chunk
                return ops.tp_interaction_linear(x, edge_attrs, w, csr, idx, info, inv, self.linear,
                                                 ops.TP_BWC), None
            agg = ops.tp_interaction(x, edge_attrs, w, csr, idx, info, inv)
        elif self.reduce == "mean":
            agg = ops.tp_interaction(x, edge_attrs, w, csr, idx, info, inv) * ops.in_degree_scale(csr)[:, None]
        else:
            # max / min / mul of the per-edge messages, then / agg_norm_const as the reference
            m = ops.tp_interaction(x, edge_attrs, w, ops.per_edge_csr(csr), idx, info, 1.0)
            agg = ops.segment_order(m, csr.rowptr, csr.num_nodes, self.reduce, covered=True) * inv
        return self.linear(agg), None


class MACELayer(torch.nn.Module):
    """``gnn/blocks.py:902-947``."""

    def __init__(self, input_irreps, edge_sh_irreps, edge_scalars_irreps, interaction_irreps,
                 output_irreps, interaction_agg_norm_const, interaction_reduction: str,
                 interaction_bias: bool, product_correlation: int, MLP_dim: int = 64,
                 MLP_layers: int = 3, storage_dtype: torch.dtype = torch.float32):
        super().__init__()
        self.interaction = TensorProductInteractionBlock(
            input_irreps, edge_sh_irreps, edge_scalars_irreps, interaction_irreps,
            interaction_agg_norm_const, interaction_reduction, interaction_bias, MLP_dim,
            MLP_layers, storage_dtype)
        self.product = EquivariantProductBlock(self.interaction.irreps_out, output_irreps,
                                               product_correlation, use_sc=False)

    def forward(self, node_ft, edge_index: EdgeIndex, edge_sh, edge_scalars,
                tp_weights: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None):
        """``residual`` (default none): returns ``residual + layer(node_ft)`` with the add fused
        into the product block's linear (``GNN_Head`` passes ``h`` for ``h + layer_i(h)``)."""
        csr, edge_sh, edge_scalars = as_csr(edge_index, node_ft.shape[0], edge_sh, edge_scalars)
        if tp_weights is not None and not isinstance(edge_index, ops.EdgeCSR):
            tp_weights = tp_weights[csr.perm]
        # the residual h is also linear_up's input: its two gradient contributions are summed
        # in linear_up's grad-x epilogue (o3.GradMailbox), not by autograd in a separate pass
        mb = GradMailbox() if (RESIDUAL_GRAD_FUSED and residual is node_ft) else None
        node_ft, sc = self.interaction(node_ft, edge_sh, edge_scalars, csr, tp_weights=tp_weights,
                                       grad_mailbox=mb)
        return self.product(node_ft, sc, residual=residual, grad_mailbox=mb)
