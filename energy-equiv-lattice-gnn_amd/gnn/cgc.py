"""Crystal-graph edge-convolution benchmark models on the HIP path.

``CrystGraphConv`` mirrors scripts/benchmark_models/cgc_modified.py:27-88 (mCGC) and
``CrystGraphConvVanilla`` mirrors scripts/benchmark_models/cgc_vanilla.py:27-74 (CGC); both
keep the reference's parameter names.  The edge convolution
(``CGCLayer``, cgc_modified.py:11-25) runs as two fused HIP kernels (``eelg_cgc_fwd`` /
``eelg_cgc_bwd``): the [E, 3D] concatenation is never formed (the linear map is split
into node-level projections gathered per edge plus one edge-level GEMM) and the
scatter-add is a register sum per receiver over the receiver-sorted CSR shared with
EnergyEquivGNN.  Weight gradients that reduce over nodes / edges use the split-K form
(``ops._wgrad``).
"""
from __future__ import annotations

from argparse import Namespace
from typing import Dict, Optional

import torch

from . import _lib, ops
from .blocks import EdgeIndex, as_csr

# Mandel 6x6 from the 21 upper-triangular outputs (cgc_modified.py:28-33)
INDS_VAL = [[0, 1, 2, 3, 4, 5],
            [1, 6, 7, 8, 9, 10],
            [2, 7, 11, 12, 13, 14],
            [3, 8, 12, 15, 16, 17],
            [4, 9, 13, 16, 18, 19],
            [5, 10, 14, 17, 19, 20]]


class _CGCConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, edge_ft, wv, bv, wm, bm, csr: ops.EdgeCSR, row_scale: Optional[torch.Tensor]):
        x, edge_ft = ops._f32(x), ops._f32(edge_ft)
        n, d = x.shape
        if edge_ft.shape != (csr.num_edges, d) or n != csr.num_nodes:
            raise ValueError(f"CGC shapes: x {tuple(x.shape)}, edge_ft {tuple(edge_ft.shape)}, "
                             f"csr {csr.num_nodes} nodes / {csr.num_edges} edges")
        w = torch.cat([wv, wm])                                   # [2D, 3D]
        ws, wr, we = w[:, :d], w[:, d: 2 * d], w[:, 2 * d:]
        ps = x @ ws.t()
        pr = torch.addmm(torch.cat([bv, bm]), x, wr.t())
        ep = edge_ft @ we.t()
        agg = torch.empty(n, d, device=x.device, dtype=torch.float32)
        tok = ops.TIMER.start("cgc_fwd")
        _lib.check(_lib.load().eelg_cgc_fwd(
            _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ep), _lib.ptr(csr.sender), _lib.ptr(csr.rowptr),
            _lib.ptr(row_scale), n, d, _lib.ptr(agg), _lib.stream(agg)), "cgc_fwd")
        ops.TIMER.stop(tok)
        ctx.save_for_backward(x, edge_ft, ps, pr, ep, w, row_scale)
        ctx.csr = csr
        return agg

    @staticmethod
    def backward(ctx, g):
        x, edge_ft, ps, pr, ep, w, row_scale = ctx.saved_tensors
        csr = ctx.csr
        n, d = x.shape
        g = ops._f32(g)
        dz = torch.empty(csr.num_edges, 2 * d, device=x.device, dtype=torch.float32)
        gr = torch.empty(n, 2 * d, device=x.device, dtype=torch.float32)
        tok = ops.TIMER.start("cgc_bwd")
        _lib.check(_lib.load().eelg_cgc_bwd(
            _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ep), _lib.ptr(csr.sender), _lib.ptr(csr.rowptr),
            _lib.ptr(row_scale), n, d, _lib.ptr(g), _lib.ptr(dz), _lib.ptr(gr), _lib.stream(g)), "cgc_bwd")
        ops.TIMER.stop(tok)
        gs = ops.segment_sum_csr(dz, csr.srowptr, n, idx=csr.sperm)   # per-sender sums of dz
        ws, wr, we = w[:, :d], w[:, d: 2 * d], w[:, 2 * d:]
        dw = torch.cat([ops._wgrad(gs, x), ops._wgrad(gr, x), ops._wgrad(dz, edge_ft)], dim=1)
        db = ops.sum_rows(gr)
        dx = gs @ ws + gr @ wr
        dedge = dz @ we
        return dx, dedge, dw[:d], db[:d], dw[d:], db[d:], None, None


class CGCLayer(torch.nn.Module):
    """``cgc_modified.py:11-25`` / ``gnn/blocks.py:949-966``: same parameters
    (``fc_values``, ``fc_multip``), same ``forward(x, edge_index, edge_ft)``; ``edge_index``
    may also be an ``ops.EdgeCSR`` (then ``edge_ft`` is in CSR edge order)."""

    def __init__(self, node_dim: int, edge_dim: int, reduction: str = "sum"):
        super().__init__()
        if edge_dim != node_dim:
            raise NotImplementedError("CGCLayer: the fused kernel needs edge_dim == node_dim "
                                      "(as in both reference models)")
        if node_dim > _lib.CGC_MAXD:
            raise NotImplementedError(f"CGCLayer: node_dim {node_dim} > {_lib.CGC_MAXD}, the widest "
                                      "built CGC kernel (include/eelg.h EELG_CGC_MAXD)")
        if reduction not in ("sum", "mean"):
            raise NotImplementedError(f"CGCLayer reduction {reduction!r}")
        self.num_hid_dim = 2 * node_dim + edge_dim
        self.fc_values = torch.nn.Linear(self.num_hid_dim, node_dim)
        self.fc_multip = torch.nn.Linear(self.num_hid_dim, node_dim)
        self.reduction = reduction

    def forward(self, x: torch.Tensor, edge_index: EdgeIndex, edge_ft: torch.Tensor) -> torch.Tensor:
        ops._require_device(x)
        csr, edge_ft = as_csr(edge_index, x.shape[0], edge_ft)
        scale = None
        if self.reduction == "mean":
            deg = (csr.rowptr[1:] - csr.rowptr[:-1]).to(torch.float32)
            scale = 1.0 / deg.clamp_min(1.0)
        return _CGCConv.apply(x, edge_ft, self.fc_values.weight, self.fc_values.bias,
                              self.fc_multip.weight, self.fc_multip.bias, csr, scale)


def _head(hidden: int) -> torch.nn.Sequential:
    return torch.nn.Sequential(torch.nn.Linear(hidden, 128), torch.nn.Softplus(),
                               torch.nn.Linear(128, 64), torch.nn.Softplus(),
                               torch.nn.Linear(64, 32), torch.nn.Softplus(),
                               torch.nn.Linear(32, 21))


def _edge_inputs(batch, csr: ops.EdgeCSR) -> torch.Tensor:
    """[normalised edge vector | length | strut radius] in CSR edge order
    (``gnn/mace.py:338-352`` with normalize=True, eps 1e-9; cgc_modified.py:71-74)."""
    pos = batch.positions
    vec = pos[csr.receiver.long()] - pos[csr.sender.long()] + batch.shifts[csr.perm]
    ln = torch.linalg.norm(vec, dim=-1, keepdim=True)
    return torch.cat([vec / (ln + 1e-9), ln, batch.edge_attr[csr.perm]], dim=1)


class _CGCBase(torch.nn.Module):
    node_inputs = 1

    def __init__(self, params: Namespace):
        super().__init__()
        self.params = params
        hid = params.hidden_irreps
        self.node_ft_embedding = torch.nn.Linear(self.node_inputs, hid)
        self.edge_ft_embedding = torch.nn.Linear(5, hid)
        self.cgc_layers = torch.nn.ModuleList(
            [CGCLayer(hid, hid, params.interaction_reduction) for _ in range(params.message_passes)])
        self.global_reduction = params.global_reduction
        self.mlp = _head(hid)

    def _encode(self, batch, node_in):
        from .model import EnergyEquivGNN
        csr = EnergyEquivGNN.edge_graph(batch)
        return csr, self.node_ft_embedding(node_in), self.edge_ft_embedding(_edge_inputs(batch, csr))

    def _pool(self, h, batch):
        return ops.graph_pool(h, batch.batch, batch.num_graphs, self.global_reduction)


class CrystGraphConv(_CGCBase):
    """mCGC (``cgc_modified.py:27-88``): node features from ``node_attrs``, no residual on
    the first layer, 21 outputs -> symmetric 6x6 -> ``positive`` ('square' | 'none')."""
    inds_val = INDS_VAL
    node_inputs = 1

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        csr, h, ef = self._encode(batch, batch.node_attrs)
        h = self.cgc_layers[0](h, csr, ef)
        for layer in self.cgc_layers[1:]:
            h = h + layer(h, csr, ef)
        a = self.mlp(self._pool(h, batch))[:, self.inds_val]
        if self.params.positive == "square":
            return {"stiffness": torch.linalg.matrix_power(a, 2)}
        if self.params.positive == "none":
            return {"stiffness": a}
        raise NotImplementedError(self.params.positive)


class CrystGraphConvVanilla(_CGCBase):
    """CGC (``cgc_vanilla.py:27-74``): node features from ``positions``, residual on every
    layer, 21 raw outputs."""
    node_inputs = 3

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        csr, h, ef = self._encode(batch, batch.positions)
        for layer in self.cgc_layers:
            h = h + layer(h, csr, ef)
        return {"stiffness": self.mlp(self._pool(h, batch))}
