"""Crystal-graph edge-convolution benchmark models on the HIP path.

``CrystGraphConv`` mirrors scripts/benchmark_models/cgc_modified.py:27-88 (mCGC) and
``CrystGraphConvVanilla`` mirrors scripts/benchmark_models/cgc_vanilla.py:27-74 (CGC); both
keep the reference's parameter names.  The edge convolution
(``CGCLayer``, cgc_modified.py:11-25) runs as two fused HIP kernels (``eelg_cgc_fwd`` /
``eelg_cgc_bwd``): the [E, 3D] concatenation is never formed (the linear map is split
into node-level projections gathered per edge plus one edge-level GEMM) and the
scatter-add is a register sum per receiver over the receiver-sorted CSR shared with
EnergyEquivGNN.  Every Linear of the models (node / edge projections, their gradients, the MLP head) runs on the
in-tree MFMA linear kernels (``gnn/dense.py``); in the models the edge features enter in
factored form (``eelg_cgc_fwd_ef``: the edge embedding composed with each layer's edge block), so
the [E, 2D] edge projection is never written.
"""
from __future__ import annotations

import os
from argparse import Namespace
from typing import Dict, Optional

import torch

from . import _lib, dense, ops
from .blocks import EdgeIndex, as_csr, mat_square

# the layer residual added inside the CGC kernels (1, default) or as a separate torch add (0).
# Same box (r06n): 32,425 vs 31,940 / 31,753 graphs/s, and the aggregation kernel's roofline
# fraction (its residual read counted) 0.436 vs 0.422 / 0.424
CGC_FUSED_RES = os.environ.get("EELG_CGC_FUSED_RES", "1") != "0"
# every layer's edge factor in one batched pass (1) or per layer (0)
CGC_EA_BATCH = os.environ.get("EELG_CGC_EA_BATCH", "1") != "0"

# Mandel 6x6 from the 21 upper-triangular outputs (cgc_modified.py:28-33)
INDS_VAL = [[0, 1, 2, 3, 4, 5],
            [1, 6, 7, 8, 9, 10],
            [2, 7, 11, 12, 13, 14],
            [3, 8, 12, 15, 16, 17],
            [4, 9, 13, 16, 18, 19],
            [5, 10, 14, 17, 19, 20]]


def _cgc_dw(x, gs, gr, db_on: bool):
    """weight / bias gradients of the node blocks: dW_s = gs^T x, dW_r = gr^T x, db = sum(gr)"""
    return dense.linear_bwd_w(x, gs), dense.linear_bwd_w(x, gr), (ops.sum_rows(gr) if db_on else None)


def _cgc_dx(gs, gr, w, d, res=None):
    """gs W_s + gr W_r (+ res, a residual's gradient): two launches of the linear kernel, each
    adding the previous term in its epilogue"""
    dx = dense.linear_bwd_x(gs, w, 2 * d, d, w_off=0, ld=3 * d, res=res)
    return dense.linear_bwd_x(gr, w, 2 * d, d, w_off=d, ld=3 * d, res=dx)


class _CGCConv(torch.autograd.Function):
    """One edge convolution with the edge features given ([E, D], CSR order): the generic
    ``CGCLayer.forward`` API.  Every projection runs on the in-tree linear kernels."""

    @staticmethod
    def forward(ctx, x, edge_ft, wv, bv, wm, bm, csr: ops.EdgeCSR, row_scale: Optional[torch.Tensor]):
        x, edge_ft = ops._f32(x).contiguous(), ops._f32(edge_ft).contiguous()
        n, d = x.shape
        if edge_ft.shape != (csr.num_edges, d) or n != csr.num_nodes:
            raise ValueError(f"CGC shapes: x {tuple(x.shape)}, edge_ft {tuple(edge_ft.shape)}, "
                             f"csr {csr.num_nodes} nodes / {csr.num_edges} edges")
        w = torch.cat([wv, wm]).contiguous()                      # [2D, 3D]
        b = torch.cat([bv, bm]).contiguous()
        ps = dense.linear_fwd(x, w, 2 * d, d, w_off=0, ld=3 * d)
        pr = dense.linear_fwd(x, w, 2 * d, d, w_off=d, ld=3 * d, bias=b)
        ep = dense.linear_fwd(edge_ft, w, 2 * d, d, w_off=2 * d, ld=3 * d)
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
        g = ops._f32(g).contiguous()
        dz = torch.empty(csr.num_edges, 2 * d, device=x.device, dtype=torch.float32)
        gr = torch.empty(n, 2 * d, device=x.device, dtype=torch.float32)
        tok = ops.TIMER.start("cgc_bwd")
        _lib.check(_lib.load().eelg_cgc_bwd(
            _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ep), _lib.ptr(csr.sender), _lib.ptr(csr.rowptr),
            _lib.ptr(row_scale), n, d, _lib.ptr(g), _lib.ptr(dz), _lib.ptr(gr), _lib.stream(g)), "cgc_bwd")
        ops.TIMER.stop(tok)
        gs = ops.segment_sum_csr(dz, csr.srowptr, n, idx=csr.sperm)   # per-sender sums of dz
        dws, dwr, db = _cgc_dw(x, gs, gr, True)
        dwe = dense.linear_bwd_w(edge_ft, dz)
        dw = torch.cat([dws, dwr, dwe], dim=1)
        dx = _cgc_dx(gs, gr, w, d)
        dedge = dense.linear_bwd_x(dz, w, 2 * d, d, w_off=2 * d, ld=3 * d)
        return dx, dedge, dw[:d], db[:d], dw[d:], db[d:], None, None


class _CGCConvEF(torch.autograd.Function):
    """The model path: edge features in factored form (``eelg_cgc_fwd_ef``), ``ef`` [E, 8] =
    [e5 | 1 | 0 | 0] (data) and ``ea`` [8, 2D] = [W5^T W_e^T ; b5 W_e^T ; 0] (a differentiable
    function of the edge embedding and the layer's edge block, formed by ``_edge_factor``).  Its
    gradient is ef^T dz, read off the same dz the node blocks use."""

    @staticmethod
    def forward(ctx, x, ea, wv, bv, wm, bm, ef, csr: ops.EdgeCSR, row_scale: Optional[torch.Tensor],
                residual: bool = False):
        """``residual``: return x + conv(x) (the models' layer residual, cgc_modified.py:77), the
        add done in the aggregation kernel's store and its gradient in grad-x's epilogue"""
        x = ops._f32(x).contiguous()
        ea = ops._f32(ea).contiguous()
        ef = ops._f32(ef).contiguous()       # read as a raw [E, 8] fp32 array by the kernels
        n, d = x.shape
        if ef.shape != (csr.num_edges, 8) or ea.shape != (8, 2 * d) or n != csr.num_nodes:
            raise ValueError(f"CGC (factored edges) shapes: x {tuple(x.shape)}, ef {tuple(ef.shape)}, "
                             f"ea {tuple(ea.shape)}, csr {csr.num_nodes} nodes / {csr.num_edges} edges")
        w = torch.cat([wv, wm]).contiguous()
        b = torch.cat([bv, bm]).contiguous()
        ps = dense.linear_fwd(x, w, 2 * d, d, w_off=0, ld=3 * d)
        pr = dense.linear_fwd(x, w, 2 * d, d, w_off=d, ld=3 * d, bias=b)
        agg = torch.empty(n, d, device=x.device, dtype=torch.float32)
        tok = ops.TIMER.start("cgc_fwd_res" if residual else "cgc_fwd")
        if residual:
            _lib.check(_lib.load().eelg_cgc_fwd_ef_res(
                _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ef), _lib.ptr(ea), _lib.ptr(csr.sender),
                _lib.ptr(csr.rowptr), _lib.ptr(row_scale), n, d, _lib.ptr(x), _lib.ptr(agg),
                _lib.stream(agg)), "cgc_fwd_ef_res")
        else:
            _lib.check(_lib.load().eelg_cgc_fwd_ef(
                _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ef), _lib.ptr(ea), _lib.ptr(csr.sender),
                _lib.ptr(csr.receiver), _lib.ptr(csr.rowptr), _lib.ptr(row_scale), n, d, _lib.ptr(agg),
                _lib.stream(agg)), "cgc_fwd_ef")
        ops.TIMER.stop(tok)
        ctx.save_for_backward(x, ea, ef, ps, pr, w, row_scale)
        ctx.csr, ctx.residual = csr, residual
        return agg

    @staticmethod
    def backward(ctx, g):
        x, ea, ef, ps, pr, w, row_scale = ctx.saved_tensors
        csr = ctx.csr
        n, d = x.shape
        g = ops._f32(g).contiguous()
        dz = torch.empty(csr.num_edges, 2 * d, device=x.device, dtype=torch.float32)
        gr = torch.empty(n, 2 * d, device=x.device, dtype=torch.float32)
        lib = _lib.load()
        nparts = int(lib.eelg_cgc_bwd_ef_parts(n))
        dea_part = torch.empty(nparts, 6, 2 * d, device=x.device, dtype=torch.float32)
        tok = ops.TIMER.start("cgc_bwd")
        _lib.check(lib.eelg_cgc_bwd_ef(
            _lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ef), _lib.ptr(ea), _lib.ptr(csr.sender),
            _lib.ptr(csr.receiver), _lib.ptr(csr.rowptr), _lib.ptr(row_scale), n, d, _lib.ptr(g),
            _lib.ptr(dz), _lib.ptr(gr), _lib.ptr(dea_part), _lib.stream(g)), "cgc_bwd_ef")
        ops.TIMER.stop(tok)
        gs = ops.segment_sum_csr(dz, csr.srowptr, n, idx=csr.sperm)
        dws, dwr, db = _cgc_dw(x, gs, gr, True)
        # d ea = ef^T dz: the kernel's per-workgroup partials (rows 0..5), summed in a fixed order
        dea = torch.cat([ops.sum_rows(dea_part) if nparts else dea_part.new_zeros(6, 2 * d),
                         dea_part.new_zeros(2, 2 * d)])
        zero = torch.zeros(2 * d, d, device=x.device, dtype=torch.float32)
        dw = torch.cat([dws, dwr, zero], dim=1)                   # the edge block: through ea
        dx = _cgc_dx(gs, gr, w, d, g if ctx.residual else None)
        return dx, dea, dw[:d], db[:d], dw[d:], db[d:], None, None, None, None


def _edge_factor(edge_emb: torch.nn.Linear, we: torch.Tensor) -> torch.Tensor:
    """ea [8, 2D] with [e5 | 1 | 0 | 0] @ ea = (e5 W5^T + b5) W_e^T: rows 0..4 = W5^T W_e^T, row 5
    = b5 W_e^T, rows 6..7 zero.  Broadcast products and sums (no GEMM); autograd carries the
    gradient to the edge embedding and to the layer's edge block."""
    w5, b5 = edge_emb.weight, edge_emb.bias                       # [D, 5], [D]
    a = (w5.t()[:, None, :] * we[None, :, :]).sum(-1)           # [5, 2D]
    c = (we * b5[None, :]).sum(-1)                               # [2D]
    pad = torch.zeros(2, we.shape[0], device=we.device, dtype=we.dtype)
    return torch.cat([a, c[None], pad], dim=0)


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

    def _scale(self, csr: ops.EdgeCSR) -> Optional[torch.Tensor]:
        if self.reduction != "mean":
            return None
        deg = (csr.rowptr[1:] - csr.rowptr[:-1]).to(torch.float32)
        return 1.0 / deg.clamp_min(1.0)

    def forward(self, x: torch.Tensor, edge_index: EdgeIndex, edge_ft: torch.Tensor) -> torch.Tensor:
        ops._require_device(x)
        csr, edge_ft = as_csr(edge_index, x.shape[0], edge_ft)
        return _CGCConv.apply(x, edge_ft, self.fc_values.weight, self.fc_values.bias,
                              self.fc_multip.weight, self.fc_multip.bias, csr, self._scale(csr))

    def edge_block(self) -> torch.Tensor:
        """W_e [2D, D]: the edge-feature columns of [W_values; W_multip]"""
        d = self.fc_values.out_features
        return torch.cat([self.fc_values.weight[:, 2 * d:], self.fc_multip.weight[:, 2 * d:]])

    def forward_factored(self, x: torch.Tensor, csr: ops.EdgeCSR, ef: torch.Tensor,
                         ea: torch.Tensor, residual: bool = False) -> torch.Tensor:
        """The same layer on factored edge features (``_CGCConvEF``): ``ef`` [E, 8] =
        [e5 | 1 | 0 | 0] in CSR order, ``ea`` = ``_edge_factor(edge embedding, edge_block())``.
        ``residual``: x + layer(x), added inside the kernels."""
        ops._require_device(x)
        return _CGCConvEF.apply(x, ea, self.fc_values.weight, self.fc_values.bias,
                                self.fc_multip.weight, self.fc_multip.bias, ef, csr,
                                self._scale(csr), residual)


def _head(hidden: int) -> torch.nn.Sequential:
    return torch.nn.Sequential(dense.Linear(hidden, 128), torch.nn.Softplus(),
                               dense.Linear(128, 64), torch.nn.Softplus(),
                               dense.Linear(64, 32), torch.nn.Softplus(),
                               dense.Linear(32, 21))


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
        # K = 1 / 3 inputs: broadcast multiply-adds; the edge embedding's parameters enter each
        # layer through _edge_factor (the [E, hid] edge features are never formed)
        self.node_ft_embedding = dense.SmallInLinear(self.node_inputs, hid)
        self.edge_ft_embedding = torch.nn.Linear(5, hid)
        self.cgc_layers = torch.nn.ModuleList(
            [CGCLayer(hid, hid, params.interaction_reduction) for _ in range(params.message_passes)])
        self.global_reduction = params.global_reduction
        self.mlp = _head(hid)

    def _encode(self, batch, node_in):
        """(csr, node embedding, ef [E, 8] = [e5 | 1 | 0 | 0] in CSR order)"""
        from .model import EnergyEquivGNN
        csr = EnergyEquivGNN.edge_graph(batch)
        e5 = _edge_inputs(batch, csr)
        ef = torch.cat([e5, torch.ones_like(e5[:, :1]), torch.zeros_like(e5[:, :2])], dim=1).contiguous()
        return csr, self.node_ft_embedding(node_in), ef

    def _edge_factors(self):
        """every layer's ``ea`` [8, 2D] (``_edge_factor``) in one batched pass: the edge embedding
        is shared, so the products and sums of the layers (and their backward) run as one set of
        launches instead of one per layer"""
        we = torch.stack([layer.edge_block() for layer in self.cgc_layers])   # [L, 2D, D]
        w5, b5 = self.edge_ft_embedding.weight, self.edge_ft_embedding.bias    # [D, 5], [D]
        a = (w5.t()[None, :, None, :] * we[:, None, :, :]).sum(-1)           # [L, 5, 2D]
        c = (we * b5[None, None, :]).sum(-1)                                 # [L, 2D]
        pad = torch.zeros(we.shape[0], 2, we.shape[1], device=we.device, dtype=we.dtype)
        return torch.cat([a, c[:, None], pad], dim=1)                        # [L, 8, 2D]

    def _layer(self, i, h, csr, ef, residual: bool = False, ea=None):
        """layer i (h + layer_i(h) when ``residual``); ``ea``: its edge factor if precomputed"""
        layer = self.cgc_layers[i]
        if ea is None:
            ea = _edge_factor(self.edge_ft_embedding, layer.edge_block())
        if residual and not CGC_FUSED_RES:
            return h + layer.forward_factored(h, csr, ef, ea)
        return layer.forward_factored(h, csr, ef, ea, residual)

    def _pool(self, h, batch):
        return ops.graph_pool(h, batch.batch, batch.num_graphs, self.global_reduction)


class CrystGraphConv(_CGCBase):
    """mCGC (``cgc_modified.py:27-88``): node features from ``node_attrs``, no residual on
    the first layer, 21 outputs -> symmetric 6x6 -> ``positive`` ('square' | 'none')."""
    inds_val = INDS_VAL
    node_inputs = 1

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        csr, h, ef = self._encode(batch, batch.node_attrs)
        ea = self._edge_factors() if CGC_EA_BATCH else [None] * len(self.cgc_layers)
        h = self._layer(0, h, csr, ef, ea=ea[0])
        for i in range(1, len(self.cgc_layers)):
            h = self._layer(i, h, csr, ef, residual=True, ea=ea[i])   # h + layer_i(h)
        a = self.mlp(self._pool(h, batch))[:, self.inds_val]
        if self.params.positive == "square":
            return {"stiffness": mat_square(a)}
        if self.params.positive == "none":
            return {"stiffness": a}
        raise NotImplementedError(self.params.positive)


class CrystGraphConvVanilla(_CGCBase):
    """CGC (``cgc_vanilla.py:27-74``): node features from ``positions``, residual on every
    layer, 21 raw outputs."""
    node_inputs = 3

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        csr, h, ef = self._encode(batch, batch.positions)
        ea = self._edge_factors() if CGC_EA_BATCH else [None] * len(self.cgc_layers)
        for i in range(len(self.cgc_layers)):
            h = self._layer(i, h, csr, ef, residual=True, ea=ea[i])   # h + layer_i(h)
        return {"stiffness": self.mlp(self._pool(h, batch))}
