"""``GNN_Head`` / ``EnergyEquivGNN`` (reference ``gnn/model.py:26-161``), MI355X-native.

Same constructor (``params`` Namespace), module tree, parameter names and
``forward(batch) -> {'stiffness': [B, 6, 6]}`` as the reference.  Per forward:

1. the batch's receiver-sorted CSR is built once on the device (or taken from
   ``batch.csr`` when the collate already made it) and every edge tensor is
   permuted once into that order;
2. ``eelg_edge_embed`` computes edge vectors, the 2x6 Gaussian edge features
   and the l<=lmax spherical harmonics in one kernel;
3. each ``MACELayer`` runs the fused HIP interaction and the HIP symmetric
   contraction; channel-mixing linears and the readout tail are GEMMs;
4. the per-graph mean pool is ``eelg_segment_sum_csr`` over the sorted
   ``batch`` vector.
"""
from __future__ import annotations

import os
from argparse import Namespace
from typing import Any, Dict

import torch

from . import ops
from .blocks import (Cart_4_to_Mandel, GeneralNonLinearReadoutBlock, MACELayer, PositiveLayer,
                     Spherical_to_Cartesian, as_csr)
from .irreps import Irreps
from .o3 import Linear


def storage_dtype(params: Namespace) -> torch.dtype:
    """Optional ``params.storage_dtype`` ('float32' default, or 'bfloat16'): storage type of
    the edge-sized interaction tensors (BASELINE config 5: bf16 storage, fp32 accumulate).
    Not a reference field; the reference path is all fp32."""
    name = str(getattr(params, "storage_dtype", "float32")).replace("torch.", "")
    table = {"float32": torch.float32, "fp32": torch.float32, "bfloat16": torch.bfloat16,
             "bf16": torch.bfloat16}
    if name not in table:
        raise ValueError(f"storage_dtype {name!r}: expected 'float32' or 'bfloat16'")
    return table[name]


# every layer's radial MLP done before layer 1 starts (they overlap layer 0 only)
RADIAL_AHEAD_OF_LAYER1 = os.environ.get("EELG_RADIAL_BEFORE_L1", "1") != "0"
# every layer's contraction coefficients issued at the start of the forward (GNN_Head._coefficients_ahead)
COEF_AHEAD = os.environ.get("EELG_COEF_AHEAD", "1") != "0"


class GNN_Head(torch.nn.Module):  # noqa: N801
    def __init__(self, params: Namespace) -> None:
        super().__init__()
        self.params = params
        hidden = Irreps(params.hidden_irreps)
        self.number_of_edge_basis = params.num_edge_bases
        node_ft_irreps = Irreps([(hidden.count("0e"), "0e")])
        edge_feats_irreps = Irreps(f"{self.number_of_edge_basis * 2}x0e")
        edge_attr_irreps = Irreps.spherical_harmonics(params.lmax)
        num_features = hidden.count("0e")
        interaction_irreps = (edge_attr_irreps * num_features).sort()[0].simplify()
        readout_irreps = Irreps(params.readout_irreps)
        self.num_interactions = params.message_passes
        storage = storage_dtype(params)

        def layer(inp):
            return MACELayer(inp, edge_attr_irreps, edge_feats_irreps, interaction_irreps, hidden,
                             params.agg_norm_const, params.interaction_reduction, True,
                             params.correlation, MLP_dim=params.inter_MLP_dim,
                             MLP_layers=params.inter_MLP_layers, storage_dtype=storage)

        self.layers = torch.nn.ModuleList([layer(node_ft_irreps)])
        for _ in range(self.num_interactions - 1):
            self.layers.append(layer(hidden))
        self.nonlin_readout = GeneralNonLinearReadoutBlock(hidden, hidden, readout_irreps,
                                                           gate=torch.nn.functional.silu)
        self.global_reduction = params.global_reduction
        self.linear = Linear(readout_irreps, Irreps("2x0e+2x2e+1x4e"), biases=True)
        self.sph_to_cart = Spherical_to_Cartesian()
        self.cart_to_Mandel = Cart_4_to_Mandel()
        self.positive_layer = PositiveLayer(params)

    def _radial_weights_ahead(self, edge_feats):
        """Every layer's radial MLP depends only on the edge features, so all of them run up
        front on a side stream and overlap the VALU-bound interaction / contraction kernels
        of the main stream (their backward runs on that stream too: autograd replays a
        backward op on its forward's stream and inserts the cross-stream waits).  Layer i
        waits for its own weights only."""
        if not (ops.OVERLAP and edge_feats.is_cuda):
            return [None] * self.num_interactions, [None] * self.num_interactions
        main = torch.cuda.current_stream(edge_feats.device)
        side = ops.side_stream(edge_feats.device)
        side.wait_stream(main)
        # edge_feats is made on the main stream and read (and saved for the MLP backward) on
        # the side stream: without this the allocator could hand its block to a main-stream
        # allocation while a side-stream kernel still reads it
        edge_feats.record_stream(side)
        ws, evs = [], []
        with torch.cuda.stream(side):
            for layer in self.layers:
                w = layer.interaction.radial_weights(edge_feats)
                ev = torch.cuda.Event()
                ev.record(side)
                ws.append(w)
                evs.append(ev)
        for w in ws:
            w.record_stream(main)        # allocator: w is also used on the main stream
        return ws, evs

    def _coefficients_ahead(self, device) -> None:
        """Every layer's contraction coefficients (``coef = U_sym W``) depend on the weights
        only: issue them all up front on the coefficient side stream (after the main stream's
        last weight update), so no layer waits on a fresh main -> side -> main round trip."""
        if not (ops.OVERLAP and COEF_AHEAD and device.type == "cuda"):
            return
        main = torch.cuda.current_stream(device)
        side = ops.side_stream(device, 1)
        side.wait_stream(main)
        for layer in self.layers:
            layer.product.symmetric_contractions.coefficients_ahead(side)

    def forward(self, edge_index, node_ft, edge_sh, edge_feats, batch_idx, num_graphs: int):
        csr, edge_sh, edge_feats = as_csr(edge_index, node_ft.shape[0], edge_sh, edge_feats)
        ws, evs = self._radial_weights_ahead(edge_feats)
        self._coefficients_ahead(node_ft.device)

        def run(i, h, residual=None):
            if evs[i] is not None:
                torch.cuda.current_stream(h.device).wait_event(evs[i])
            return self.layers[i](h, csr, edge_sh, edge_feats, tp_weights=ws[i], residual=residual)

        node_ft = run(0, node_ft)
        if RADIAL_AHEAD_OF_LAYER1 and evs[-1] is not None:
            # the later layers' interaction kernels run without the MLP GEMMs beside them
            torch.cuda.current_stream(node_ft.device).wait_event(evs[-1])
        for i in range(1, self.num_interactions):
            # node_ft + layer_i(node_ft) (gnn/model.py:95), the add fused into the layer's
            # last linear
            node_ft = run(i, node_ft, residual=node_ft)
        out = self.nonlin_readout(node_ft)
        graph_ft = ops.graph_pool(out, batch_idx, num_graphs, self.global_reduction)
        stiff = self.sph_to_cart(self.linear(graph_ft))
        return self.positive_layer(self.cart_to_Mandel(stiff))


class _Embed1(torch.autograd.Function):
    """y = b + a w^T for one input feature a [N, 1]: forward torch.addcmul, backward the two
    column sums on ``ops.sum_rows`` (deterministic; torch's reductions were 2 x 33 us per step
    at [32768, 32], r06i).  No gradient w.r.t. the node attributes (data)."""

    @staticmethod
    def forward(ctx, attrs, weight, bias):
        ctx.save_for_backward(attrs)
        ctx.has_bias = bias is not None
        w = weight[:, 0]
        return torch.addcmul(bias, attrs, w) if bias is not None else attrs * w

    @staticmethod
    def backward(ctx, gy):
        from . import ops
        (attrs,) = ctx.saved_tensors
        gy = ops._f32(gy).contiguous()
        gw = ops.sum_rows(gy * attrs).unsqueeze(1) if ctx.needs_input_grad[1] else None
        gb = ops.sum_rows(gy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return None, gw, gb


def _embed(lin: torch.nn.Linear, attrs: torch.Tensor) -> torch.Tensor:
    """``Linear(1 -> 32)`` of the node attributes (``gnn/model.py:122,142``).  With one input
    feature it is an outer product plus bias: one broadcast multiply-add instead of a K = 1
    library GEMM (0.19 ms per step on MI355X for [32768 x 1] x [1 x 32], r02q), and its weight
    and bias gradients are column sums.  Same values (a single product per output plus the bias)."""
    if lin.in_features != 1:
        return lin(attrs)
    if attrs.is_cuda and not attrs.requires_grad:
        return _Embed1.apply(attrs, lin.weight, lin.bias)
    return torch.addcmul(lin.bias, attrs, lin.weight[:, 0]) if lin.bias is not None \
        else attrs * lin.weight[:, 0]


class EnergyEquivGNN(torch.nn.Module):
    def __init__(self, params: Namespace, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        self.params = params
        hidden = Irreps(params.hidden_irreps)
        self.node_ft_embedding = torch.nn.Linear(1, hidden.count("0e"))
        self.number_of_edge_basis = params.num_edge_bases
        self.max_edge_radius = params.max_edge_radius
        self.lmax = params.lmax
        self.stiffness_head = GNN_Head(params)

    @staticmethod
    def edge_graph(batch) -> ops.EdgeCSR:
        """Receiver-sorted CSR of ``batch.edge_index`` on its device (cached on the batch)."""
        n = batch.node_attrs.shape[0]
        ei = batch.edge_index
        dev = ei.device
        # the cache is valid only for this very edge_index: same storage, no in-place edits
        # since (autograd version counter), same node and edge counts, same device
        key = (ei.data_ptr(), ei._version, tuple(ei.shape), n, str(dev))
        cached = getattr(batch, "_eelg_csr", None)
        if cached is not None and getattr(batch, "_eelg_csr_key", None) == key:
            return cached
        pre = getattr(batch, "csr", None)
        if isinstance(pre, dict) and torch.is_tensor(pre.get("perm")):
            csr = ops.EdgeCSR.from_dict({k: (v.to(dev) if torch.is_tensor(v) else v)
                                         for k, v in pre.items()}, n)
        else:
            csr = ops.EdgeCSR.build(batch.edge_index, n)
        try:
            batch._eelg_csr = csr
            batch._eelg_csr_key = key
        except AttributeError:
            pass
        return csr

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        dev = batch.positions.device
        if dev.type != "cuda":
            raise RuntimeError("the EnergyEquivGNN hot path runs only on a HIP device "
                               "(got a CPU batch); move the model and batch to 'cuda'")
        with torch.cuda.device(dev):        # kernels launch on the batch's device
            return self._forward(batch)

    def _forward(self, batch) -> Dict[str, torch.Tensor]:
        csr = self.edge_graph(batch)
        node_ft = _embed(self.node_ft_embedding, batch.node_attrs)
        shifts = batch.shifts[csr.perm]
        radius = batch.edge_attr[csr.perm].reshape(-1)
        edge_sh, edge_feats = ops.edge_embed(batch.positions, csr, shifts, radius, self.lmax,
                                             self.number_of_edge_basis, 0.6, self.max_edge_radius)
        c = self.stiffness_head(csr, node_ft, edge_sh, edge_feats, batch.batch, batch.num_graphs)
        return {"stiffness": c}
