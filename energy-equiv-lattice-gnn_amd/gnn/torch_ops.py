"""Dispatcher-visible form of the fused interaction (TORCH_LIBRARY ops).

``torch.ops.eelg.tp_interaction`` / ``torch.ops.eelg.tp_interaction_bwd`` and
``torch.ops.eelg.segment_sum_csr`` are ``torch.library`` custom ops over the same C-ABI
library the autograd path in ``ops.py`` calls (``eelg_tp_fwd``, ``eelg_tp_bwd`` /
``eelg_tp_bwd_sender``, ``eelg_segment_sum_csr``).  Each has a fake (meta) kernel, so fx
tracing and ``torch.compile`` see output shapes without running HIP code, and the forward op
carries its autograd formula.  Reference call site: ``gnn/blocks.py:591-597``
(``conv_tp(node_feats[sender], edge_attrs, tp_weights)`` + ``scatter(..., receiver) /
agg_norm_const``).  The CSR tensors are ``ops.EdgeCSR``'s fields; ``sh`` is the padded-row view
``ops.edge_embed`` returns (or any [E, nsh] tensor, padded here).
"""
from typing import Tuple

import torch
from torch import Tensor

from . import _lib, ops


def _csr(sender, receiver, rowptr, sperm, srowptr, n_nodes=None) -> "ops.EdgeCSR":
    n = int(srowptr.shape[0]) - 1 if n_nodes is None else n_nodes    # x rows (sender CSR)
    return ops.EdgeCSR(sender, sender, receiver, rowptr, sperm, srowptr, n)


def _info(cfg: int):
    got = _lib._tp_info(cfg)
    if got is None:
        raise _lib.EELGError(f"bad tp config {cfg}")
    return got[0]


@torch.library.custom_op("eelg::tp_interaction", mutates_args=(), device_types="cuda")
def tp_interaction(x: Tensor, sh: Tensor, w: Tensor, sender: Tensor, receiver: Tensor,
                   rowptr: Tensor, sperm: Tensor, srowptr: Tensor, cfg: int,
                   inv_norm: float) -> Tensor:
    csr = _csr(sender, receiver, rowptr, sperm, srowptr)
    return ops._TPInteraction.forward(_Ctx(), x, sh, w, csr, cfg, _info(cfg), inv_norm)


@tp_interaction.register_fake
def _(x, sh, w, sender, receiver, rowptr, sperm, srowptr, cfg, inv_norm):
    return x.new_empty(rowptr.shape[0] - 1, _info(cfg)["dmid"], dtype=torch.float32)


@torch.library.custom_op("eelg::tp_interaction_bwd", mutates_args=(), device_types="cuda")
def tp_interaction_bwd(g: Tensor, x: Tensor, sh: Tensor, w: Tensor, sender: Tensor,
                       receiver: Tensor, rowptr: Tensor, sperm: Tensor, srowptr: Tensor,
                       cfg: int, inv_norm: float) -> Tuple[Tensor, Tensor]:
    ctx = _Ctx()
    ctx.saved_tensors = (x.contiguous(), ops.padded_sh(sh), w.contiguous())
    ctx.csr, ctx.cfg, ctx.info, ctx.inv_norm = (_csr(sender, receiver, rowptr, sperm, srowptr),
                                                cfg, _info(cfg), inv_norm)
    gx, _, gw, *_ = ops._TPInteraction.backward(ctx, g.contiguous())
    return gx, gw


@tp_interaction_bwd.register_fake
def _(g, x, sh, w, sender, receiver, rowptr, sperm, srowptr, cfg, inv_norm):
    return x.new_empty(x.shape, dtype=torch.float32), torch.empty_like(w)


def _setup(ctx, inputs, output):
    x, sh, w, sender, receiver, rowptr, sperm, srowptr, cfg, inv_norm = inputs
    ctx.save_for_backward(x, sh, w, sender, receiver, rowptr, sperm, srowptr)
    ctx.cfg, ctx.inv_norm = cfg, inv_norm


def _backward(ctx, g):
    x, sh, w, sender, receiver, rowptr, sperm, srowptr = ctx.saved_tensors
    gx, gw = torch.ops.eelg.tp_interaction_bwd(g, x, sh, w, sender, receiver, rowptr, sperm,
                                               srowptr, ctx.cfg, ctx.inv_norm)
    return gx, None, gw, None, None, None, None, None, None, None


tp_interaction.register_autograd(_backward, setup_context=_setup)


@torch.library.custom_op("eelg::segment_sum_csr", mutates_args=(), device_types="cuda")
def segment_sum_csr(src: Tensor, rowptr: Tensor, scale: float = 1.0) -> Tensor:
    """out[r] = scale * sum of src rows rowptr[r]:rowptr[r+1] (``eelg_segment_sum_csr``)."""
    return ops.segment_sum_csr(src, rowptr, int(rowptr.shape[0]) - 1, scale=scale)


@segment_sum_csr.register_fake
def _(src, rowptr, scale=1.0):
    return src.new_empty((rowptr.shape[0] - 1,) + tuple(src.shape[1:]), dtype=torch.float32)


def _seg_setup(ctx, inputs, output):
    src, rowptr, scale = inputs
    ctx.save_for_backward(rowptr)
    ctx.n_src, ctx.scale = src.shape[0], scale


def _seg_backward(ctx, g):
    """grad src[j] = scale * g[row of j]; rows outside every segment get 0."""
    (rowptr,) = ctx.saved_tensors
    j = torch.arange(ctx.n_src, device=g.device, dtype=torch.int64)
    row = torch.searchsorted(rowptr[1:].to(torch.int64), j, right=True)
    j0 = (j >= rowptr[0].to(torch.int64)).to(g.dtype).view(-1, *([1] * (g.dim() - 1)))
    gpad = torch.cat([g, g.new_zeros((1,) + tuple(g.shape[1:]))])     # row n: outside
    return gpad[row] * j0 * ctx.scale, None, None


segment_sum_csr.register_autograd(_seg_backward, setup_context=_seg_setup)


class _Ctx:
    """Stand-in for an autograd ctx: lets the custom ops reuse ``ops._TPInteraction``'s
    forward / backward bodies (one launch sequence, not two copies of it)."""

    def save_for_backward(self, *ts):
        self.saved_tensors = ts
