"""Dense ``torch.nn.Linear`` layers on the in-tree fp32 MFMA linear kernels (``eelg_linear_*``).

The CGC / mCGC benchmark models (``scripts/benchmark_models/cgc_modified.py:11-88``,
``cgc_vanilla.py:11-74``) are chains of plain Linear layers around the edge convolution.  A
Linear ``y = x W^T + b`` is the channel-mixing linear of ``o3.Linear`` with one scalar slot
(``d = 1``), so the same kernels run it: the descriptor reads ``W`` in torch layout
(``B[k][j] = W[j, k]``: ``ldk = 1``, ``ldj = ld``), the gradient w.r.t. ``x`` swaps the strides
(``gx = gy W``), and the weight gradient comes from ``eelg_linear_bwd_w`` as per-node-slice
partials summed in a fixed order (``ops.sum_rows``), so no library GEMM runs.  ``w_off`` / ``ld``
address a column block of a wider weight (the sender / receiver / edge blocks of the CGC layer's
``[2D, 3D]`` weight) without a copy.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import _lib, ops

LINW_WG = 4096          # weight-gradient workgroups (node slices x 32x32 tiles), as o3.Linear
LINW_MAX_SLICES = 128
# forward / grad-x with K in [LIN_X6_MINK, 320] (whole 32-wide chunks, n_out % 32 == 0) on the
# fp32-accurate split-bf16 packed kernel (eelg_linear_fwd_pk), the weight packed per call
# (~7 us; the CGC layer's [W_v; W_m] is a fresh concatenation every forward, so a cache keyed
# by address and version could hand back a stale pack).  The CGC projections (K = 128 / 256 at
# 262k rows) run at ~144 TFLOP/s on the fp32 MFMA, its peak; the split form does a 16-deep K
# block in 3/8 of the MFMA cycles.  r05v, 150-step runs alternating on one box: 30,001 / 30,513
# / 30,907 vs 29,003 / 29,356 / 29,393 graphs/s (fp32); traced linear time 3.29 vs 3.73 ms/step
# (r05s).  EELG_DENSE_X6=0: the fp32 kernels.
DENSE_X6 = os.environ.get("EELG_DENSE_X6", "1") != "0"
# the weight gradient on the same split form when K (= the Linear's input width) is 32..128
# and there are enough rows for the MFMA tiles to pay: workgroups of 128 output rows x a split
# of rows (eelg_linear_bwd_w_x6)
LINW_X6_MINROWS = 4096
LINW_X6_WG = int(os.environ.get("EELG_LINW_X6_WG", "512"))


def _slot_desc(n_out: int, k: int, w_off: int, ldk: int, ldj: int, bias: bool, n: int):
    d = _lib.LinDesc()
    d.n_slots = 1
    d.max_jt = (n_out + 31) // 32
    d.max_rows = n
    sl = d.slot[0]
    sl.y_off, sl.n_out, sl.d = 0, n_out, 1
    sl.bias_off = 0 if bias else -1
    sl.n_src = 1
    s = sl.src[0]
    s.x_off, s.k, s.w_off, s.ldk, s.ldj, s.alpha = 0, k, w_off, ldk, ldj, 1.0
    return d


def _x6(x, w, bias, res, n, y, n_out, k, desc) -> bool:
    from .o3 import LIN_X6_MINK
    if not (DENSE_X6 and k % 32 == 0 and LIN_X6_MINK <= k <= 320 and n_out % 32 == 0
            and x.shape[1] % 4 == 0 and x.data_ptr() % 16 == 0 and y.data_ptr() % 16 == 0
            and (res is None or res.data_ptr() % 16 == 0)):
        return False
    lib = _lib.load()
    pk = torch.empty(3, int(lib.eelg_linear_pack_size(ctypes.byref(desc))), device=w.device,
                     dtype=torch.bfloat16)
    _lib.check(lib.eelg_linear_pack(_lib.ptr(w), ctypes.byref(desc), _lib.ptr(pk), _lib.stream(pk)),
               "dense_pack")
    _lib.check(lib.eelg_linear_fwd_pk(
        _lib.ptr(x), x.shape[1], _lib.ptr(pk), _lib.ptr(bias), _lib.ptr(res), n, _lib.ptr(y), n_out,
        ctypes.byref(desc), _lib.stream(y)), "dense_fwd_pk")
    return True


def linear_fwd(x: torch.Tensor, w: torch.Tensor, n_out: int, k: int, w_off: int = 0,
               ld: Optional[int] = None, bias: Optional[torch.Tensor] = None,
               res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x[:, :k] @ W_blk^T (+ bias) (+ res)`` with ``W_blk[j, c] = w.flat[w_off + j * ld + c]``
    (a column block of a row-major ``[n_out, ld]`` weight)."""
    ld = k if ld is None else ld
    n = x.shape[0]
    y = torch.empty(n, n_out, device=x.device, dtype=torch.float32)
    desc = _slot_desc(n_out, k, w_off, 1, ld, bias is not None, n)
    if _x6(x, w, bias, res, n, y, n_out, k, desc):
        return y
    _lib.check(_lib.load().eelg_linear_fwd_res(
        _lib.ptr(x), x.shape[1], _lib.ptr(w), _lib.ptr(bias), _lib.ptr(res), n, _lib.ptr(y), n_out,
        ctypes.byref(desc), _lib.stream(y)), "dense_fwd")
    return y


def linear_bwd_x(gy: torch.Tensor, w: torch.Tensor, n_out: int, k: int, w_off: int = 0,
                 ld: Optional[int] = None, res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``gy @ W_blk (+ res)``: the gradient of ``linear_fwd`` w.r.t. ``x`` ([N, k])."""
    ld = k if ld is None else ld
    n = gy.shape[0]
    gx = torch.empty(n, k, device=gy.device, dtype=torch.float32)
    desc = _slot_desc(k, n_out, w_off, ld, 1, False, n)
    if _x6(gy, w, None, res, n, gx, k, n_out, desc):
        return gx
    _lib.check(_lib.load().eelg_linear_fwd_res(
        _lib.ptr(gy), gy.shape[1], _lib.ptr(w), None, _lib.ptr(res), n, _lib.ptr(gx), k,
        ctypes.byref(desc), _lib.stream(gx)), "dense_bwd_x")
    return gx


def linear_bwd_w(x: torch.Tensor, gy: torch.Tensor) -> torch.Tensor:
    """``gy^T @ x`` ([n_out, k], torch weight layout) over the rows of ``x`` [N, k] / ``gy``
    [N, n_out]: node-slice partials of ``x^T gy`` (``eelg_linear_bwd_w``) summed in a fixed order,
    then transposed."""
    n, k = x.shape
    n_out = gy.shape[1]
    if n == 0:
        return torch.zeros(n_out, k, device=x.device, dtype=torch.float32)
    if DENSE_X6 and k in (32, 64, 96, 128) and n >= LINW_X6_MINROWS:
        # split-bf16 MFMA (eelg_linear_bwd_w_x6): about LINW_X6_WG workgroups of 128 output rows
        # x one row split each, partials [splits, n_out, k] summed in a fixed order
        ntile = -(-n // 32)
        nblk = -(-n_out // 128)
        tps = max(1, -(-ntile // max(1, LINW_X6_WG // nblk)))
        splits = -(-ntile // tps)
        part = torch.empty(splits, n_out * k, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().eelg_linear_bwd_w_x6(
            _lib.ptr(gy), gy.stride(0), _lib.ptr(x), x.stride(0), n, n_out, k, tps, _lib.ptr(part),
            _lib.stream(part)), "dense_bwd_w_x6")
        return ops.sum_rows(part).view(n_out, k)
    tiles = ((k + 31) // 32) * ((n_out + 31) // 32)
    slices = max(1, min((n + 31) // 32, -(-LINW_WG // tiles), LINW_MAX_SLICES))
    nps = -(-n // slices)
    slices = -(-n // nps)
    wd = _lib.LinWDesc()
    wd.n_ins, wd.max_jt, wd.max_ut, wd.max_rows = 1, (n_out + 31) // 32, (k + 31) // 32, n
    e = wd.ins[0]
    e.x_off, e.k, e.g_off, e.n_out, e.d, e.w_off, e.alpha = 0, k, 0, n_out, 1, 0, 1.0
    part = torch.empty(slices, k * n_out, device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().eelg_linear_bwd_w(
        _lib.ptr(x), k, _lib.ptr(gy), n_out, n, nps, _lib.ptr(part), slices, k * n_out,
        ctypes.byref(wd), _lib.stream(part)), "dense_bwd_w")
    return ops.sum_rows(part).view(k, n_out).t()


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        x = ops._f32(x).contiguous()
        n_out, k = weight.shape
        y = linear_fwd(x, weight.contiguous(), n_out, k, bias=bias)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = ops._f32(gy).contiguous()
        n_out, k = weight.shape
        gx = linear_bwd_x(gy, weight.contiguous(), n_out, k) if ctx.needs_input_grad[0] else None
        gw = linear_bwd_w(x, gy) if ctx.needs_input_grad[1] else None
        gb = ops.sum_rows(gy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class Linear(torch.nn.Linear):
    """``torch.nn.Linear`` (same parameters, initialisation and state_dict) whose forward and
    backward run on the HIP linear kernels; device tensors only (no CPU fallback)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ops._require_device(x)
        shape = x.shape
        y = _DenseFn.apply(x.reshape(-1, shape[-1]), self.weight, self.bias)
        return y.view(*shape[:-1], self.out_features)


# the K <= 8 node-embedding linear as addcmul + sum_rows (1) or autograd's broadcast form (0)
SMALLIN_FUSED = os.environ.get("EELG_SMALLIN_FUSED", "1") != "0"


class _SmallIn(torch.autograd.Function):
    """``x @ W^T + b`` for K <= 8 inputs that need no gradient (node attributes / positions):
    forward one ``addcmul`` per input column onto the bias, backward the weight and bias
    gradients as fixed-order column sums on ``ops.sum_rows`` (one [N, K * n_out] product for the
    weight) instead of autograd's broadcast multiplies and ``torch.sum`` reductions."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        n, k = x.shape
        if bias is not None:
            out = torch.addcmul(bias, x[:, :1], weight[:, 0])
        else:
            out = x[:, :1] * weight[:, 0]
        for c in range(1, k):
            out.addcmul_(x[:, c: c + 1], weight[:, c])
        ctx.save_for_backward(x)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        gy = ops._f32(gy).contiguous()
        n, k = x.shape
        gw = gb = None
        if ctx.needs_input_grad[1]:
            prod = (x.float()[:, :, None] * gy[:, None, :]).reshape(n, -1)     # [N, K * n_out]
            gw = ops.sum_rows(prod).view(k, -1).t()
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = ops.sum_rows(gy)
        return None, gw, gb


def small_in_linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """``x @ W^T + b`` for a handful of inputs (the node embeddings, K = 1 or 3) as broadcast
    multiply-adds: a K-term outer product is elementwise work, not a GEMM."""
    if SMALLIN_FUSED and x.is_cuda and not x.requires_grad and x.dtype == torch.float32 and x.shape[1] <= 8:
        return _SmallIn.apply(x, weight, bias)
    out = bias.expand(x.shape[0], -1) if bias is not None else None
    for c in range(x.shape[1]):
        term = x[:, c: c + 1] * weight[:, c]
        out = term if out is None else out + term
    return out


class SmallInLinear(torch.nn.Linear):
    """``torch.nn.Linear`` with few inputs (K <= 8) evaluated by ``small_in_linear``."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return small_in_linear(x, self.weight, self.bias)


__all__ = ["Linear", "SmallInLinear", "linear_fwd", "linear_bwd_x", "linear_bwd_w",
           "small_in_linear"]
