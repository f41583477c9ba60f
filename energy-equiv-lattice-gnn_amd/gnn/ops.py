"""PyTorch autograd wrappers over the C ABI (``include/eelg.h``).

Every op requires HIP device tensors and launches on the current stream.
There is no eager/CPU fallback: a missing library or a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import _lib


class KernelTimer:
    """Optional HIP-event timing of selected launches (used by ``bench.py``).

    Events are recorded on the current stream, the one every op launches on."""

    def __init__(self):
        self.enabled = False
        self.records: Dict[str, list] = {}

    def start(self, name: str):
        if not self.enabled:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return (name, ev)

    def stop(self, tok) -> None:
        if tok is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.records.setdefault(tok[0], []).append((tok[1], ev))

    def summary(self) -> Dict[str, Dict[str, float]]:
        torch.cuda.synchronize()
        out = {}
        for name, pairs in self.records.items():
            ms = [a.elapsed_time(b) for a, b in pairs]
            out[name] = {"count": len(ms), "mean_ms": sum(ms) / len(ms), "total_ms": sum(ms)}
        return out


TIMER = KernelTimer()

# side-stream overlap of independent work (radial MLPs, symmetric-contraction coefficient
# chain and its gradient); EELG_OVERLAP=0 runs everything in line on the current stream
OVERLAP = os.environ.get("EELG_OVERLAP", "1") != "0"
SC_CMAJOR_ON_SIDE = os.environ.get("EELG_SC_CMAJOR_SIDE", "0") != "0"   # measured equal; fused keeps fewer bytes
# the contraction's coefficient gradient on the coefficient side stream (1) or in line (0)
SC_COEF_ON_SIDE = os.environ.get("EELG_SC_COEF_SIDE", "1") != "0"
# radial MLP backward (hidden 64): the chain kernel + weight gradients on the linear kernels (1),
# or the fused small-layer kernel with per-workgroup partials (0)
RADIAL_CHAIN = os.environ.get("EELG_RADIAL_CHAIN", "1") != "0"
# TP backward in sender order (eelg_tp_bwd_sender) instead of per-edge gxe + sender segment sum:
# "1" always, "0" never (default), "auto" for bf16 storage only.  fp32: measured slower (r02s1:
# tp_bws 1.40 ms vs tp_bwd 1.05 + sender sum 0.16 ms; 1832 vs 1862 graphs/s) -- each edge
# gathers its receiver's 29 KB grad_agg row out of receiver order.  bf16 storage (config 5):
# equal speed in round 2 (r02s2: 912.1 vs 912.4 graphs/s), so "auto" was the default, summing
# grad_x in fp32 instead of from per-edge terms rounded to bf16; with round 3-6's edge kernel
# (deeper prefetch, XCD-ordered blocks) the edge path is faster (r08m, two alternating pairs:
# 1145.6 / 1143.7 vs 1130.0 / 1127.9 graphs/s; tp_bwd 1.90 vs tp_bws 2.23 ms per launch)
# edge-order backward: gxe rows stored at their sender-order position (eelg_tp_bwd_sorted), so
# the sender sum reads them contiguously instead of gathering through sperm.  Bitwise-equal
# results; measured equal (r02s3: sender sum 169 -> 137 us, tp_bwd 1036 -> 1128 us from the
# scattered row stores; 1844 / 1855 vs 1844 / 1847 graphs/s), so off by default.
TP_BWD_SPOS = os.environ.get("EELG_TP_BWD_SPOS", "0") != "0"
_TBS = os.environ.get("EELG_TP_BWD_SENDER", "0")
TP_BWD_SENDER = None if _TBS == "auto" else _TBS != "0"
# fused backward of the interaction's output linear and the TP (eelg_tp_bwd_fused): the
# linear's grad-x [N, dmid] is computed per receiver tile into LDS inside the TP backward instead
# of being written to HBM by the linear and read back by tp_bwd.  Measured slower (r09c kbench:
# 1.10 ms vs 0.68 + 0.32 ms for tp_bwd + the linear's grad-x; r09a step 2002 vs ~2190 graphs/s):
# the per-tile MFMA stage is latency-bound at the occupancy its LDS block allows.  Off by default.
TP_BWF = os.environ.get("EELG_TP_BWF", "0") != "0"
# the output linear's grad-x and tp_bwd in C node chunks (C > 1): each chunk's grad_agg rows
# (N / C x 29 KB) are read back by tp_bwd right after the linear wrote them, from the 256 MB
# MALL instead of HBM (chunk edge ranges from one host read of the CSR, cached per graph).
# Bitwise equal to the one-pass kernels; measured slower (r09g, same box, default 2205 / 2200
# graphs/s: C 4 2171, C 8 2121, C 16 2007) -- each extra launch pair adds two kernel tails.
TP_BWC = int(os.environ.get("EELG_TP_BWC", "0"))
_SIDE: Dict[tuple, "torch.cuda.Stream"] = {}


def side_stream(device, which: int = 0) -> "torch.cuda.Stream":
    """Side stream ``which`` of ``device``: 0 = radial MLPs, 1 = contraction coefficients,
    2 = linear weight gradients."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    if (idx, which) not in _SIDE:
        _SIDE[(idx, which)] = torch.cuda.Stream(device=torch.device("cuda", idx))
    return _SIDE[(idx, which)]


def _require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("the EnergyEquivGNN hot path runs only on a HIP device "
                               "(got a CPU tensor); move the model and batch to 'cuda'")


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"expected float32, got {t.dtype}")
    return t.contiguous()


def _a16(t: torch.Tensor) -> torch.Tensor:
    """contiguous fp32 with a 16-byte aligned data pointer (float4 row access), copying a
    misaligned view"""
    t = _f32(t)
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _i32(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.int32).contiguous()


# ---------------------------------------------------------------------------
# edge graph in receiver-sorted order
# ---------------------------------------------------------------------------
@dataclass
class EdgeCSR:
    """Edges in receiver-sorted order.

    ``perm`` maps the sorted order back to the caller's edge order
    (``sorted_edge_j = original_edge[perm[j]]``).  ``rowptr`` is the receiver
    CSR; ``sperm`` / ``srowptr`` group the sorted edges by sender."""
    perm: torch.Tensor
    sender: torch.Tensor
    receiver: torch.Tensor
    rowptr: torch.Tensor
    sperm: torch.Tensor
    srowptr: torch.Tensor
    num_nodes: int

    @property
    def num_edges(self) -> int:
        return int(self.sender.shape[0])

    def sender_pos(self) -> torch.Tensor:
        """[E] int32 inverse of ``sperm``: the sender-order position of each edge (cached)."""
        sp = getattr(self, "_spos", None)
        if sp is None:
            sp = torch.empty_like(self.sperm)
            sp[self.sperm.long()] = torch.arange(self.sperm.shape[0], device=self.sperm.device,
                                                 dtype=self.sperm.dtype)
            self._spos = sp
        return sp

    @staticmethod
    def from_dict(d: Dict, num_nodes: int) -> "EdgeCSR":
        return EdgeCSR(d["perm"], d["sender"], d["receiver"], d["rowptr"], d["sperm"],
                       d["srowptr"], num_nodes)

    @staticmethod
    def build(edge_index: torch.Tensor, num_nodes: int) -> "EdgeCSR":
        from .data import build_edge_csr
        return EdgeCSR.from_dict(build_edge_csr(edge_index, num_nodes), num_nodes)


# ---------------------------------------------------------------------------
# edge embedding (no gradient: positions and radii are data)
# ---------------------------------------------------------------------------
def edge_embed(pos, csr: EdgeCSR, shifts_sorted, radius_sorted, lmax: int, nb: int,
               len_end: float, rad_end: float):
    _require_device(pos, shifts_sorted, radius_sorted)
    if pos.requires_grad or shifts_sorted.requires_grad:
        raise NotImplementedError("gradients w.r.t. positions are not part of the hot path "
                                  "(the reference never differentiates through geometry)")
    e = csr.num_edges
    nsh = (lmax + 1) ** 2
    sh = torch.empty(e, sh_row_stride(nsh), device=pos.device, dtype=torch.float32)
    feats = torch.empty(e, 2 * nb, device=pos.device, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.eelg_edge_embed(
        _lib.ptr(_f32(pos)), _lib.ptr(csr.sender), _lib.ptr(csr.receiver),
        _lib.ptr(_f32(shifts_sorted)), _lib.ptr(_f32(radius_sorted)), e, lmax, nb,
        float(len_end), float(rad_end), _lib.ptr(sh), _lib.ptr(feats), _lib.stream(sh)), "edge_embed")
    return sh[:, :nsh], feats          # [E, nsh] view of the padded rows the TP kernels read


def sh_row_stride(nsh: int) -> int:
    """SH rows are padded to 16 bytes in HBM (float4 loads in the TP kernels)."""
    return (nsh + 3) // 4 * 4


def padded_sh(sh: torch.Tensor) -> torch.Tensor:
    """The padded-row buffer behind ``sh`` ([E, nsh]): the tensor itself when it is already a
    view of padded rows (as ``edge_embed`` returns), else a padded copy."""
    nsh = sh.shape[1]
    nshp = sh_row_stride(nsh)
    if (sh.dtype == torch.float32 and sh.stride() == (nshp, 1) and sh.storage_offset() == 0
            and sh.untyped_storage().nbytes() >= sh.shape[0] * nshp * 4):
        return sh
    out = torch.zeros(sh.shape[0], nshp, device=sh.device, dtype=torch.float32)
    out[:, :nsh] = sh
    return out[:, :nsh]


# ---------------------------------------------------------------------------
# CSR segmented sum
# ---------------------------------------------------------------------------
def segment_sum_csr(src, rowptr, n_rows: int, idx=None, row_scale=None, scale: float = 1.0):
    """fp32 output; ``src`` is fp32, or bf16 (widened exactly, fp32 accumulation)."""
    _require_device(src)
    bf = src.dtype == torch.bfloat16
    src = src.contiguous() if bf else _f32(src)
    width = src[0].numel() if src.shape[0] > 0 else int(torch.tensor(src.shape[1:]).prod())
    out = torch.empty((n_rows,) + tuple(src.shape[1:]), device=src.device, dtype=torch.float32)
    lib = _lib.load()
    fn = lib.eelg_segment_sum_csr_bf16 if bf else lib.eelg_segment_sum_csr
    _lib.check(fn(_lib.ptr(src), _lib.ptr(rowptr), _lib.ptr(idx), _lib.ptr(row_scale), float(scale),
                  n_rows, int(width), _lib.ptr(out), _lib.stream(out)), "segment_sum_csr")
    return out


def segment_sum_long(src: torch.Tensor, rowptr: torch.Tensor, n_rows: int,
                     row_scale: Optional[torch.Tensor] = None, scale: float = 1.0) -> torch.Tensor:
    """``segment_sum_csr`` for few long segments (graph pooling): each segment is split
    into pieces summed in parallel, then combined in a fixed order (deterministic)."""
    _require_device(src)
    src = _f32(src)
    width = src.shape[1]
    n_split = max(1, min(64, -(-2048 // max(n_rows, 1))))
    work = torch.empty(n_rows, n_split, width, device=src.device, dtype=torch.float32)
    out = torch.empty(n_rows, width, device=src.device, dtype=torch.float32)
    tok = TIMER.start("segment_sum_split")
    _lib.check(_lib.load().eelg_segment_sum_split(
        _lib.ptr(src), _lib.ptr(rowptr), None, _lib.ptr(row_scale), float(scale), n_rows, width,
        n_split, _lib.ptr(work), _lib.ptr(out), _lib.stream(out)), "segment_sum_split")
    TIMER.stop(tok)
    return out


class _SegmentMean(torch.autograd.Function):
    """Per-graph mean/sum pool over sorted ``batch`` (``gnn/model.py:100-106``)."""

    @staticmethod
    def forward(ctx, src, ptr32, batch, inv_cnt):
        ctx.save_for_backward(batch, inv_cnt)
        n_rows = ptr32.shape[0] - 1
        if src.shape[0] >= 64 * max(n_rows, 1):          # long segments: split them
            return segment_sum_long(src, ptr32, n_rows, row_scale=inv_cnt)
        return segment_sum_csr(src, ptr32, n_rows, row_scale=inv_cnt)

    @staticmethod
    def backward(ctx, g):
        batch, inv_cnt = ctx.saved_tensors
        return (g * inv_cnt[:, None])[batch], None, None, None


def graph_pool(src, batch, num_graphs: int, reduce: str = "mean"):
    _require_device(src)
    # ``batch`` is sorted (PyG collation), so the segment bounds are a searchsorted: no
    # device -> host sync (bincount sizes its output from the data and would stall the host)
    bounds = torch.arange(num_graphs + 1, device=batch.device, dtype=batch.dtype)
    ptr = torch.searchsorted(batch, bounds).to(torch.int32)
    cnt = (ptr[1:] - ptr[:-1]).to(torch.int64)
    if reduce == "mean":
        inv = 1.0 / cnt.clamp_min(1).to(torch.float32)
    elif reduce in ("sum", "add"):
        inv = torch.ones(num_graphs, device=src.device, dtype=torch.float32)
    elif reduce in ("max", "min", "mul"):
        return segment_pool_order(src, ptr, num_graphs, reduce)
    else:
        raise ValueError(f"global_reduction {reduce!r} not supported "
                         "(torch_scatter reduces: sum, add, mean, max, min, mul)")
    return _SegmentMean.apply(src, ptr, batch, inv)


_ORDER_OPS = {"max": 0, "min": 1, "mul": 2}


class _SegmentOrder(torch.autograd.Function):
    """torch_scatter ``scatter(..., reduce='max'|'min'|'mul')`` over CSR segments of ``src``
    rows (``eelg_segment_order``).  max / min: the first extreme of a segment is kept and the
    whole gradient goes to it (torch_scatter's scatter_max / scatter_min arg); empty segments
    give 0 (max / min) or 1 (mul), as torch_scatter fills rows that receive nothing."""

    @staticmethod
    def forward(ctx, src, rowptr, n_rows: int, op: int, covered: bool):
        src = _f32(src)
        width = src.shape[1]
        out = torch.empty(n_rows, width, device=src.device, dtype=torch.float32)
        arg = (torch.empty(n_rows, width, device=src.device, dtype=torch.int32)
               if op != _ORDER_OPS["mul"] else None)
        _lib.check(_lib.load().eelg_segment_order(_lib.ptr(src), _lib.ptr(rowptr), n_rows, width,
                                                  op, _lib.ptr(out), _lib.ptr(arg),
                                                  _lib.stream(out)), "segment_order")
        ctx.save_for_backward(src, rowptr, arg)
        ctx.n_rows, ctx.op, ctx.covered = n_rows, op, covered
        return out

    @staticmethod
    def backward(ctx, g):
        src, rowptr, arg = ctx.saved_tensors
        g = _f32(g)
        # every row of every segment is written; rows outside all segments must read 0
        gs = torch.empty_like(src) if ctx.covered else torch.zeros_like(src)
        _lib.check(_lib.load().eelg_segment_order_bwd(
            _lib.ptr(src), _lib.ptr(rowptr), _lib.ptr(arg), _lib.ptr(g), ctx.n_rows, src.shape[1],
            ctx.op, _lib.ptr(gs), _lib.stream(gs)), "segment_order_bwd")
        return gs, None, None, None, None


def segment_order(src, rowptr32, n_rows: int, reduce: str, covered: bool = False):
    """``reduce`` in max / min / mul over the CSR segments ``rowptr32`` (int32, [n_rows + 1]).
    ``covered``: the segments cover every row of ``src`` (the backward then skips a zero fill)."""
    _require_device(src)
    if reduce not in _ORDER_OPS:
        raise ValueError(f"segment_order: reduce {reduce!r} (max, min, mul)")
    return _SegmentOrder.apply(src, rowptr32, n_rows, _ORDER_OPS[reduce], covered)


def segment_pool_order(src, ptr32, num_graphs: int, reduce: str):
    """Per-graph max / min / mul pool (``gnn/model.py:100-106`` passes any torch_scatter
    reduce) over the sorted ``batch`` segments ``ptr32``."""
    return segment_order(src, ptr32, num_graphs, reduce)


# ---------------------------------------------------------------------------
# fused interaction: gather -> uvu tensor product -> segmented sum / norm
# ---------------------------------------------------------------------------
class _TPInteraction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, sh, w, csr: EdgeCSR, cfg: int, info: Dict[str, int], inv_norm: float):
        # w: fp32, or bf16 storage (BASELINE config 5; fp32 arithmetic in the kernels)
        agg, x, sh, w = _tp_fwd(x, sh, w, csr, cfg, info, inv_norm)
        ctx.save_for_backward(x, sh, w)
        ctx.csr, ctx.cfg, ctx.info, ctx.inv_norm = csr, cfg, info, inv_norm
        return agg

    @staticmethod
    def backward(ctx, g):
        x, sh, w = ctx.saved_tensors
        csr, info = ctx.csr, ctx.info
        g = _f32(g)
        e = csr.num_edges
        gw = torch.empty_like(w)                       # same storage type as w
        lib = _lib.load()
        sender = TP_BWD_SENDER if TP_BWD_SENDER is not None else w.dtype == torch.bfloat16
        if sender:
            # sender-order pass: grad_x summed per sender in registers, no gxe round trip
            gx = torch.empty(csr.num_nodes, info["din"], device=x.device, dtype=torch.float32)
            bws = lib.eelg_tp_bwd_sender_bf16 if w.dtype == torch.bfloat16 else lib.eelg_tp_bwd_sender
            tok = TIMER.start(f"tp_bwd_sender[din={info['din']}]")
            _lib.check(bws(ctx.cfg, _lib.ptr(x), _lib.ptr(sh), _lib.ptr(w), _lib.ptr(csr.sperm),
                           _lib.ptr(csr.srowptr), _lib.ptr(csr.receiver), csr.num_nodes,
                           _lib.ptr(g), float(ctx.inv_norm), _lib.ptr(gw), _lib.ptr(gx),
                           _lib.stream(gx)), "tp_bwd_sender")
            TIMER.stop(tok)
            return gx, None, gw, None, None, None, None
        gxe = torch.empty(e, info["din"], device=x.device, dtype=w.dtype)
        spos = csr.sender_pos() if TP_BWD_SPOS else None
        bwd = lib.eelg_tp_bwd_sorted_bf16 if w.dtype == torch.bfloat16 else lib.eelg_tp_bwd_sorted
        tok = TIMER.start(f"tp_bwd[din={info['din']}]")
        _lib.check(bwd(ctx.cfg, _lib.ptr(x), _lib.ptr(sh), _lib.ptr(w), _lib.ptr(csr.sender),
                       _lib.ptr(csr.receiver), _lib.ptr(spos), e, _lib.ptr(g), float(ctx.inv_norm),
                       _lib.ptr(gw), _lib.ptr(gxe), _lib.stream(gxe)), "tp_bwd")
        TIMER.stop(tok)
        gx = segment_sum_csr(gxe, csr.srowptr, csr.num_nodes,
                             idx=None if spos is not None else csr.sperm)
        return gx, None, gw, None, None, None, None


def tp_interaction(x, sh, w, csr: EdgeCSR, cfg: int, info: Dict[str, int], inv_norm: float):
    _require_device(x, sh, w)
    return _TPInteraction.apply(x, sh, w, csr, cfg, info, inv_norm)


def _tp_fwd(x, sh, w, csr: EdgeCSR, cfg: int, info: Dict[str, int], inv_norm: float):
    """tp_fwd launch with the input checks of ``_TPInteraction``; returns (agg, x, sh, w) with
    the operands as the kernels read them"""
    bf = w.dtype == torch.bfloat16
    x = _a16(x)
    if bf:
        w = w.contiguous()
        w = w if w.data_ptr() % 16 == 0 else w.clone()
    else:
        w = _a16(w)
    if sh.dtype != torch.float32:
        raise TypeError(f"expected float32 SH, got {sh.dtype}")
    sh = padded_sh(sh)
    n = x.shape[0]
    if x.shape[1] != info["din"] or sh.shape[1] != info["nsh"] or w.shape[1] != info["wn"]:
        raise ValueError(f"shape mismatch: x {tuple(x.shape)} sh {tuple(sh.shape)} "
                         f"w {tuple(w.shape)} vs config {info}")
    if sh.shape[0] != csr.num_edges or w.shape[0] != csr.num_edges or n != csr.num_nodes:
        raise ValueError("edge/node counts do not match the CSR")
    n_out = csr.rowptr.shape[0] - 1
    agg = torch.empty(n_out, info["dmid"], device=x.device, dtype=torch.float32)
    lib = _lib.load()
    tok = TIMER.start(f"tp_fwd[din={info['din']}]")
    fwd = lib.eelg_tp_fwd_bf16 if bf else lib.eelg_tp_fwd
    _lib.check(fwd(cfg, _lib.ptr(x), _lib.ptr(sh), _lib.ptr(w), _lib.ptr(csr.sender),
                   _lib.ptr(csr.rowptr), n_out, float(inv_norm), _lib.ptr(agg), _lib.stream(agg)),
               "tp_fwd")
    TIMER.stop(tok)
    return agg, x, sh, w


def tp_linear_fusable(cfg: int, lin, paths) -> bool:
    """whether ``eelg_tp_bwd_fused`` serves ``lin(tp_interaction(...))`` for TP config ``cfg``:
    generated for it (mul 32), and its slot table (weight offset, alpha, gy offset per TP slot)
    equals what ``lin`` (an ``o3.Linear`` over the TP's output irreps) computes.  ``paths``:
    ``cg.tp_paths`` of the block (slot, l3, out_off).  Cached on the linear, per config (not by
    ``id()``: a freed linear's id can be reused by a new one)."""
    cache = lin.__dict__.setdefault("_bwf_ok", {})
    if cfg not in cache:
        cache[cfg] = _bwf_table_matches(cfg, lin, paths)
    return cache[cfg]


def _bwf_table_matches(cfg: int, lin, paths) -> bool:
    lib = _lib.load()
    wo, al, go = ctypes.c_int(), ctypes.c_float(), ctypes.c_int()
    if lin.bias_slots and any(lin.irreps_out[o].ir.l != 0 for o in lin.bias_slots):
        return False
    ins_of_in = {}
    for t, (i, o) in enumerate(lin.instructions):
        if i in ins_of_in:                 # an input block read by two outputs: not the TP layout
            return False
        ins_of_in[i] = (t, o)
    for p in paths:
        if lib.eelg_tp_bwf_slot(cfg, p.slot, ctypes.byref(wo), ctypes.byref(al), ctypes.byref(go)) != 0:
            return False
        hit = None
        for i, (mul, ir) in enumerate(lin.irreps_in):
            lo = lin._in_off[i]
            if lo <= p.out_off < lo + mul * ir.dim and ir.l == p.l3:
                hit = i
                break
        if hit is None or hit not in ins_of_in:
            return False
        t, o = ins_of_in[hit]
        d = 2 * p.l3 + 1
        q, rem = divmod(p.out_off - lin._in_off[hit], 32 * d)
        mo = lin.irreps_out[o].mul
        if rem or mo != 32 or p.mul != 32:
            return False
        if (wo.value != lin._w_offs[t] + q * 32 * mo or go.value != lin._out_off[o]
                or abs(al.value - lin.alpha[t]) > 1e-6 * lin.alpha[t]):
            return False
    return True


class _TPInteractionLinear(torch.autograd.Function):
    """``lin(tp_interaction(x, sh, w))``: the forward runs tp_fwd and the linear as two kernels;
    the backward runs the linear's weight / bias gradients (side stream) and ONE fused kernel
    for the TP's grad-x / grad-w from the linear's output gradient (``eelg_tp_bwd_fused``)."""

    @staticmethod
    def forward(ctx, x, sh, w, lw, lb, csr: EdgeCSR, cfg: int, info: Dict[str, int],
                inv_norm: float, lin, side, chunks: int = 0):
        agg, x, sh, w = _tp_fwd(x, sh, w, csr, cfg, info, inv_norm)
        y = lin._fwd(agg, lw, lb)
        ctx.save_for_backward(x, sh, w, agg, lw)
        ctx.csr, ctx.cfg, ctx.info, ctx.inv_norm, ctx.lin, ctx.side = csr, cfg, info, inv_norm, lin, side
        ctx.chunks = chunks
        return y

    @staticmethod
    def backward(ctx, gy):
        x, sh, w, agg, lw = ctx.saved_tensors
        csr, info, lin, side = ctx.csr, ctx.info, ctx.lin, ctx.side
        gy = _a16(gy)
        want_w, want_b = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        gW = gb = None
        if want_w or want_b:
            if side is None:
                gW = lin._bwd_w(agg, gy) if want_w else None
                gb = lin._bwd_bias(gy) if want_b else None
            else:
                side.wait_stream(torch.cuda.current_stream(gy.device))
                agg.record_stream(side)
                gy.record_stream(side)
                with torch.cuda.stream(side):
                    gW = lin._bwd_w(agg, gy) if want_w else None
                    gb = lin._bwd_bias(gy) if want_b else None
        gw = torch.empty_like(w)
        if ctx.chunks > 1:
            return _tp_linear_bwd_chunked(ctx, x, sh, w, lw, gy, gw) + (gW, gb) + (None,) * 7
        lwc = lw.detach().contiguous()
        if lwc.data_ptr() % 16:
            lwc = lwc.clone()
        gxe = torch.empty(csr.num_edges, info["din"], device=x.device, dtype=w.dtype)
        lib = _lib.load()
        bwf = lib.eelg_tp_bwd_fused_bf16 if w.dtype == torch.bfloat16 else lib.eelg_tp_bwd_fused
        tok = TIMER.start(f"tp_bwf[din={info['din']}]")
        _lib.check(bwf(ctx.cfg, _lib.ptr(x), _lib.ptr(sh), _lib.ptr(w), _lib.ptr(csr.sender),
                       _lib.ptr(csr.receiver), _lib.ptr(csr.rowptr), csr.num_nodes, _lib.ptr(gy), _lib.ptr(lwc),
                       float(ctx.inv_norm), _lib.ptr(gw), _lib.ptr(gxe), _lib.stream(gxe)),
                   "tp_bwd_fused")
        TIMER.stop(tok)
        gx = segment_sum_csr(gxe, csr.srowptr, csr.num_nodes, idx=csr.sperm)
        return gx, None, gw, gW, gb, None, None, None, None, None, None, None


def _chunk_bounds(csr: EdgeCSR, chunks: int):
    """[(n0, n1, e0, e1)]: ``chunks`` receiver ranges of about equal edge counts (one host read
    of rowptr, cached on the CSR)"""
    key = ("_chunks", chunks)
    hit = getattr(csr, "_chunk_cache", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    rp = csr.rowptr.cpu()
    n, e = csr.num_nodes, csr.num_edges
    bounds, n0 = [], 0
    for c in range(1, chunks + 1):
        n1 = n if c == chunks else int(torch.searchsorted(rp, torch.tensor(e * c // chunks, dtype=rp.dtype)))
        n1 = max(n0, min(n, n1))
        if n1 > n0:
            bounds.append((n0, n1, int(rp[n0]), int(rp[n1])))
        n0 = n1
    csr._chunk_cache = (key, bounds)
    return bounds


def _tp_linear_bwd_chunked(ctx, x, sh, w, lw, gy, gw):
    """the unfused kernels (linear grad-x, tp_bwd) per receiver chunk: grad_agg of a chunk is
    consumed while it is still in the MALL; tp_bwd's receiver indices are global, so its grad_agg
    pointer is offset back by the chunk's first row"""
    csr, info, lin = ctx.csr, ctx.info, ctx.lin
    lib = _lib.load()
    dmid, din, wn = info["dmid"], info["din"], info["wn"]
    gxe = torch.empty(csr.num_edges, din, device=x.device, dtype=w.dtype)
    esz = w.element_size()
    bwd = lib.eelg_tp_bwd_sorted_bf16 if w.dtype == torch.bfloat16 else lib.eelg_tp_bwd_sorted
    for n0, n1, e0, e1 in _chunk_bounds(csr, ctx.chunks):
        gagg = lin._bwd_x(gy[n0:n1], lw)
        if e1 <= e0:
            continue
        tok = TIMER.start(f"tp_bwd[din={din}]")
        _lib.check(bwd(ctx.cfg, _lib.ptr(x), sh.data_ptr() + 4 * e0 * sh.stride(0),
                       w.data_ptr() + esz * e0 * wn, csr.sender.data_ptr() + 4 * e0,
                       csr.receiver.data_ptr() + 4 * e0, None, e1 - e0,
                       gagg.data_ptr() - 4 * n0 * dmid, float(ctx.inv_norm),
                       gw.data_ptr() + esz * e0 * wn, gxe.data_ptr() + esz * e0 * din,
                       _lib.stream(gxe)), "tp_bwd")
        TIMER.stop(tok)
    gx = segment_sum_csr(gxe, csr.srowptr, csr.num_nodes, idx=csr.sperm)
    return gx, None, gw


def tp_interaction_linear(x, sh, w, csr: EdgeCSR, cfg: int, info: Dict[str, int],
                          inv_norm: float, lin, chunks: int = 0):
    """``lin(tp_interaction(x, sh, w, csr, cfg, info, inv_norm))`` with the fused backward;
    the caller checks ``tp_linear_fusable`` first.  ``lin``'s weight / bias gradients run on
    its side stream as ``o3.Linear.forward`` arranges them."""
    _require_device(x, sh, w)
    from .o3 import _OnStream
    lw, lb = lin.weight, lin.bias
    side = None
    if OVERLAP and x.is_cuda and torch.is_grad_enabled() and lw.requires_grad:
        side = side_stream(x.device, 2)
        with torch.cuda.stream(side):
            lw = _OnStream.apply(lw, side)
            if lb is not None:
                lb = _OnStream.apply(lb, side)
    return _TPInteractionLinear.apply(x, sh, w, lw, lb, csr, cfg, info, inv_norm, lin, side, chunks)


def per_edge_csr(csr: EdgeCSR) -> EdgeCSR:
    """The same edges with every edge its own receiver segment (``rowptr = 0..E``,
    ``receiver = e``): ``tp_interaction`` over it returns the per-edge messages
    ``conv_tp(x[sender], sh, w) * inv_norm`` as ``[E, dmid]`` rows in receiver-sorted order, and
    its backward reads one grad row per edge.  The sender CSR (grad-x) is the base graph's.
    Cached on ``csr``."""
    pe = getattr(csr, "_per_edge", None)
    if pe is None:
        e = csr.num_edges
        ar = torch.arange(e + 1, device=csr.rowptr.device, dtype=torch.int32)
        pe = EdgeCSR(csr.perm, csr.sender, ar[:e], ar, csr.sperm, csr.srowptr, csr.num_nodes)
        csr._per_edge = pe
    return pe


def in_degree_scale(csr: EdgeCSR) -> torch.Tensor:
    """[N] fp32 ``1 / max(in-degree, 1)`` (torch_scatter 'mean' divides by the clamped count);
    cached on ``csr``."""
    s = getattr(csr, "_inv_deg", None)
    if s is None:
        deg = (csr.rowptr[1:] - csr.rowptr[:-1]).to(torch.float32)
        s = 1.0 / deg.clamp_min(1.0)
        csr._inv_deg = s
    return s


# ---------------------------------------------------------------------------
# symmetric contraction
# ---------------------------------------------------------------------------
class _SymCon(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, coef, cfg: int, info: Dict[str, int], mul: int, side=None):
        x, coef = _a16(x), _a16(coef)
        n = x.shape[0]
        # rows of mul channels x D (Dout) components; info's x_row / out_row are those of mul 32
        if x.shape[1] != mul * info["D"] or coef.shape != (mul, info["coef_ld"]):
            raise ValueError(f"shape mismatch: x {tuple(x.shape)} coef {tuple(coef.shape)} vs mul {mul}, {info}")
        out = torch.empty(n, mul * info["Dout"], device=x.device, dtype=torch.float32)
        lib = _lib.load()
        tok = TIMER.start("sc_fwd")
        _lib.check(lib.eelg_sc_fwd(cfg, _lib.ptr(x), _lib.ptr(coef), n, mul, _lib.ptr(out),
                                   _lib.stream(out)), "sc_fwd")
        TIMER.stop(tok)
        ctx.save_for_backward(x, coef)
        ctx.cfg, ctx.info, ctx.mul, ctx.side = cfg, info, mul, side
        return out

    @staticmethod
    def backward(ctx, g):
        x, coef = ctx.saved_tensors
        g = _a16(g)
        n = x.shape[0]
        lib = _lib.load()
        gx = gcoef = None
        want_x, want_c = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        # the coefficient gradient reads channel-major copies of x / grad_out, which grad-x
        # writes from the tiles it stages anyway
        if want_c:
            xt = torch.empty(ctx.mul * ctx.info["D"], n, device=x.device, dtype=torch.float32)
            gt = torch.empty(ctx.mul * ctx.info["Dout"], n, device=x.device, dtype=torch.float32)
        # with a side stream, the channel-major transposes move there with the coef-grad
        # (off the main chain); in line, grad-x writes them from the tiles it stages anyway
        cm_side = want_c and ctx.side is not None and SC_CMAJOR_ON_SIDE
        if cm_side:
            # launched before grad-x: the transposes need only x and grad_out, and run beside it
            side = ctx.side
            side.wait_stream(torch.cuda.current_stream(x.device))
            for t in (x, g, xt, gt):
                t.record_stream(side)
            with torch.cuda.stream(side):
                _lib.check(lib.eelg_sc_cmajor(ctx.cfg, 0, _lib.ptr(x), n, ctx.mul, _lib.ptr(xt),
                                              _lib.stream(xt)), "sc_cmajor")
                _lib.check(lib.eelg_sc_cmajor(ctx.cfg, 1, _lib.ptr(g), n, ctx.mul, _lib.ptr(gt),
                                              _lib.stream(gt)), "sc_cmajor")
        if want_x:
            gx = torch.empty_like(x)
            tok = TIMER.start("sc_bwd_x")
            fuse = want_c and not cm_side
            _lib.check(lib.eelg_sc_bwd_x_cm(ctx.cfg, _lib.ptr(x), _lib.ptr(coef), _lib.ptr(g), n,
                                            ctx.mul, _lib.ptr(gx),
                                            _lib.ptr(xt) if fuse else None,
                                            _lib.ptr(gt) if fuse else None, _lib.stream(gx)),
                       "sc_bwd_x")
            TIMER.stop(tok)
        if want_c:
            if not (want_x or cm_side):
                tok = TIMER.start("sc_cmajor")
                _lib.check(lib.eelg_sc_cmajor(ctx.cfg, 0, _lib.ptr(x), n, ctx.mul, _lib.ptr(xt),
                                              _lib.stream(xt)), "sc_cmajor")
                _lib.check(lib.eelg_sc_cmajor(ctx.cfg, 1, _lib.ptr(g), n, ctx.mul, _lib.ptr(gt),
                                              _lib.stream(gt)), "sc_cmajor")
                TIMER.stop(tok)
            chunk = ctx.info["coef_chunk"]          # nodes per streamed (LDS-staged) chunk
            nch = int(lib.eelg_sc_bwd_coef_parts(ctx.cfg, n, ctx.mul))   # partial rows (node ranges)
            part = torch.empty(nch, ctx.mul, ctx.info["coef_ld"], device=x.device, dtype=torch.float32)
            if ctx.info["coef_ld"] != ctx.info["nterms"]:
                part[:, :, ctx.info["nterms"]:].zero_()   # the kernel writes terms < nterms
            side = ctx.side if (SC_COEF_ON_SIDE or cm_side) else None
            if side is not None:
                # the coefficient gradient runs on the side stream, where its consumer (the
                # coefficient chain's backward) runs too; the main stream goes on meanwhile
                if not cm_side:
                    side.wait_stream(torch.cuda.current_stream(x.device))
                for t in (xt, gt, part):
                    t.record_stream(side)
            with torch.cuda.stream(side) if side is not None else _nullctx():
                tok = TIMER.start("sc_bwd_coef")
                _lib.check(lib.eelg_sc_bwd_coef(ctx.cfg, _lib.ptr(xt), _lib.ptr(gt), n, ctx.mul,
                                                chunk, _lib.ptr(part), _lib.stream(part)), "sc_bwd_coef")
                TIMER.stop(tok)
                gcoef = sum_rows(part)
        return gx, gcoef, None, None, None, None


def symmetric_contraction(x, coef, cfg: int, info: Dict[str, int], mul: int, side=None):
    """``side``: the stream ``coef`` was produced on (its backward's stream); the
    coefficient gradient is then computed there."""
    _require_device(x, coef)
    return _SymCon.apply(x, coef, cfg, info, mul, side)


class ScgTable:
    """Term table of a symmetric contraction for the table-driven kernels (``eelg_scg_*``,
    correlation 4): ``plan`` = ``cg.symcon_plan`` (terms sorted by output component), ``ls_in``
    / ``ls_out`` the coupling / output l's (one block of ``mul`` channels each, mul-major)."""

    def __init__(self, plan, ls_in, ls_out, mul: int):
        d = _lib.ScgDesc()
        D = sum(2 * l + 1 for l in ls_in)
        Dout = sum(2 * l + 1 for l in ls_out)
        if D > _lib.SCG_MAXD or Dout > _lib.SCG_MAXD:
            raise NotImplementedError(f"table-driven contraction: {D} / {Dout} components per channel "
                                      f"(at most {_lib.SCG_MAXD})")
        d.D, d.Dout, d.mul, d.nterms = D, Dout, mul, len(plan.terms)

        def layout(ls, base, stride):
            a, off = 0, 0
            for l in ls:
                for m in range(2 * l + 1):
                    base[a], stride[a] = mul * off + m, 2 * l + 1
                    a += 1
                off += 2 * l + 1
        layout(ls_in, d.xb, d.xs)
        layout(ls_out, d.ob, d.os)
        self.ldc = max(64, -(-len(plan.terms) // 64) * 64)
        packed, outs = [], []
        for q, (nu, cls, o) in enumerate(plan.terms):
            idx = [i if i >= 0 else D for i in cls] + [D] * (4 - len(cls))
            if len(idx) != 4:
                raise ValueError(f"term {cls}: more than four factors")
            packed.append(idx[0] | idx[1] << 8 | idx[2] << 16 | idx[3] << 24)
            outs.append(o)
        if outs != sorted(outs):
            raise ValueError("table-driven contraction: terms must be sorted by output component")
        for q in range(Dout + 1):
            d.orow[q] = sum(1 for o in outs if o < q)
        pad = self.ldc - len(packed)
        packed += [D | D << 8 | D << 16 | D << 24] * pad
        outs += [Dout] * pad
        self.desc, self.D, self.Dout, self.mul = d, D, Dout, mul
        self._terms = torch.tensor(packed, dtype=torch.int64).to(torch.int32)
        self._outs = torch.tensor(outs, dtype=torch.int32)
        self._dev = {}

    def on(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (self._terms.to(device), self._outs.to(device))
        return self._dev[key]


class _SymConTable(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, coef, tab: ScgTable):
        x, coef = _f32(x), _f32(coef)
        n = x.shape[0]
        if x.shape[1] != tab.mul * tab.D or coef.shape != (tab.mul, tab.ldc):
            raise ValueError(f"shape mismatch: x {tuple(x.shape)} coef {tuple(coef.shape)} vs mul "
                             f"{tab.mul}, D {tab.D}, ldc {tab.ldc}")
        terms, _ = tab.on(x.device)
        out = torch.empty(n, tab.mul * tab.Dout, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().eelg_scg_fwd(ctypes.byref(tab.desc), _lib.ptr(terms), _lib.ptr(x), x.shape[1],
                                            _lib.ptr(coef), tab.ldc, n, _lib.ptr(out), out.shape[1],
                                            _lib.stream(out)), "scg_fwd")
        ctx.save_for_backward(x, coef)
        ctx.tab = tab
        return out

    @staticmethod
    def backward(ctx, g):
        x, coef = ctx.saved_tensors
        tab = ctx.tab
        g = _f32(g)
        n = x.shape[0]
        lib = _lib.load()
        terms, outs = tab.on(x.device)
        gx = gcoef = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _lib.check(lib.eelg_scg_bwd_x(ctypes.byref(tab.desc), _lib.ptr(terms), _lib.ptr(x), x.shape[1],
                                          _lib.ptr(coef), tab.ldc, _lib.ptr(g), g.shape[1], n, _lib.ptr(gx),
                                          _lib.stream(gx)), "scg_bwd_x")
        if ctx.needs_input_grad[1]:
            nch = max(1, -(-n // _lib.SCG_CHUNK))
            part = torch.zeros(nch, tab.mul, tab.ldc, device=x.device, dtype=torch.float32)
            _lib.check(lib.eelg_scg_bwd_coef(ctypes.byref(tab.desc), _lib.ptr(terms), _lib.ptr(outs), tab.ldc,
                                             _lib.ptr(x), x.shape[1], _lib.ptr(g), g.shape[1], n,
                                             _lib.ptr(part), _lib.stream(part)), "scg_bwd_coef")
            gcoef = sum_rows(part)
        return gx, gcoef, None


def symmetric_contraction_table(x, coef, tab: ScgTable):
    """The table-driven contraction (correlation 4): ``x`` [N, mul*D] rows, ``coef`` [mul, tab.ldc]."""
    _require_device(x, coef)
    return _SymConTable.apply(x, coef, tab)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


# ---------------------------------------------------------------------------
# radial MLP (conv_tp_weights, gnn/blocks.py:537-549)
# ---------------------------------------------------------------------------
def _wgrad(g: torch.Tensor, x: torch.Tensor, chunk: int = 512) -> torch.Tensor:
    """g^T @ x over a long row dimension as a split-K batched GEMM + fixed-order sum (the CGC
    models' weight gradients, gnn/cgc.py; library GEMMs pick no split-K for
    [64 x 131072] @ [131072 x 64] and run on a few CUs)."""
    e = g.shape[0]
    c = e // chunk
    acc = torch.promote_types(g.dtype, torch.float32)     # bf16 operands: fp32 sums
    out = None
    if c > 1:
        m = c * chunk
        prod = torch.bmm(g[:m].view(c, chunk, -1).transpose(1, 2), x[:m].view(c, chunk, -1))
        out = sum_rows(prod) if prod.dtype == torch.float32 else prod.sum(0, dtype=acc)
        g, x = g[m:], x[m:]
    if g.shape[0]:
        rest = (g.t() @ x).to(acc)
        out = rest if out is None else out + rest
    return out if out is not None else torch.zeros(g.shape[1], x.shape[1], device=g.device,
                                                   dtype=acc)


def split_bf16x3(t: torch.Tensor) -> torch.Tensor:
    """[3, *t.shape] bf16 parts of an fp32 tensor with t == parts.sum(0) exactly
    (``eelg_split_bf16x3``): the operand form of the fp32-accurate bf16 MFMA GEMMs."""
    _require_device(t)
    t = _f32(t)
    parts = torch.empty((3,) + tuple(t.shape), device=t.device, dtype=torch.bfloat16)
    _lib.check(_lib.load().eelg_split_bf16x3(_lib.ptr(t), t.numel(), _lib.ptr(parts),
                                             _lib.stream(parts)), "split_bf16x3")
    return parts


def sum_rows(part: torch.Tensor, out: torch.Tensor = None, scale: float = 1.0) -> torch.Tensor:
    """``scale * part.sum(0)`` on the device in a fixed order (``eelg_sum_rows``): ``part`` is
    [rows, ...] with contiguous trailing dims, or a 2-D view whose rows are strided (a column
    block of a wider tensor: the bias gradient of one output slot).  ``out`` (contiguous,
    ``part.shape[1:]``) receives the sum when given."""
    _require_device(part)
    if part.dtype != torch.float32:
        raise TypeError(f"sum_rows: float32 expected, got {part.dtype}")
    rows = part.shape[0]
    if part.dim() == 2 and part.stride(1) == 1:
        ld, cols = part.stride(0), part.shape[1]
    else:
        part = part.contiguous()
        cols = math.prod(part.shape[1:])
        ld = cols
    if out is None:
        out = torch.empty(part.shape[1:], device=part.device, dtype=torch.float32)
    lib = _lib.load()
    nw = lib.eelg_sum_rows_work(rows, cols)
    work = torch.empty(nw, device=part.device, dtype=torch.float32) if nw else None
    _lib.check(lib.eelg_sum_rows(_lib.ptr(part), max(ld, cols), rows, cols, float(scale), _lib.ptr(out),
                                 _lib.ptr(work), nw, _lib.stream(out)), "sum_rows")
    return out


def _radial_desc(params, n_feat: int):
    n_hidden = (len(params) - 1) // 2
    hidden = params[0].shape[0]
    n_out = params[-1].shape[0]
    d = _lib.RadialDesc()
    d.n_feat, d.hidden, d.n_hidden, d.n_out = n_feat, hidden, n_hidden, n_out
    for i in range(n_hidden):
        d.w[i] = params[2 * i].data_ptr()
        d.b[i] = params[2 * i + 1].data_ptr()
    return d


def _radial_chunks(e: int, n_out: int, out_es: int, hidden: int, n_hidden: int):
    """Edge ranges under the radial kernels' 2 GiB per-stream limit (their buffer descriptors
    use 32-bit byte offsets): ``E * n_out * out_es`` for the [E, W] output / its gradient and
    ``E * hidden * n_hidden * 4`` for the saved pre-activations.  One range below the limit."""
    per_edge = max(n_out * out_es, hidden * n_hidden * 4, 1)
    cap = ((1 << 31) - 1) // per_edge // 128 * 128
    if cap <= 0:
        raise ValueError(f"radial MLP: one edge row ({per_edge} B) exceeds the 2 GiB stream limit")
    return [(a, min(a + cap, e)) for a in range(0, e, cap)] or [(0, 0)]


class _RadialMLP(torch.autograd.Function):
    """Linear(+bias)-SiLU-...-Linear(no bias) on edge features as one fused HIP kernel
    (``eelg_radial_fwd``: hidden layers on fp32 MFMA, the output layer fp32-accurate on bf16
    MFMA with split operands, hidden activations in LDS, only the pre-activations and the
    [E, W] output reach HBM), backward as three (``eelg_radial_bwd``).  No grad w.r.t.
    the features, which come from eelg_edge_embed without grad.  Edge sets past
    the kernels' 2 GiB per-stream limit run as several launches (``_radial_chunks``)."""

    @staticmethod
    def forward(ctx, feats, out_dtype, *params):
        _require_device(feats)
        feats = _f32(feats)
        params = tuple(_f32(p) for p in params)
        e, nf = feats.shape
        d = _radial_desc(params, nf)
        wo = params[-1]
        if wo.shape[1] != d.hidden or any(p.shape[0] != d.hidden for p in params[:-1]):
            raise ValueError("radial MLP: hidden widths differ between layers")
        # the kernels take the output width in whole 16-B pieces of bf16 (a multiple of 8, as every
        # generated TP weight count is); another width runs on zero-padded W_o rows
        n_out = d.n_out
        wp = -(-n_out // 8) * 8
        if wp != n_out:
            wo = torch.cat([wo, wo.new_zeros(wp - n_out, wo.shape[1])])
            d.n_out = wp
        out = torch.empty(e, wp, device=feats.device, dtype=out_dtype)
        wo_parts = split_bf16x3(wo)                  # [3, n_out, hidden]: the output layer's B operand
        lib = _lib.load()
        chunks = _radial_chunks(e, d.n_out, out.element_size(), d.hidden, d.n_hidden)
        zs = []
        for a, b in chunks:
            z = torch.empty(d.n_hidden, b - a, d.hidden, device=feats.device, dtype=torch.float32)
            _lib.check(lib.eelg_radial_fwd(_lib.ptr(feats[a:b]), b - a, ctypes.byref(d),
                                           _lib.ptr(wo_parts), int(out_dtype == torch.bfloat16),
                                           _lib.ptr(z), _lib.ptr(out[a:b]), _lib.stream(feats)),
                       "radial_fwd")
            zs.append(z)
        ctx.chunks = chunks
        ctx.save_for_backward(feats, *params, *zs)
        ctx.n_params = len(params)
        return out if wp == n_out else out[:, :n_out]

    @staticmethod
    def backward(ctx, g):
        feats, *rest = ctx.saved_tensors
        params, zs = rest[:ctx.n_params], rest[ctx.n_params:]
        e, nf = feats.shape
        d = _radial_desc(params, nf)
        n_out = d.n_out
        wp = -(-n_out // 8) * 8
        wo = params[-1]
        if wp != n_out:                                            # zero-padded width (forward)
            wo = torch.cat([wo, wo.new_zeros(wp - n_out, wo.shape[1])])
            g = torch.cat([g, g.new_zeros(g.shape[0], wp - n_out)], 1)
            d.n_out = wp
        g = g.contiguous()
        if g.data_ptr() % 16:
            g = g.clone()
        lib = _lib.load()
        wot_parts = split_bf16x3(wo.t().contiguous())             # [3, hidden, n_out]
        h = d.hidden
        if RADIAL_CHAIN and h == 64:
            return _RadialMLP._backward_chain(ctx, g, feats, params, zs, d, wot_parts, wp, n_out)
        n_small = h * nf + h + (d.n_hidden - 1) * (h * h + h)
        small, gwo = None, None
        for (a, b), z in zip(ctx.chunks, zs):
            ec = b - a
            npart, ns = ctypes.c_int(), ctypes.c_int()
            _lib.check(lib.eelg_radial_plan(ec, d.n_out, ctypes.byref(npart), ctypes.byref(ns)),
                       "radial_plan")
            part_h = torch.empty(npart.value, n_small, device=g.device, dtype=torch.float32)
            part_wo = torch.empty(ns.value, d.n_out, h, device=g.device, dtype=torch.float32)
            grad_h = torch.empty(ec, h, device=g.device, dtype=torch.float32)
            if ec == 0:
                part_h.zero_()
                part_wo.zero_()
            _lib.check(lib.eelg_radial_bwd(_lib.ptr(g[a:b]), int(g.dtype == torch.bfloat16), ec,
                                           ctypes.byref(d), _lib.ptr(wot_parts), _lib.ptr(z),
                                           _lib.ptr(feats[a:b]), _lib.ptr(grad_h), _lib.ptr(part_h),
                                           _lib.ptr(part_wo), _lib.stream(g)), "radial_bwd")
            sm, wo = sum_rows(part_h), sum_rows(part_wo)
            small = sm if small is None else small + sm
            gwo = wo if gwo is None else gwo + wo
        grads, off = [], 0
        for p in params[:-1]:
            grads.append(small[off: off + p.numel()].view_as(p))
            off += p.numel()
        grads.append(gwo if wp == n_out else gwo[:n_out].contiguous())
        return (None, None, *grads)

    @staticmethod
    def _backward_chain(ctx, g, feats, params, zs, d, wot_parts, wp, n_out):
        """``eelg_radial_bwd_chain``: the kernels leave gz_n and the hidden-layer inputs; the
        weight gradients gz_n^T h_n are long-K reductions on the linear weight-gradient kernel and
        the bias gradients column sums (``eelg_sum_rows``), all in a fixed order"""
        from . import dense
        lib = _lib.load()
        h, nh = d.hidden, d.n_hidden
        acc = [None] * (2 * nh)
        gwo = None
        for (a, b), z in zip(ctx.chunks, zs):
            ec = b - a
            npart, ns = ctypes.c_int(), ctypes.c_int()
            _lib.check(lib.eelg_radial_plan(ec, d.n_out, ctypes.byref(npart), ctypes.byref(ns)),
                       "radial_plan")
            part_wo = torch.empty(ns.value, d.n_out, h, device=g.device, dtype=torch.float32)
            grad_h = torch.empty(ec, h, device=g.device, dtype=torch.float32)
            gz = torch.empty(nh, ec, h, device=g.device, dtype=torch.float32)
            hin = torch.empty(max(nh - 1, 1), ec, h, device=g.device, dtype=torch.float32)
            if ec == 0:
                part_wo.zero_()
            _lib.check(lib.eelg_radial_bwd_chain(_lib.ptr(g[a:b]), int(g.dtype == torch.bfloat16), ec,
                                                 ctypes.byref(d), _lib.ptr(wot_parts), _lib.ptr(z),
                                                 _lib.ptr(grad_h), _lib.ptr(gz), _lib.ptr(hin),
                                                 _lib.ptr(part_wo), _lib.stream(g)), "radial_bwd_chain")
            for n in range(nh):
                x_n = feats[a:b] if n == 0 else hin[n - 1]
                gw = dense.linear_bwd_w(x_n, gz[n]) if ec else torch.zeros_like(params[2 * n])
                gb = sum_rows(gz[n]) if ec else torch.zeros_like(params[2 * n + 1])
                acc[2 * n] = gw if acc[2 * n] is None else acc[2 * n] + gw
                acc[2 * n + 1] = gb if acc[2 * n + 1] is None else acc[2 * n + 1] + gb
            wo = sum_rows(part_wo)
            gwo = wo if gwo is None else gwo + wo
        grads = [t.view_as(p) for t, p in zip(acc, params[:-1])]
        grads.append(gwo if wp == n_out else gwo[:n_out].contiguous())
        return (None, None, *grads)


def radial_mlp(feats: torch.Tensor, mlp: torch.nn.Sequential,
               out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """Apply ``mlp`` = [Linear(bias), SiLU]*k + [Linear(no bias)] with the fused backward.
    ``out_dtype`` bf16: the [E, W] output (the TP weights) is stored in bf16."""
    mods = list(mlp)
    params = []
    for i, mod in enumerate(mods):
        if isinstance(mod, torch.nn.Linear):
            last = i == len(mods) - 1
            if last != (mod.bias is None):
                raise ValueError("radial MLP: expected biases on hidden layers only")
            params.append(mod.weight)
            if not last:
                params.append(mod.bias)
        elif not isinstance(mod, torch.nn.SiLU):
            raise ValueError(f"radial MLP: unsupported module {type(mod).__name__}")
    tok = TIMER.start("radial_mlp_fwd")
    out = _RadialMLP.apply(_f32(feats), out_dtype, *params)
    TIMER.stop(tok)
    return out


# ---------------------------------------------------------------------------
# symmetric-contraction coefficients coef = (U_sym @ W)^T with a sparse U_sym
# ---------------------------------------------------------------------------
class SparseRows:
    """CSR of a fixed matrix and of its transpose (device int32 / fp32)."""

    def __init__(self, dense: torch.Tensor):
        d = dense.detach().to(torch.float64).cpu()
        self.shape = tuple(d.shape)
        for name, m in (("a", d), ("t", d.t())):
            nz = m != 0
            rowptr = torch.zeros(m.shape[0] + 1, dtype=torch.int32)
            rowptr[1:] = torch.cumsum(nz.sum(1), 0).to(torch.int32)
            r, c = torch.nonzero(nz, as_tuple=True)
            setattr(self, name, (rowptr, c.to(torch.int32), m[r, c].to(torch.float32)))
        self._dev = {}

    def on(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = tuple(tuple(t.to(device) for t in trip) for trip in (self.a, self.t))
        return self._dev[key]


def _spmm(trip, n_rows, B, ldb_r, ldb_c, n_cols, out, ldo_r, ldo_c):
    rp, col, val = trip
    _lib.check(_lib.load().eelg_csr_spmm(_lib.ptr(rp), _lib.ptr(col), _lib.ptr(val), n_rows,
                                         _lib.ptr(B), ldb_r, ldb_c, n_cols, _lib.ptr(out), ldo_r,
                                         ldo_c, _lib.stream(out)), "csr_spmm")


class _SymConCoef(torch.autograd.Function):
    """coef[c, t] = sum_k U[t, k] W[k, c]  ([mul, ld], the layout the sc kernels read: rows
    padded to ``ld`` >= nterms, the padding zero)."""

    @staticmethod
    def forward(ctx, w, sp: SparseRows, ld: int):
        _require_device(w)
        w = _f32(w)
        nt, nk = sp.shape
        mul = w.shape[1]
        a, t = sp.on(w.device)
        coef = torch.empty(mul, ld, device=w.device, dtype=torch.float32)
        if ld != nt:
            coef[:, nt:].zero_()
        _spmm(a, nt, w, mul, 1, mul, coef, 1, ld)                 # out[t, c] at c*ld + t
        ctx.sp, ctx.mul = sp, mul
        return coef

    @staticmethod
    def backward(ctx, g):
        g = _f32(g)
        sp, mul = ctx.sp, ctx.mul
        nt, nk = sp.shape
        a, t = sp.on(g.device)
        gt = g.t().contiguous()                                   # [ld, mul]: coalesced over c
        gw = torch.empty(nk, mul, device=g.device, dtype=torch.float32)
        _spmm(t, nk, gt, mul, 1, mul, gw, mul, 1)                 # reads rows t < nterms only
        return gw, None, None


def symcon_coefficients(w: torch.Tensor, sp: SparseRows, ld: Optional[int] = None) -> torch.Tensor:
    """[mul, ld] coefficients (``ld``: the contraction config's ``coef_ld``; default nterms)."""
    return _SymConCoef.apply(w, sp, sp.shape[0] if ld is None else ld)
