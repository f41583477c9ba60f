"""Device-side equivalents of the e3nn modules the hot path uses.

* ``Linear``  -- ``o3.Linear`` (path normalisation 'element', 0e biases zero-init),
  parameter ``weight`` flat in e3nn instruction order (i_in major, i_out minor),
  so ``state_dict`` keys/shapes match the reference (``gnn/blocks.py:516-521``).
  Channel mixing is a per-irrep GEMM on the mul axis.
* ``Gate``    -- ``nn.Gate`` with normalize2mom(SiLU) (``gnn/blocks.py:268-274``).
* ``TensorProduct`` -- holds the 'uvu' instruction table of ``o3.TensorProduct``
  (``gnn/blocks.py:528-535``); its arithmetic is the fused HIP interaction.
"""
from __future__ import annotations

import ctypes
import math
import os
from collections import Counter
from typing import List, Tuple

import torch

from . import cg
from .irreps import Irreps

# grad-W launch shape: target workgroups and a cap on the node slices (partials)
# r04ac kbench: 1024 / 64 -> 4096 / 128 takes grad-W 7360 -> 800 from 0.324 to 0.264 ms and
# 800 -> 800 from 0.056 to 0.049 ms (a grid of about one round left the D = 9 tiles, 9x the
# bytes per node of D = 1, as the tail); the step is unchanged (these run on a side stream)
LINW_WG = int(os.environ.get("EELG_LINW_WG", "4096"))
LINW_MAX_SLICES = int(os.environ.get("EELG_LINW_MAX_SLICES", "128"))
# forward / grad-x of the eligible linears on bf16 MFMA with fp32-accurate split operands (1),
# or on the fp32 MFMA kernels (0).  Only descriptors whose every slot sums K >= LIN_X6_MINK take
# it: r04b kbench, 7360->800 fwd (K 160..320) 0.261 vs 0.290 ms fp32; K = 32 (the 800->800
# linears, every grad-x of the 7360->800) 0.056-0.391 vs 0.050-0.325 ms -- one 32-wide chunk per
# group leaves the split and LDS B-fragment reads unamortised
LIN_X6 = os.environ.get("EELG_LIN_X6", "1") != "0"
LIN_X6_MINK = int(os.environ.get("EELG_LIN_X6_MINK", "128"))
# the readout Gate as fused HIP passes (1) or torch elementwise ops (0)
GATE_FUSED = os.environ.get("EELG_GATE_FUSED", "1") != "0"


def _output_mask(irreps_out, covered) -> torch.Tensor:
    """e3nn 0.5 ``output_mask``: 1 on the output irreps some instruction writes, else 0."""
    if not irreps_out.dim:
        return torch.ones(0)
    return torch.cat([torch.full((mul * ir.dim,), 1.0 if o in covered else 0.0)
                      for o, (mul, ir) in enumerate(irreps_out)])


def _accept_output_mask(state_dict, key: str, irreps_out, covered, error_msgs) -> None:
    """e3nn's ``Linear`` / ``TensorProduct`` register an ``output_mask`` buffer (1 on the output
    irreps some instruction writes).  Reference checkpoints may carry it: it is derived data,
    so it is accepted and checked against this module's instructions, not stored."""
    m = state_dict.pop(key, None)
    if m is None:
        return
    want = _output_mask(irreps_out, covered)
    if tuple(m.shape) != tuple(want.shape) or not torch.equal(m.detach().cpu().float() != 0, want != 0):
        error_msgs.append(f"{key}: output mask does not match the module's instructions")


def _accept_empty(state_dict, key: str, error_msgs) -> None:
    """e3nn registers ``torch.Tensor()`` placeholders (``register_buffer('weight' | 'bias',
    torch.Tensor())``) where a module has no internal weight / bias: a ``TensorProduct`` with
    external weights, a bias-less ``Linear``, the Gate's ``ElementwiseTensorProduct``.  They
    are accepted when empty; anything else would be a weight this module does not have."""
    t = state_dict.pop(key, None)
    if t is not None and t.numel() != 0:
        error_msgs.append(f"{key}: expected e3nn's empty placeholder buffer, got shape "
                          f"{tuple(t.shape)}")


def _emit_e3nn_buffers(state_dict, prefix: str, entries) -> None:
    """``state_dict()`` carries e3nn's derived buffers (output masks, empty placeholders) under
    the reference's names, so a checkpoint of this model loads strictly into the reference."""
    for name, t in entries:
        state_dict[prefix + name] = t


class _OnStream(torch.autograd.Function):
    """Identity (a view) applied while ``stream`` is current, so that autograd runs its
    backward -- and the gradient accumulation of the parameter behind it -- on ``stream``."""

    @staticmethod
    def forward(ctx, t, stream):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return g, None


class GradMailbox:
    """Hands the layer residual's gradient from the linear that adds the residual (forward
    ``residual=h``) to the linear that reads ``h`` first (``linear_up``), whose grad-x kernel
    adds it in its epilogue: autograd would otherwise sum the two gradient contributions of
    ``h`` in a separate pass over [N, 800].  Backward order is fixed by the data flow (the
    residual's linear is downstream of ``linear_up``), so the deposit precedes the collection."""

    def __init__(self):
        self.grad = None


class _IrrepsLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, lin: "Linear", side=None, residual=None, mailbox=None):
        ctx.save_for_backward(x, weight)
        ctx.lin, ctx.side, ctx.mailbox = lin, side, mailbox
        ctx.deposit = residual is not None
        return lin._fwd(x, weight, bias, residual)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        lin, side, mb = ctx.lin, ctx.side, ctx.mailbox
        gy = gy.contiguous()
        gres = gy if ctx.needs_input_grad[5] else None      # y = linear(x) + residual
        if gres is not None and mb is not None:
            mb.grad, gres = gres, None                      # added by the collecting linear
        extra = None
        if mb is not None and not ctx.deposit:
            extra, mb.grad = mb.grad, None
        gx = lin._bwd_x(gy, weight, extra) if ctx.needs_input_grad[0] else None
        want_w, want_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        if side is None or not (want_w or want_b):
            gw = lin._bwd_w(x, gy) if want_w else None
            gb = lin._bwd_bias(gy) if want_b else None
            return gx, gw, gb, None, None, gres, None
        # weight / bias gradients on the side stream the parameters' views were made on:
        # their consumers (the views' backward, the accumulation) run there as well, and
        # the main stream carries on with grad-x
        side.wait_stream(torch.cuda.current_stream(x.device))
        x.record_stream(side)
        gy.record_stream(side)
        with torch.cuda.stream(side):
            gw = lin._bwd_w(x, gy) if want_w else None
            gb = lin._bwd_bias(gy) if want_b else None
        return gx, gw, gb, None, None, gres, None


class Linear(torch.nn.Module):
    """e3nn ``o3.Linear`` on mul-major rows; HIP kernels (``eelg_linear_*``): forward and grad-x
    on bf16 MFMA with fp32-accurate split operands where the irreps qualify
    (``eelg_linear_fwd_pk``), fp32 MFMA otherwise and for grad-W."""

    def __init__(self, irreps_in, irreps_out, internal_weights: bool = True,
                 shared_weights: bool = True, biases: bool = False):
        super().__init__()
        self.irreps_in, self.irreps_out = Irreps(irreps_in), Irreps(irreps_out)
        self.instructions: List[Tuple[int, int]] = [
            (i, o) for i, (_, a) in enumerate(self.irreps_in)
            for o, (_, b) in enumerate(self.irreps_out) if a == b]
        fan = Counter()
        for i, o in self.instructions:
            fan[o] += self.irreps_in[i].mul
        self.alpha = [1.0 / math.sqrt(fan[o]) for _, o in self.instructions]
        self.weight_numel = sum(self.irreps_in[i].mul * self.irreps_out[o].mul
                                for i, o in self.instructions)
        self.weight = torch.nn.Parameter(torch.randn(self.weight_numel))
        self.bias_slots = [o for o, (_, ir) in enumerate(self.irreps_out)
                           if biases and ir.l == 0 and ir.p == 1]
        nb = sum(self.irreps_out[o].mul for o in self.bias_slots)
        if nb:
            self.bias = torch.nn.Parameter(torch.zeros(nb))
        else:
            self.register_parameter("bias", None)
        self._in_off, self._out_off = self.irreps_in.offsets(), self.irreps_out.offsets()
        self._build_descriptors()
        self._register_state_dict_hook(Linear._emit_derived)

    def _covered(self):
        # e3nn 0.5 masks by the weight instructions only (not the bias instructions)
        return {o for _, o in self.instructions}

    @staticmethod
    def _emit_derived(module, state_dict, prefix, local_metadata):
        ents = [("output_mask", _output_mask(module.irreps_out, module._covered()))]
        if module.bias is None:
            ents.append(("bias", torch.Tensor()))
        _emit_e3nn_buffers(state_dict, prefix, ents)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        _accept_output_mask(state_dict, prefix + "output_mask", self.irreps_out,
                            self._covered(), error_msgs)
        if self.bias is None:
            _accept_empty(state_dict, prefix + "bias", error_msgs)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)
        self.invalidate_packed()

    def invalidate_packed(self) -> None:
        """forget the packed split weights (after a write the version counter does not see)"""
        if hasattr(self, "_pk_cache"):
            self._pk_cache.clear()

    # -- descriptor tables for the C ABI (built once) ---------------------------
    def _build_descriptors(self):
        from . import _lib
        w_offs, off = [], 0
        for i, o in self.instructions:
            w_offs.append(off)
            off += self.irreps_in[i].mul * self.irreps_out[o].mul
        self._w_offs = w_offs
        b_offs, boff = {}, 0
        for o in self.bias_slots:
            b_offs[o] = boff
            boff += self.irreps_out[o].mul
        self._b_offs = b_offs

        def slots(n_slots, dims, muls, offs, srcs, bias):
            if n_slots > _lib.LIN_MAXSLOT:
                raise NotImplementedError("too many irreps slots for eelg_linear")
            desc = _lib.LinDesc()
            desc.n_slots = n_slots
            desc.max_jt = max((m + 31) // 32 for m in muls)
            self_max_d = max(dims)
            for s in range(n_slots):
                sl = desc.slot[s]
                sl.y_off, sl.n_out, sl.d = offs[s], muls[s], dims[s]
                sl.bias_off = bias.get(s, -1)
                if len(srcs[s]) > _lib.LIN_MAXSRC:
                    raise NotImplementedError("too many sources for one irreps slot")
                sl.n_src = len(srcs[s])
                for t, (xo, k, wo, ldk, ldj, a) in enumerate(srcs[s]):
                    sl.src[t].x_off, sl.src[t].k, sl.src[t].w_off = xo, k, wo
                    sl.src[t].ldk, sl.src[t].ldj, sl.src[t].alpha = ldk, ldj, a
            return desc, self_max_d

        out_srcs = [[] for _ in self.irreps_out]
        in_srcs = [[] for _ in self.irreps_in]
        for (i, o), wo, a in zip(self.instructions, w_offs, self.alpha):
            mi, mo = self.irreps_in[i].mul, self.irreps_out[o].mul
            out_srcs[o].append((self._in_off[i], mi, wo, mo, 1, a))
            in_srcs[i].append((self._out_off[o], mo, wo, 1, mo, a))
        self._fwd_desc, self._fwd_maxd = slots(
            len(self.irreps_out), [ir.dim for _, ir in self.irreps_out],
            [m for m, _ in self.irreps_out], self._out_off, out_srcs, b_offs)
        self._bx_desc, self._bx_maxd = slots(
            len(self.irreps_in), [ir.dim for _, ir in self.irreps_in],
            [m for m, _ in self.irreps_in], self._in_off, in_srcs, {})
        if len(self.instructions) > _lib.LINW_MAXINS:
            raise NotImplementedError("too many instructions for eelg_linear_bwd_w")
        wd = _lib.LinWDesc()
        wd.n_ins = len(self.instructions)
        wd.max_jt = max([(self.irreps_out[o].mul + 31) // 32 for _, o in self.instructions] or [1])
        wd.max_ut = max([(self.irreps_in[i].mul + 31) // 32 for i, _ in self.instructions] or [1])
        for t, ((i, o), wo, a) in enumerate(zip(self.instructions, w_offs, self.alpha)):
            e = wd.ins[t]
            e.x_off, e.k, e.g_off = self._in_off[i], self.irreps_in[i].mul, self._out_off[o]
            e.n_out, e.d, e.w_off, e.alpha = self.irreps_out[o].mul, self.irreps_in[i].ir.dim, wo, a
        self._bw_desc = wd
        self._pk_ok = {"fwd": self._packable(self._fwd_desc), "bx": self._packable(self._bx_desc)}
        self._pk_cache = {}
        self._bw_maxd = max([self.irreps_in[i].ir.dim for i, _ in self.instructions] or [1])
        self._bw_tiles = sum(((self.irreps_in[i].mul + 31) // 32) * ((self.irreps_out[o].mul + 31) // 32)
                             for i, o in self.instructions) or 1

    @staticmethod
    def _packable(desc) -> bool:
        """the descriptor qualifies for eelg_linear_fwd_pk (whole 32-wide K chunks and column
        tiles, d odd <= 9, 16-B aligned slot offsets; the row alignment is checked per call)"""
        for s in range(desc.n_slots):
            sl = desc.slot[s]
            if sl.n_src == 0 or sl.n_out % 32 or sl.y_off % 4 or sl.d not in (1, 3, 5, 7, 9):
                return False
            if sl.bias_off >= 0 and sl.d != 1:
                return False
            ks = sum(sl.src[t].k for t in range(sl.n_src))
            if ks > 320 or ks < LIN_X6_MINK:
                return False
            for t in range(sl.n_src):
                if sl.src[t].k % 32 or sl.src[t].x_off % 4:
                    return False
        return True

    def _packed(self, which: str, weight):
        """split, alpha-scaled weights of descriptor ``which`` ('fwd' or 'bx') for the packed
        kernel, rebuilt when the weight changes (cached per weight version).  A write through
        ``weight.data`` does not bump the version counter: such writers call
        ``invalidate_packed()`` (``parallel.broadcast_parameters`` and ``load_state_dict`` do)."""
        from . import _lib
        key = (weight.data_ptr(), weight._version, weight.device)
        hit = self._pk_cache.get(which)
        if hit is not None and hit[0] == key:
            return hit[1]
        desc = self._fwd_desc if which == "fwd" else self._bx_desc
        n = int(_lib.load().eelg_linear_pack_size(ctypes.byref(desc)))
        pk = torch.empty(3, n, device=weight.device, dtype=torch.bfloat16)
        _lib.check(_lib.load().eelg_linear_pack(_lib.ptr(weight), ctypes.byref(desc), _lib.ptr(pk),
                                                _lib.stream(pk)), "linear_pack")
        self._pk_cache[which] = (key, pk)
        return pk

    def _run_pk(self, which, x, x_row, weight, bias, extra, n, out, out_row, desc) -> bool:
        """the packed launch when eligible; False leaves the call to the fp32 kernels"""
        from . import _lib
        if not (LIN_X6 and self._pk_ok[which] and x_row % 4 == 0 and out_row % 4 == 0
                and x.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
                and (extra is None or extra.data_ptr() % 16 == 0)):
            return False
        pk = self._packed(which, weight.detach())
        _lib.check(_lib.load().eelg_linear_fwd_pk(
            _lib.ptr(x), x_row, _lib.ptr(pk), _lib.ptr(bias), _lib.ptr(extra), n, _lib.ptr(out),
            out_row, ctypes.byref(desc), _lib.stream(out)), "linear_fwd_pk")
        return True

    # -- launches ---------------------------------------------------------------
    def _fwd(self, x, weight, bias, residual=None):
        from . import _lib
        n = x.shape[0]
        y = torch.empty(n, self.irreps_out.dim, device=x.device, dtype=torch.float32)
        self._fwd_desc.max_rows = n * self._fwd_maxd
        if residual is not None and (residual.shape != y.shape or residual.dtype != torch.float32
                                     or not residual.is_contiguous()):
            raise ValueError(f"residual {tuple(residual.shape)} {residual.dtype}: expected a "
                             f"contiguous float32 {tuple(y.shape)}")
        if self._run_pk("fwd", x, self.irreps_in.dim, weight, bias, residual, n, y,
                        self.irreps_out.dim, self._fwd_desc):
            return y
        _lib.check(_lib.load().eelg_linear_fwd_res(
            _lib.ptr(x), self.irreps_in.dim, _lib.ptr(weight), _lib.ptr(bias), _lib.ptr(residual), n,
            _lib.ptr(y), self.irreps_out.dim, ctypes.byref(self._fwd_desc), _lib.stream(y)),
            "linear_fwd")
        return y

    def _bwd_x(self, gy, weight, extra=None):
        """grad-x; ``extra`` ([N, dim_in], e.g. a residual's gradient) is added in the epilogue"""
        from . import _lib
        n = gy.shape[0]
        gx = torch.empty(n, self.irreps_in.dim, device=gy.device, dtype=torch.float32)
        self._bx_desc.max_rows = n * self._bx_maxd
        if extra is not None:
            extra = extra.contiguous()
            if extra.shape != gx.shape or extra.dtype != torch.float32:
                raise ValueError(f"linear grad-x: added gradient {tuple(extra.shape)} does not "
                                 f"match {tuple(gx.shape)}")
        if self._run_pk("bx", gy, self.irreps_out.dim, weight, None, extra, n, gx,
                        self.irreps_in.dim, self._bx_desc):
            return gx
        _lib.check(_lib.load().eelg_linear_fwd_res(
            _lib.ptr(gy), self.irreps_out.dim, _lib.ptr(weight), None, _lib.ptr(extra), n,
            _lib.ptr(gx), self.irreps_in.dim, ctypes.byref(self._bx_desc), _lib.stream(gx)),
            "linear_bwd_x")
        return gx

    def _bwd_w(self, x, gy):
        from . import _lib, ops
        n = x.shape[0]
        if not self.instructions:
            return torch.zeros_like(self.weight)
        # ~LINW_WG workgroups in total: (node slices) x (32x32 weight tiles of all
        # instructions); each slice leaves one partial weight gradient that the sum reads back
        slices = max(1, min((n + 31) // 32, -(-LINW_WG // self._bw_tiles), LINW_MAX_SLICES))
        nps = -(-n // slices)
        slices = -(-n // nps)
        self._bw_desc.max_rows = n * self._bw_maxd
        part = torch.empty(slices, self.weight_numel, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().eelg_linear_bwd_w(
            _lib.ptr(x), self.irreps_in.dim, _lib.ptr(gy), self.irreps_out.dim, n, nps,
            _lib.ptr(part), slices, self.weight_numel, ctypes.byref(self._bw_desc), _lib.stream(part)),
            "linear_bwd_w")
        return ops.sum_rows(part)

    def _bwd_bias(self, gy):
        from . import ops
        out = torch.empty(sum(self.irreps_out[o].mul for o in self.bias_slots), device=gy.device,
                          dtype=torch.float32)
        k = 0
        for o in self.bias_slots:
            m = self.irreps_out[o].mul
            ops.sum_rows(gy[:, self._out_off[o]: self._out_off[o] + m], out=out[k: k + m])
            k += m
        return out

    def forward(self, x: torch.Tensor, residual: torch.Tensor = None,
                grad_mailbox: "GradMailbox" = None) -> torch.Tensor:
        """``o3.Linear``; with ``residual`` returns ``linear(x) + residual`` with the add in the
        kernel epilogue (the layer residual of ``gnn/model.py:92-96``).  ``grad_mailbox``
        shared by the residual-adding linear and the first linear reading the residual moves
        the residual's gradient into that linear's grad-x epilogue (``GradMailbox``)."""
        from .ops import _f32, _require_device
        _require_device(x)
        if x.shape[-1] != self.irreps_in.dim:
            raise ValueError(f"Linear expects [..., {self.irreps_in.dim}], got {tuple(x.shape)}")
        from . import ops
        weight, bias = self.weight, self.bias
        side = None
        if ops.OVERLAP and x.is_cuda and torch.is_grad_enabled() and weight.requires_grad:
            side = ops.side_stream(x.device, 2)
            with torch.cuda.stream(side):
                weight = _OnStream.apply(weight, side)
                if bias is not None:
                    bias = _OnStream.apply(bias, side)
        if residual is not None:
            _require_device(residual)
            residual = _f32(residual)
        return _IrrepsLinearFn.apply(_f32(x), weight, bias, self, side, residual, grad_mailbox)


class _GateFn(torch.autograd.Function):
    """e3nn ``nn.Gate`` as two fused HIP passes (``eelg_gate_fwd`` / ``eelg_gate_bwd``)."""

    @staticmethod
    def forward(ctx, x, gate: "Gate"):
        from . import _lib
        y = torch.empty(x.shape[0], gate.irreps_out.dim, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().eelg_gate_fwd(_lib.ptr(x), x.shape[0], ctypes.byref(gate._desc()),
                                             float(gate.cst), _lib.ptr(y), _lib.stream(y)), "gate_fwd")
        ctx.save_for_backward(x)
        ctx.gate = gate
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import _lib
        (x,) = ctx.saved_tensors
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        _lib.check(_lib.load().eelg_gate_bwd(_lib.ptr(x), _lib.ptr(gy), x.shape[0],
                                             ctypes.byref(ctx.gate._desc()), float(ctx.gate.cst),
                                             _lib.ptr(gx), _lib.stream(gx)), "gate_bwd")
        return gx, None


class Gate(torch.nn.Module):
    def __init__(self, irreps_scalars, irreps_gates, irreps_gated):
        super().__init__()
        self.irreps_scalars = Irreps(irreps_scalars)
        self.irreps_gates = Irreps(irreps_gates)
        self.irreps_gated = Irreps(irreps_gated)
        assert self.irreps_gates.num_irreps == self.irreps_gated.num_irreps
        self.irreps_in = self.irreps_scalars + self.irreps_gates + self.irreps_gated
        self.irreps_out = self.irreps_scalars + self.irreps_gated
        self.cst = cg.silu_normalize2mom()
        self._register_state_dict_hook(Gate._emit_derived)

    # e3nn's Gate multiplies with an ElementwiseTensorProduct submodule ``mul`` (external
    # weights: an empty ``weight`` placeholder, and an output mask over the gated irreps)
    @staticmethod
    def _emit_derived(module, state_dict, prefix, local_metadata):
        g = module.irreps_gated
        _emit_e3nn_buffers(state_dict, prefix, [
            ("mul.weight", torch.Tensor()),
            ("mul.output_mask", _output_mask(g, set(range(len(g)))))])

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        _accept_output_mask(state_dict, prefix + "mul.output_mask", self.irreps_gated,
                            set(range(len(self.irreps_gated))), error_msgs)
        _accept_empty(state_dict, prefix + "mul.weight", error_msgs)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def _desc(self):
        from . import _lib
        if getattr(self, "_gdesc", None) is None:
            d = _lib.GateDesc()
            d.n_scal, d.n_gates, d.n_blk = self.irreps_scalars.dim, self.irreps_gates.dim, len(self.irreps_gated)
            for b, (mul, ir) in enumerate(self.irreps_gated):
                d.blk_mul[b], d.blk_dim[b] = mul, ir.dim
            self._gdesc = d
        return self._gdesc

    def _fits_kernel(self) -> bool:
        from . import _lib
        return (len(self.irreps_gated) <= _lib.GATE_MAXBLK and self.irreps_gated.dim <= _lib.GATE_MAXGATED
                and self.irreps_gates.dim <= _lib.GATE_MAXGATES)

    def forward(self, x):
        # the fused HIP passes cover gates up to the kernels' table sizes; wider readouts use
        # the torch form below (the readout tail is outside the HIP hot path)
        if x.is_cuda and x.dtype == torch.float32 and GATE_FUSED and self._fits_kernel():
            from .ops import _f32
            return _GateFn.apply(_f32(x), self)
        # one torch.split instead of per-block slices: its backward is a single cat, where
        # slice backwards would each zero-fill a full [n, dim_in] gradient and add it up
        # (six zero-fill + add pairs per gate; the values are identical either way)
        gated = [mul * ir.dim for mul, ir in self.irreps_gated]
        pieces = torch.split(x, [self.irreps_scalars.dim, self.irreps_gates.dim] + gated, dim=1)
        act = torch.nn.functional.silu
        scalars = self.cst * act(pieces[0])
        gates = torch.split(self.cst * act(pieces[1]), [mul for mul, _ in self.irreps_gated], dim=1)
        out = [scalars]
        for (mul, ir), blk, g in zip(self.irreps_gated, pieces[2:], gates):
            out.append((blk.reshape(-1, mul, ir.dim) * g[:, :, None]).reshape(-1, mul * ir.dim))
        return torch.cat(out, dim=1)


class TensorProduct(torch.nn.Module):
    """Instruction table of the 'uvu' ``o3.TensorProduct`` (no parameters)."""

    def __init__(self, irreps_in1, irreps_in2, irreps_out, instructions):
        super().__init__()
        self.irreps_in1, self.irreps_in2 = Irreps(irreps_in1), Irreps(irreps_in2)
        self.irreps_out = Irreps(irreps_out)
        self.instructions = list(instructions)
        self.weight_numel = sum(self.irreps_in1[i1].mul * self.irreps_in2[i2].mul
                                for i1, i2, *_ in self.instructions)
        self._register_state_dict_hook(TensorProduct._emit_derived)

    # external (per-edge) weights: e3nn holds an empty ``weight`` placeholder buffer
    @staticmethod
    def _emit_derived(module, state_dict, prefix, local_metadata):
        _emit_e3nn_buffers(state_dict, prefix, [
            ("weight", torch.Tensor()),
            ("output_mask", _output_mask(module.irreps_out, {ins[2] for ins in module.instructions}))])

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        _accept_output_mask(state_dict, prefix + "output_mask", self.irreps_out,
                            {ins[2] for ins in self.instructions}, error_msgs)
        _accept_empty(state_dict, prefix + "weight", error_msgs)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)
