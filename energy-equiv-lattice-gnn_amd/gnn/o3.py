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

import math
from collections import Counter
from typing import List, Tuple

import torch

from . import cg
from .irreps import Irreps


class Linear(torch.nn.Module):
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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n = x.shape[0]
        parts = [None] * len(self.irreps_out)
        w_off = 0
        for (i, o), a in zip(self.instructions, self.alpha):
            mi, ir = self.irreps_in[i]
            mo = self.irreps_out[o].mul
            w = self.weight[w_off: w_off + mi * mo].view(mi, mo)
            w_off += mi * mo
            xi = x[:, self._in_off[i]: self._in_off[i] + mi * ir.dim].view(n, mi, ir.dim)
            y = torch.matmul(xi.transpose(1, 2), w * a).transpose(1, 2)   # [n, mo, d]
            parts[o] = y if parts[o] is None else parts[o] + y
        out, b_off = [], 0
        for o, (mo, ir) in enumerate(self.irreps_out):
            y = parts[o]
            if y is None:
                y = x.new_zeros(n, mo, ir.dim)
            if o in self.bias_slots:
                y = y + self.bias[b_off: b_off + mo].view(1, mo, 1)
                b_off += mo
            out.append(y.reshape(n, mo * ir.dim))
        return torch.cat(out, dim=1)


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

    def forward(self, x):
        ns, ng = self.irreps_scalars.dim, self.irreps_gates.dim
        act = torch.nn.functional.silu
        scalars = self.cst * act(x[:, :ns])
        gates = self.cst * act(x[:, ns: ns + ng])
        out, g_off, x_off = [scalars], 0, ns + ng
        for mul, ir in self.irreps_gated:
            blk = x[:, x_off: x_off + mul * ir.dim].view(-1, mul, ir.dim)
            out.append((blk * gates[:, g_off: g_off + mul, None]).reshape(-1, mul * ir.dim))
            g_off += mul
            x_off += mul * ir.dim
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
