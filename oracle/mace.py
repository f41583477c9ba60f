"""Restatement of the MACE-derived helpers in ``gnn/mace.py``.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Each function cites the reference lines it follows.  The symmetric
contraction keeps the reference's dense formulation and contraction order
(opt_einsum 3.3.0 picks U.W first for these shapes),
so that the CPU baseline has the reference's cost structure.
"""
from __future__ import annotations

import collections
import functools
from typing import List, Tuple

import torch

from .o3 import Irrep, Irreps, wigner_3j

_TP = collections.namedtuple("_TP", "op, args")
_INPUT = collections.namedtuple("_INPUT", "tensor, start, stop")


def tp_out_irreps_with_instructions(irreps1, irreps2, target_irreps) -> Tuple[Irreps, List]:
    """``gnn/mace.py:286-314``."""
    irreps1, irreps2, target_irreps = Irreps(irreps1), Irreps(irreps2), Irreps(target_irreps)
    out_list, instructions = [], []
    for i, (mul, ir_in) in enumerate(irreps1):
        for j, (_, ir_edge) in enumerate(irreps2):
            for ir_out in ir_in * ir_edge:
                if ir_out in target_irreps:
                    k = len(out_list)
                    out_list.append((mul, ir_out))
                    instructions.append((i, j, k, "uvu", True))
    irreps_out, permut, _ = Irreps(out_list).sort()
    instructions = [(a, b, permut[k], m, t) for a, b, k, m, t in instructions]
    instructions = sorted(instructions, key=lambda x: x[2])
    return irreps_out, instructions


def reshape_irreps(irreps, tensor: torch.Tensor) -> torch.Tensor:
    """``gnn/mace.py:316-332``: [N, mul-major irreps] -> [N, mul, sum(2l+1)]."""
    ix, out = 0, []
    b = tensor.shape[0]
    for mul, ir in Irreps(irreps):
        d = ir.dim
        out.append(tensor[:, ix: ix + mul * d].reshape(b, mul, d))
        ix += mul * d
    return torch.cat(out, dim=-1)


def get_edge_vectors_and_lengths(positions, edge_index, shifts, normalize=False, eps=1e-9):
    """``gnn/mace.py:338-352`` (``normalize`` divides by ``length + eps``)."""
    sender, receiver = edge_index
    vectors = positions[receiver] - positions[sender] + shifts
    lengths = torch.linalg.norm(vectors, dim=-1, keepdim=True)
    if normalize:
        return vectors / (lengths + eps), lengths
    return vectors, lengths


# ``filter_ir_mid`` of U_matrix_real for correlation 4 (gnn/mace.py:444-458): natural parity, l <= 11
_FILTER_MID_C4 = tuple((l, 1 if l % 2 == 0 else -1) for l in range(12))


def _wigner_nj(irrepss, dtype=torch.float64, filter_ir_mid=None):
    """``gnn/mace.py:363-432`` (normalization='component')."""
    irrepss = [Irreps(x) for x in irrepss]
    names = {str(x) for x in irrepss}
    if len(names) == 1 and dtype == torch.float64:
        # n copies of one irreps (every U_matrix_real call): memoised per process, the
        # result is shared by every output irrep and contraction of that coupling
        return list(_wigner_nj_same(names.pop(), len(irrepss), filter_ir_mid))
    return _wigner_nj_impl(irrepss, dtype, filter_ir_mid)


@functools.lru_cache(maxsize=None)
def _wigner_nj_same(irreps: str, n: int, filter_ir_mid=None):
    return tuple(_wigner_nj_impl([Irreps(irreps)] * n, torch.float64, filter_ir_mid))


def _wigner_nj_impl(irrepss, dtype, filter_ir_mid=None):
    if len(irrepss) == 1:
        (irreps,) = irrepss
        ret, e, i = [], torch.eye(irreps.dim, dtype=dtype), 0
        for mul, ir in irreps:
            for _ in range(mul):
                sl = slice(i, i + ir.dim)
                ret.append((ir, _INPUT(0, sl.start, sl.stop), e[sl]))
                i += ir.dim
        return ret
    *left, right = irrepss
    ret = []
    for ir_left, path_left, c_left in _wigner_nj(left, dtype, filter_ir_mid):
        i = 0
        for mul, ir in right:
            for ir_out in ir_left * ir:
                if filter_ir_mid is not None and (ir_out.l, ir_out.p) not in filter_ir_mid:
                    continue
                c = wigner_3j(ir_out.l, ir_left.l, ir.l, dtype=dtype) * ir_out.dim ** 0.5
                c = torch.einsum("jk,ijl->ikl", c_left.flatten(1), c)
                c = c.reshape(ir_out.dim, *(x.dim for x in left), ir.dim)
                for u in range(mul):
                    e = torch.zeros(ir_out.dim, *(x.dim for x in left), right.dim, dtype=dtype)
                    sl = slice(i + u * ir.dim, i + (u + 1) * ir.dim)
                    e[..., sl] = c
                    ret.append((ir_out, _TP(op=(ir_left, ir, ir_out),
                                            args=(path_left, _INPUT(len(left), sl.start, sl.stop))), e))
            i += mul * ir.dim
    # stable sort by irrep
    return sorted(ret, key=lambda x: x[0]._key())


def U_matrix_real(irreps_in, irreps_out, correlation: int, dtype=torch.float64):
    """``gnn/mace.py:435-477`` (correlation 4 couples through ``filter_ir_mid``, :444-458)."""
    ir, u = _U_matrix_real_cached(str(Irreps(irreps_in)), str(Irreps(irreps_out)), correlation)
    return [ir, u.to(dtype).clone()]


@functools.lru_cache(maxsize=None)
def _U_matrix_real_cached(irreps_in: str, irreps_out: str, correlation: int):
    dtype = torch.float64
    irreps_out = Irreps(irreps_out)
    filt = _FILTER_MID_C4 if correlation == 4 else None
    wigners = _wigner_nj([Irreps(irreps_in)] * correlation, dtype, filt)
    current_ir = wigners[0][0]
    out, stack, last_ir = [], None, None
    for ir, _, base in wigners:
        if ir in irreps_out and ir == current_ir:
            b = base.squeeze().unsqueeze(-1)
            stack = b if stack is None else torch.cat((stack, b), dim=-1)
            last_ir = current_ir
        elif ir in irreps_out and ir != current_ir:
            if stack is not None:
                out += [last_ir, stack]
            stack = base.squeeze().unsqueeze(-1)
            current_ir, last_ir = ir, ir
        else:
            current_ir = ir
    return last_ir, stack


class Contraction(torch.nn.Module):
    """``gnn/mace.py:180-280``, non-element-dependent branch (``:225-240,261-275``)."""

    def __init__(self, irreps_in, irrep_out, correlation: int, dtype=torch.float64):
        super().__init__()
        irreps_in = Irreps(irreps_in)
        self.num_features = irreps_in.count((0, 1))
        self.coupling_irreps = Irreps([ir for _, ir in irreps_in])
        self.correlation = correlation
        for nu in range(1, correlation + 1):
            u = U_matrix_real(self.coupling_irreps, irrep_out, nu, dtype=dtype)[-1]
            self.register_buffer(f"U_matrix_{nu}", u.to(torch.get_default_dtype()))
        self.weights = torch.nn.ParameterDict({})
        for i in range(1, correlation + 1):
            k = self.U_tensors(i).size()[-1]
            self.weights[str(i)] = torch.nn.Parameter(torch.randn(k, self.num_features) / k)

    def U_tensors(self, nu):
        return self._buffers[f"U_matrix_{nu}"]

    def forward(self, x):
        u = self.U_tensors(self.correlation).to(x.dtype)
        w = self.weights[str(self.correlation)].to(x.dtype)
        # "...ik,kc,bci -> bc..." evaluated as (U.W) then x, the opt_einsum order
        uw = torch.einsum("...ik,kc->...ic", u, w)
        out = torch.einsum("...ic,bci->bc...", uw, x)
        for corr in range(self.correlation - 1, 0, -1):
            c = torch.einsum("...k,kc->c...", self.U_tensors(corr).to(x.dtype),
                             self.weights[str(corr)].to(x.dtype))
            c = c + out
            out = torch.einsum("bc...i,bci->bc...", c, x)
        return out.reshape(out.shape[0], -1)


class SymmetricContraction(torch.nn.Module):
    """``gnn/mace.py:112-177`` with ``element_dependent=False``."""

    def __init__(self, irreps_in, irreps_out, correlation: int):
        super().__init__()
        self.irreps_in = Irreps(irreps_in)
        self.irreps_out = Irreps(irreps_out)
        self.contractions = torch.nn.ModuleDict()
        for mul, ir in self.irreps_out:  # keys as the reference: str(irrep_out) == '32x0e'
            self.contractions[f"{mul}x{ir}"] = Contraction(self.irreps_in, Irreps(str(ir)), correlation)

    # Test-only memory bound (tests/test_gpu_fullsize.py): > 0 evaluates node chunks of this
    # size under activation checkpointing.  Every node's arithmetic is unchanged (the
    # contraction is node-wise); only the [nodes, 32, 2l+1, 25, 25] intermediates are
    # recomputed in the backward instead of held (~48 GB for one 1k-node 4-layer graph in
    # fp64).  0 (default) keeps the reference's cost structure for the CPU baseline.
    node_chunk = 0

    def _forward(self, x):
        return torch.cat([self.contractions[f"{m}x{ir}"](x) for m, ir in self.irreps_out], dim=-1)

    def forward(self, x):
        c = SymmetricContraction.node_chunk
        if c and x.shape[0] > c:
            from torch.utils.checkpoint import checkpoint
            return torch.cat([checkpoint(self._forward, xc, use_reentrant=False)
                              for xc in x.split(c)], dim=0)
        return self._forward(x)
