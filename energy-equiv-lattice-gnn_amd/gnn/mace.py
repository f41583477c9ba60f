"""MACE-derived pieces of the hot path (reference ``gnn/mace.py``).

``SymmetricContraction`` keeps the reference's module/parameter layout
(``contractions['32x0e'].weights['1'|'2'|'3']`` with shapes ``[K_nu, mul]``,
``gnn/mace.py:112-240``) but evaluates the contraction as the sparse
symmetrised polynomial of ``gnn/cg.py:symcon_plan``: the per-term coefficients
``coef[c, t] = (U_sym @ W)[t, c]`` are one small GEMM per call, and the
polynomial itself runs in the generated HIP kernels (``sc_fwd/bwd_*``).  The
dense ``[N, 32, 2l+1, 25, 25]`` intermediate of the reference never exists.
"""
from __future__ import annotations

import torch

from . import _lib, cg, kernel_sets, ops
from .irreps import Ir, Irreps

tp_out_irreps_with_instructions = cg.tp_out_irreps_with_instructions


def get_edge_vectors_and_lengths(positions, edge_index, shifts):
    """``gnn/mace.py:338-352`` (normalize=False); the model itself uses the fused
    ``eelg_edge_embed`` kernel."""
    sender, receiver = edge_index
    vectors = positions[receiver] - positions[sender] + shifts
    return vectors, torch.linalg.norm(vectors, dim=-1, keepdim=True)


class Contraction(torch.nn.Module):
    """Parameter holder with the reference's names (``gnn/mace.py:230-238``)."""

    def __init__(self, ks, num_features: int):
        super().__init__()
        self.weights = torch.nn.ParameterDict(
            {str(nu): torch.nn.Parameter(torch.randn(k, num_features) / k)
             for nu, k in enumerate(ks, start=1)})


class SymmetricContraction(torch.nn.Module):
    def __init__(self, irreps_in, irreps_out, correlation: int):
        super().__init__()
        self.irreps_in, self.irreps_out = Irreps(irreps_in), Irreps(irreps_out)
        self.mul = self.irreps_in.count("0e")
        self.correlation = correlation
        coupling = "+".join(str(ir) for _, ir in self.irreps_in)
        lmax = self.irreps_in.lmax
        ls = tuple(ir.l for _, ir in self.irreps_out)
        if any(ir.l > lmax for _, ir in self.irreps_out):
            raise NotImplementedError(
                f"output irreps {self.irreps_out} beyond the coupling lmax {lmax}: the reference "
                "U_matrix_real has no degree-1 path for them (gnn/mace.py:466-476)")
        if any(m != self.mul or ir.p != (-1) ** ir.l for m, ir in self.irreps_out):
            raise NotImplementedError(
                f"symmetric contraction outputs {self.irreps_out}: the kernels are generated for "
                f"{self.mul}x natural-parity outputs")
        # fail at construction, with the supported list, for structures without generated kernels
        kernel_sets.check_sc(self.irreps_in, tuple(ir.l for _, ir in self.irreps_out), correlation)
        plan = cg.symcon_plan(coupling, ls, correlation)
        self._sig = cg.fnv1a64(cg.sc_signature(coupling, ls, correlation))
        self.block_order = [(l, nu) for l, nu, _ in plan.weight_blocks]
        ks = {}
        for l, nu, k in plan.weight_blocks:
            ks.setdefault(l, []).append(k)
        self.contractions = torch.nn.ModuleDict()
        for mul, ir in self.irreps_out:
            self.contractions[f"{mul}x{ir}"] = Contraction(ks[ir.l], self.mul)
        self.register_buffer("u_sym", torch.tensor(plan.ubig, dtype=torch.float32), persistent=False)
        self._cfg = None
        self._coupling, self._ls = coupling, ls
        self._u_loaded = {}          # (l, nu) -> U adopted from a loaded state_dict (CPU f32)
        self._register_state_dict_hook(SymmetricContraction._emit_reference_U)

    # -- reference checkpoints (gnn/mace.py:198-205: U_matrix_{nu} buffers per Contraction) --
    def _u_keys(self, prefix: str):
        for mul, ir in self.irreps_out:
            for nu in range(1, self.correlation + 1):
                yield ir.l, nu, f"{prefix}contractions.{mul}x{ir}.U_matrix_{nu}"

    @staticmethod
    def _emit_reference_U(module, state_dict, prefix, local_metadata):
        """``state_dict()`` carries the reference's U buffers too (derived data, not held on
        the device), so a checkpoint of this model loads strictly into the reference."""
        for l, nu, key in module._u_keys(prefix):
            u = module._u_loaded.get((l, nu))
            if u is None:
                shape = cg.reference_U_shape(module._coupling, l, nu)
                u = torch.tensor(cg.U_matrix(module._coupling, l, nu), dtype=torch.float32).reshape(shape)
            state_dict[key] = u

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        """Accepts the reference's ``U_matrix_{nu}`` buffers.  A U equal to the derived one
        (to fp32 accuracy) is simply verified.  A U in another basis of the same space (e.g.
        a different path order or sign convention) is adopted: its symmetrisation replaces
        the matching block of ``u_sym``, so the contraction computes exactly what the
        reference computes with that U and the loaded weights.  A U with symmetric weight on
        monomials the generated kernels do not evaluate raises."""
        for l, nu, key in list(self._u_keys(prefix)):
            if key not in state_dict:
                continue
            u = state_dict.pop(key).detach().to("cpu", torch.float64)
            want = cg.reference_U_shape(self._coupling, l, nu)
            if tuple(u.shape) != want:
                error_msgs.append(f"size mismatch for {key}: copying a param with shape "
                                  f"{tuple(u.shape)}, the reference shape is {want}")
                continue
            ref = torch.from_numpy(cg.U_matrix(self._coupling, l, nu)).reshape(want)
            if float((u - ref).abs().max()) <= 1e-6 * float(ref.abs().max()):
                self._u_loaded.pop((l, nu), None)
                continue
            plan = cg.symcon_plan(self._coupling, self._ls, self.correlation)
            try:
                k0, block = cg.symcon_block_from_U(plan, l, nu, u.numpy())
            except ValueError as e:
                error_msgs.append(f"{key}: {e}")
                continue
            with torch.no_grad():
                self.u_sym[:, k0: k0 + block.shape[1]] = torch.from_numpy(block).to(self.u_sym)
            self._u_csr = None
            self._u_loaded[(l, nu)] = u.to(torch.float32)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def _config(self):
        if self._cfg is None:
            self._cfg = _lib.sc_config_by_sig(self._sig)
        return self._cfg

    def weight_matrix(self) -> torch.Tensor:
        ws = []
        for l, nu in self.block_order:
            ir = Ir(l, (-1) ** l)
            ws.append(self.contractions[f"{self.mul}x{ir}"].weights[str(nu)])
        return torch.cat(ws, dim=0)                     # [K_total, mul]

    def coefficients(self) -> torch.Tensor:
        """[mul, nterms] = (U_sym @ W)^T with the 1.6 %-dense U_sym applied as CSR on the GPU."""
        if self.u_sym.is_cuda:
            if getattr(self, "_u_csr", None) is None:
                self._u_csr = ops.SparseRows(self.u_sym)
            return ops.symcon_coefficients(self.weight_matrix(), self._u_csr)
        return torch.matmul(self.u_sym, self.weight_matrix()).t().contiguous()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idx, info = self._config()
        side = ops.side_stream(x.device, 1) if (ops.OVERLAP and x.is_cuda) else None
        if side is None:
            return ops.symmetric_contraction(x, self.coefficients(), idx, info, self.mul)
        # the coefficient chain (weight matrix -> U_sym SpMM) runs on the side stream, so its
        # backward -- and the coefficient-gradient kernel launched there by the contraction's
        # backward -- overlaps the rest of the backward on the main stream
        main = torch.cuda.current_stream(x.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            coef = self.coefficients()
        main.wait_stream(side)
        coef.record_stream(main)
        return ops.symmetric_contraction(x, coef, idx, info, self.mul, side=side)
