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

import functools

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


class reshape_irreps(torch.nn.Module):  # noqa: N801
    """``gnn/mace.py:316-332``: mul-major rows ``[N, Σ mul·d]`` -> ``[N, mul, Σ d]``.  The
    product block keeps it as a submodule for API parity; its own path reads the rows."""

    def __init__(self, irreps) -> None:
        super().__init__()
        self.irreps = Irreps(irreps)

    def forward(self, tensor: torch.Tensor) -> torch.Tensor:
        n = tensor.shape[0]
        fields, ix = [], 0
        for mul, ir in self.irreps:
            d = ir.dim
            fields.append(tensor[:, ix: ix + mul * d].reshape(n, mul, d))
            ix += mul * d
        return torch.cat(fields, dim=-1)


def unreshape_irreps(irreps: Irreps, t: torch.Tensor) -> torch.Tensor:
    """Inverse of ``reshape_irreps``: ``[N, mul, Σ d]`` -> mul-major rows ``[N, Σ mul·d]``."""
    n, mul = t.shape[0], t.shape[1]
    rows, ix = [], 0
    for m, ir in irreps:
        if m != mul:
            raise ValueError(f"reshape_irreps layout needs one multiplicity, got {irreps}")
        rows.append(t[:, :, ix: ix + ir.dim].reshape(n, mul * ir.dim))
        ix += ir.dim
    if ix != t.shape[2]:
        raise ValueError(f"input {tuple(t.shape)} does not match {irreps}")
    return torch.cat(rows, dim=1).contiguous()


@functools.lru_cache(maxsize=None)
def _reference_U(coupling: str, l: int, nu: int) -> torch.Tensor:
    """The reference's ``U_matrix_{nu}`` buffer (fp32, reference shape), built once per process
    and shared by every layer's ``state_dict()`` (≈217 MB per lmax-4 layer): periodic
    checkpointing does not rebuild it.  Like any state_dict entry it aliases held state."""
    shape = cg.reference_U_shape(coupling, l, nu)
    return torch.tensor(cg.U_matrix(coupling, l, nu), dtype=torch.float32).reshape(shape)


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
        # correlation 4: the table-driven kernels (csrc/eelg_scg.hip) over the same plan
        self._table = (ops.ScgTable(plan, tuple(ir.l for _, ir in self.irreps_in), ls, self.mul)
                       if kernel_sets.table_driven(correlation) else None)
        self._sig = None if self._table else cg.fnv1a64(cg.sc_signature(coupling, ls, correlation))
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
        self._ahead = None           # (coef, event, stream) issued by coefficients_ahead
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
            state_dict[key] = u if u is not None else _reference_U(module._coupling, l, nu)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        """Accepts the reference's ``U_matrix_{nu}`` buffers.  A U equal to the derived one
        (to fp32 accuracy) is simply verified.  A U in another basis of the same space (e.g.
        a different path order or sign convention) is adopted: its symmetrisation replaces
        the matching block of ``u_sym``, so the contraction computes exactly what the
        reference computes with that U and the loaded weights.  A U with symmetric weight on
        monomials the generated kernels do not evaluate raises.

        Every load that carries U buffers for this module starts from the derived basis: a
        block not carried by (or equal to the derived one in) this checkpoint goes back to the
        derived block, so loading a standard checkpoint after one in another basis computes
        with the derived U again.  A load with no U buffer of this module (a weights-only
        partial load) keeps the basis in use.  The adopted
        blocks are computed first and written only when every U of the module checked out."""
        plan = None
        adopted, loaded, failed, seen = [], {}, False, False
        for l, nu, key in list(self._u_keys(prefix)):
            if key not in state_dict:
                continue
            seen = True
            u = state_dict.pop(key).detach().to("cpu", torch.float64)
            want = cg.reference_U_shape(self._coupling, l, nu)
            if tuple(u.shape) != want:
                error_msgs.append(f"size mismatch for {key}: copying a param with shape "
                                  f"{tuple(u.shape)}, the reference shape is {want}")
                failed = True
                continue
            ref = torch.from_numpy(cg.U_matrix(self._coupling, l, nu)).reshape(want)
            if float((u - ref).abs().max()) <= 1e-6 * float(ref.abs().max()):
                continue
            plan = plan or cg.symcon_plan(self._coupling, self._ls, self.correlation)
            try:
                k0, block = cg.symcon_block_from_U(plan, l, nu, u.numpy())
            except ValueError as e:
                error_msgs.append(f"{key}: {e}")
                failed = True
                continue
            adopted.append((k0, block))
            loaded[(l, nu)] = u.to(torch.float32)
        if seen and not failed:
            plan = plan or cg.symcon_plan(self._coupling, self._ls, self.correlation)
            fresh = torch.tensor(plan.ubig, dtype=torch.float64)
            for k0, block in adopted:
                fresh[:, k0: k0 + block.shape[1]] = torch.from_numpy(block)
            with torch.no_grad():
                self.u_sym.copy_(fresh.to(self.u_sym))
            self._u_csr = None
            self._u_loaded = loaded
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
        """(U_sym @ W)^T with the 1.6 %-dense U_sym applied as CSR on the GPU: [mul, coef_ld],
        rows zero-padded from nterms to the kernels' coefficient stride (CPU: [mul, nterms])."""
        if self.u_sym.is_cuda:
            if getattr(self, "_u_csr", None) is None:
                self._u_csr = ops.SparseRows(self.u_sym)
            ld = self._table.ldc if self._table else self._config()[1]["coef_ld"]
            return ops.symcon_coefficients(self.weight_matrix(), self._u_csr, ld)
        return torch.matmul(self.u_sym, self.weight_matrix()).t().contiguous()

    def forward(self, x: torch.Tensor, y: torch.Tensor = None) -> torch.Tensor:
        """``x``: the node rows ``[N, Σ mul·(2l+1)]`` in e3nn mul-major order (the fast path
        used by ``EquivariantProductBlock``), or the reference's ``reshape_irreps`` output
        ``[N, mul, Σ(2l+1)]`` (``gnn/mace.py:171-175,316-332``; that layout is converted back
        to rows, one copy).  ``y`` is the reference's element attribute, unused in its
        non-element-dependent branch (``gnn/mace.py:261-275``); it must be None here.
        Returns ``[N, Σ mul·(2l_out+1)]`` mul-major, as the reference's ``torch.cat``."""
        if y is not None:
            raise NotImplementedError("element-dependent symmetric contraction (y given) is not "
                                      "on the hot path: the model passes y=None (gnn/blocks.py:486)")
        if x.dim() == 3:
            x = unreshape_irreps(self.irreps_in, x)
        if self._table is not None:
            ahead, self._ahead = self._ahead, None
            if ahead is not None:
                coef = ahead[0]
                torch.cuda.current_stream(x.device).wait_event(ahead[1])
                coef.record_stream(torch.cuda.current_stream(x.device))
            else:
                coef = self.coefficients()
            return ops.symmetric_contraction_table(x, coef, self._table)
        idx, info = self._config()
        side = ops.side_stream(x.device, 1) if (ops.OVERLAP and x.is_cuda) else None
        if side is None:
            return ops.symmetric_contraction(x, self.coefficients(), idx, info, self.mul)
        # the coefficient chain (weight matrix -> U_sym SpMM) runs on the side stream, so its
        # backward -- and the coefficient-gradient kernel launched there by the contraction's
        # backward -- overlaps the rest of the backward on the main stream
        main = torch.cuda.current_stream(x.device)
        ahead, self._ahead = self._ahead, None
        if ahead is not None and ahead[2] is side:
            coef, ev = ahead[0], ahead[1]
            main.wait_event(ev)
        else:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                coef = self.coefficients()
            main.wait_stream(side)
        coef.record_stream(main)
        return ops.symmetric_contraction(x, coef, idx, info, self.mul, side=side)

    def coefficients_ahead(self, side) -> None:
        """Issue the coefficient chain (weight matrix -> U_sym SpMM) on the side stream now and
        keep (coef, event) for this module's next forward.  The model calls it for every layer
        at the start of its forward (the coefficients depend on the weights only), so each
        layer's main stream waits on work finished long before, instead of a main -> side ->
        main round trip at the layer (two cross-stream waits of ~20 us each on the critical
        path).  The caller orders ``side`` after the main stream's last weight update."""
        with torch.cuda.stream(side):
            coef = self.coefficients()
        ev = torch.cuda.Event()
        ev.record(side)
        self._ahead = (coef, ev, side)
