"""The irreps structures ``libeelg.so`` has generated kernels for (single source of truth: the
generator ``csrc/gen_kernels.py`` builds exactly these, and the modules check their structure
against them at construction, so an unsupported ``params`` fails when the model is built, with
the supported list, not at the first forward).

Reference ``params`` space (``gnn/model.py:31-42``, ``gnn/mace.py:112-177``): ``lmax`` (SH),
``hidden_irreps``, ``correlation``.  Generated here:

* tensor product: SH lmax 1..4, node irreps ``{mul}x0e`` (first layer) or the natural-parity
  hidden irreps ``{mul}x0e+{mul}x1o+...`` up to the SH lmax (later layers);
* symmetric contraction: the same lmax, outputs = those hidden irreps, correlation 1..3
  generated; correlation 4 (the reference's ``filter_ir_mid`` coupling) runs the table-driven
  kernels (``csrc/eelg_scg.hip``) for SH lmax <= 3 (``TABLE_LMAX``: at lmax 4 the reference's
  own ``U_matrix_4`` is a [9, 25, 25, 25, 25, K] tensor, gigabytes, and so is its host build);
* ``mul`` (channels per irrep) in ``MULS``: one lane per channel in the interaction kernels, a
  half-wave per 32 channels (mul = 64: two channel groups; mul = 16: half a half-wave).  The
  reference default and the benchmark configurations are 32; bf16 storage of the edge tensors
  (BASELINE config 5) is generated for 32 only.
"""
from __future__ import annotations

from typing import Tuple

MUL = 32
MULS = (16, 32, 64)
LMAX = (1, 2, 3, 4)
CORRELATIONS = (1, 2, 3)
TABLE_CORRELATIONS = (4,)
TABLE_LMAX = 3


def natural(l: int) -> str:
    return f"{l}{'e' if l % 2 == 0 else 'o'}"


def hidden_irreps_str(lmax: int, mul: int = MUL) -> str:
    return "+".join(f"{mul}x{natural(l)}" for l in range(lmax + 1))


def coupling_str(lmax: int) -> str:
    return "+".join(natural(l) for l in range(lmax + 1))


def supported_text() -> str:
    return (f"generated kernel sets: SH lmax in {LMAX} with hidden_irreps "
            f"'{hidden_irreps_str(1)}' .. '{hidden_irreps_str(4)}' (mul channels of every l up to "
            f"the SH lmax, mul in {MULS}), correlation in {CORRELATIONS}; correlation "
            f"{TABLE_CORRELATIONS[0]} (table-driven) for SH lmax <= {TABLE_LMAX}")


def mul_of(irreps) -> int:
    """the channel count of an all-equal-mul irreps (0 when the muls differ)"""
    muls = {m for m, _ in irreps}
    return muls.pop() if len(muls) == 1 else 0


def check_tp(node, sh, target) -> None:
    """Raise NotImplementedError unless the interaction (node irreps x SH -> target) is a
    generated tensor-product set."""
    lmax = sh.lmax
    mul = mul_of(node)
    ok = (lmax in LMAX and mul in MULS and str(sh) == str(_sh(lmax))
          and str(node) in (f"{mul}x0e", hidden_irreps_str(lmax, mul))
          and str(target) == coupling_target(lmax, mul))
    if not ok:
        raise NotImplementedError(
            f"no HIP tensor-product kernels for {node} x {sh} -> {target}; {supported_text()}")


def check_sc(irreps_in, ls: Tuple[int, ...], correlation: int) -> None:
    """Raise NotImplementedError unless the symmetric contraction is a generated set (or a
    table-driven one: correlation 4)."""
    lmax = irreps_in.lmax
    mul = mul_of(irreps_in)
    ok = (lmax in LMAX and mul in MULS and str(irreps_in) == hidden_irreps_str(lmax, mul)
          and tuple(ls) == tuple(range(lmax + 1))
          and (correlation in CORRELATIONS or (correlation in TABLE_CORRELATIONS and lmax <= TABLE_LMAX)))
    if not ok:
        raise NotImplementedError(
            f"no HIP symmetric-contraction kernels for {irreps_in} -> l in {tuple(ls)}, "
            f"correlation {correlation}; {supported_text()}")


def coupling_target(lmax: int, mul: int = MUL) -> str:
    """The interaction irreps ``(SH * mul).sort().simplify()`` (``gnn/model.py:36-37``)."""
    return hidden_irreps_str(lmax, mul)


def _sh(lmax: int):
    from .irreps import Irreps
    return Irreps.spherical_harmonics(lmax)


def table_driven(correlation: int) -> bool:
    """the contraction runs the table-driven kernels (eelg_scg_*) instead of a generated set"""
    return correlation in TABLE_CORRELATIONS
