"""The irreps structures ``libeelg.so`` has generated kernels for (single source of truth: the
generator ``csrc/gen_kernels.py`` builds exactly these, and the modules check their structure
against them at construction, so an unsupported ``params`` fails when the model is built, with
the supported list, not at the first forward).

Reference ``params`` space (``gnn/model.py:31-42``, ``gnn/mace.py:112-177``): ``lmax`` (SH),
``hidden_irreps``, ``correlation``.  Generated here:

* tensor product: SH lmax 1..4, node irreps ``32x0e`` (first layer) or the natural-parity
  hidden irreps ``32x0e+32x1o+...`` up to the SH lmax (later layers);
* symmetric contraction: the same lmax, outputs = those hidden irreps, correlation 1..3.

``mul`` (channels per irrep) is 32: one lane per channel in the interaction kernels.
"""
from __future__ import annotations

from typing import Tuple

MUL = 32
LMAX = (1, 2, 3, 4)
CORRELATIONS = (1, 2, 3)


def natural(l: int) -> str:
    return f"{l}{'e' if l % 2 == 0 else 'o'}"


def hidden_irreps_str(lmax: int, mul: int = MUL) -> str:
    return "+".join(f"{mul}x{natural(l)}" for l in range(lmax + 1))


def coupling_str(lmax: int) -> str:
    return "+".join(natural(l) for l in range(lmax + 1))


def supported_text() -> str:
    return (f"generated kernel sets: SH lmax in {LMAX} with hidden_irreps "
            f"'{hidden_irreps_str(1)}' .. '{hidden_irreps_str(4)}' (32 channels of every l up to "
            f"the SH lmax), correlation in {CORRELATIONS}")


def check_tp(node, sh, target) -> None:
    """Raise NotImplementedError unless the interaction (node irreps x SH -> target) is a
    generated tensor-product set."""
    lmax = sh.lmax
    ok = (lmax in LMAX and str(sh) == str(_sh(lmax))
          and str(node) in (f"{MUL}x0e", hidden_irreps_str(lmax))
          and str(target) == coupling_target(lmax))
    if not ok:
        raise NotImplementedError(
            f"no HIP tensor-product kernels for {node} x {sh} -> {target}; {supported_text()}")


def check_sc(irreps_in, ls: Tuple[int, ...], correlation: int) -> None:
    """Raise NotImplementedError unless the symmetric contraction is a generated set."""
    lmax = irreps_in.lmax
    ok = (lmax in LMAX and str(irreps_in) == hidden_irreps_str(lmax)
          and tuple(ls) == tuple(range(lmax + 1)) and correlation in CORRELATIONS)
    if not ok:
        raise NotImplementedError(
            f"no HIP symmetric-contraction kernels for {irreps_in} -> l in {tuple(ls)}, "
            f"correlation {correlation}; {supported_text()}")


def coupling_target(lmax: int) -> str:
    """The interaction irreps ``(SH * mul).sort().simplify()`` (``gnn/model.py:36-37``)."""
    return hidden_irreps_str(lmax)


def _sh(lmax: int):
    from .irreps import Irreps
    return Irreps.spherical_harmonics(lmax)
