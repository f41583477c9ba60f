"""Independent pin of the Clebsch-Gordan half of the e3nn restatement.

``gnn/cg.py`` (Racah 3j formula with exact integer sums, then the SU(2) CG phase) and
``oracle/o3.py`` (the CG form of the Racah formula with exact rationals, restating e3nn
``o3/_wigner.py``) are both checked here against ``sympy.physics.wigner.clebsch_gordan``, an
implementation neither of them shares code with:

* every coupling of the hot path's tensor products and of the symmetric contraction's U matrices
  at the reference params (``gnn/mace.py:399-405``: ``wigner_3j`` of irreps up to lmax 4, output
  l up to 8);
* every (l1, l2, l3) with l1, l2, l3 <= 8 for the generalised couplings (``U_matrix_real``
  couples intermediate irreps up to l = 8 at lmax 4, correlation 3).

What stays unpinned offline is the complex -> real change of basis (e3nn's
``change_basis_real_to_complex`` phase convention) and the ReducedTensorProducts basis.
"""
import math
import os
import sys

import numpy as np
import pytest

sympy = pytest.importorskip("sympy")
from sympy.physics.wigner import clebsch_gordan, wigner_3j  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd"))
sys.path.insert(0, ROOT)

from gnn import cg  # noqa: E402
import oracle.o3 as oo3  # noqa: E402


def _triples(lmax_in, lmax_out):
    for l1 in range(lmax_in + 1):
        for l2 in range(lmax_in + 1):
            for l3 in range(abs(l1 - l2), min(l1 + l2, lmax_out) + 1):
                yield l1, l2, l3


def _sympy_cg(l1, l2, l3):
    out = np.zeros((2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1))
    for m1 in range(-l1, l1 + 1):
        for m2 in range(-l2, l2 + 1):
            m3 = m1 + m2
            if abs(m3) <= l3:
                out[l1 + m1, l2 + m2, l3 + m3] = float(clebsch_gordan(l1, l2, l3, m1, m2, m3))
    return out


@pytest.mark.parametrize("lmax_in,lmax_out", [(4, 8), (8, 8)])
def test_su2_clebsch_gordan_matches_sympy(lmax_in, lmax_out):
    n = 0
    for l1, l2, l3 in _triples(lmax_in, lmax_out):
        ref = _sympy_cg(l1, l2, l3)
        mine = cg._su2_cg(l1, l2, l3)
        orac = oo3._su2_cg(l1, l2, l3).numpy()
        assert np.abs(mine - ref).max() < 1e-13, (l1, l2, l3)
        assert np.abs(orac - ref).max() < 1e-13, (l1, l2, l3)
        n += 1
    assert n == sum(1 for _ in _triples(lmax_in, lmax_out))


def test_three_j_symbol_matches_sympy():
    """``gnn/cg._three_j`` (the Racah 3j formula the build's CG is made from) equals sympy's exact
    3j symbol, including the selection rules that make it vanish."""
    for l1, l2, l3 in _triples(4, 8):
        for m1 in range(-l1, l1 + 1):
            for m2 in range(-l2, l2 + 1):
                m3 = -m1 - m2
                if abs(m3) > l3:
                    continue
                ref = float(wigner_3j(l1, l2, l3, m1, m2, m3))
                assert abs(cg._three_j(l1, l2, l3, m1, m2, m3) - ref) < 1e-13, (l1, l2, l3, m1, m2)
    # outside the triangle / m-sum rules
    assert cg._three_j(1, 1, 3, 0, 0, 0) == 0.0
    assert cg._three_j(2, 2, 2, 1, 1, 1) == 0.0


def test_real_cg_is_the_unitary_image_of_the_sympy_cg():
    """The real-basis tensor ``cg.wigner_3j`` is sympy's complex CG moved by the build's change of
    basis and Frobenius-normalised: only that change of basis (an e3nn convention) is not pinned
    by sympy.  Here it is checked to be unitary and to map sympy's CG onto the real tensor."""
    for l1, l2, l3 in _triples(4, 8):
        q1, q2, q3 = (cg._real_to_complex(l) for l in (l1, l2, l3))
        for q in (q1, q2, q3):
            assert np.abs(q.conj().T @ q - np.eye(q.shape[0])).max() < 1e-13
        c = np.einsum("ij,kl,nm,ikn->jlm", q1, q2, np.conj(q3), _sympy_cg(l1, l2, l3).astype(complex))
        assert np.abs(c.imag).max() < 1e-12
        c = c.real / np.linalg.norm(c.real)
        assert np.abs(c - cg.wigner_3j(l1, l2, l3)).max() < 1e-12, (l1, l2, l3)
        # and the SU(2) CG's own normalisation: sum over m1, m2 of |<..|l3 m3>|^2 = 1 per m3
        s = (_sympy_cg(l1, l2, l3) ** 2).sum(axis=(0, 1))
        assert np.allclose(s, 1.0, atol=1e-13)
        assert math.isclose(np.linalg.norm(cg.wigner_3j(l1, l2, l3)), 1.0, rel_tol=1e-13)
