"""Init-time constants of the hot path, computed in numpy (float64).

* ``wigner_3j(l1, l2, l3)`` -- real Clebsch-Gordan tensor in e3nn's real basis
  (the one ``gnn/mace.py:399`` and ``o3.TensorProduct`` use).  Built from the
  Racah *3j-symbol* formula, converted to SU(2) CG, then moved to the real
  basis with e3nn's ``change_basis_real_to_complex`` convention and
  Frobenius-normalised.  (The test oracle builds the same tensor from the CG
  form of the Racah formula with exact rationals; ``tests/`` cross-checks.)
* spherical-harmonic recursion ``Y_{l+1} = s_l C(l,1,l+1).(Y_l (x) Y_1)``
  (e3nn's generator for its hard-coded polynomials; y is the polar axis).
* TP instruction table (``tp_out_irreps_with_instructions``,
  ``gnn/mace.py:286-314``).
* MACE ``U_matrix_real`` coupling bases (``gnn/mace.py:363-477``) and their
  symmetrised sparse form used by the HIP symmetric-contraction kernels.
* the rank-4 stiffness change of basis standing in for
  ``ReducedTensorProducts('ijkl=jikl=ijlk=klij')`` (``gnn/blocks.py:427-442``).
"""
from __future__ import annotations

import functools
import itertools
import math
from typing import Dict, List, NamedTuple, Tuple

import numpy as np

from .irreps import Ir, Irreps


# --------------------------------------------------------------------------
# Clebsch-Gordan
# --------------------------------------------------------------------------
def _fact(n: int) -> int:
    return math.factorial(n)


def _three_j(j1: int, j2: int, j3: int, m1: int, m2: int, m3: int) -> float:
    """Wigner 3j symbol (Racah formula), integer arguments."""
    if m1 + m2 + m3 != 0 or not (abs(j1 - j2) <= j3 <= j1 + j2):
        return 0.0
    if abs(m1) > j1 or abs(m2) > j2 or abs(m3) > j3:
        return 0.0
    tri_num = _fact(j1 + j2 - j3) * _fact(j1 - j2 + j3) * _fact(-j1 + j2 + j3)
    tri_den = _fact(j1 + j2 + j3 + 1)
    mprod = (_fact(j1 + m1) * _fact(j1 - m1) * _fact(j2 + m2) * _fact(j2 - m2)
             * _fact(j3 + m3) * _fact(j3 - m3))
    kmin = max(0, j2 - j3 - m1, j1 - j3 + m2)
    kmax = min(j1 + j2 - j3, j1 - m1, j2 + m2)
    # exact rational sum with a common denominator
    terms = []
    for k in range(kmin, kmax + 1):
        den = (_fact(k) * _fact(j3 - j2 + k + m1) * _fact(j3 - j1 + k - m2)
               * _fact(j1 + j2 - j3 - k) * _fact(j1 - k - m1) * _fact(j2 - k + m2))
        terms.append(((-1) ** k, den))
    if not terms:
        return 0.0
    lcm = 1
    for _, d in terms:
        lcm = lcm * d // math.gcd(lcm, d)
    num = sum(s * (lcm // d) for s, d in terms)
    # value = sign * sqrt(tri_num*mprod/tri_den) * num / lcm
    sign = (-1) ** (j1 - j2 - m3)
    mag2_num = tri_num * mprod * num * num
    mag2_den = tri_den * lcm * lcm
    g = math.gcd(mag2_num, mag2_den)
    val = math.sqrt((mag2_num // g) / (mag2_den // g)) if mag2_num else 0.0
    return float(sign * (1 if num >= 0 else -1) * val)


def _su2_cg(l1: int, l2: int, l3: int) -> np.ndarray:
    """<l1 m1 l2 m2 | l3 m3> indexed [l1+m1, l2+m2, l3+m3]."""
    out = np.zeros((2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1))
    for m1 in range(-l1, l1 + 1):
        for m2 in range(-l2, l2 + 1):
            m3 = m1 + m2
            if abs(m3) <= l3:
                out[l1 + m1, l2 + m2, l3 + m3] = ((-1) ** (l1 - l2 + m3) * math.sqrt(2 * l3 + 1)
                                                  * _three_j(l1, l2, l3, m1, m2, -m3))
    return out


def _real_to_complex(l: int) -> np.ndarray:
    """e3nn convention: rows = complex m, columns = real index, times (-i)^l."""
    q = np.zeros((2 * l + 1, 2 * l + 1), dtype=np.complex128)
    r = 1.0 / math.sqrt(2.0)
    for m in range(1, l + 1):
        q[l - m, l + m] = r
        q[l - m, l - m] = -1j * r
        q[l + m, l + m] = (-1) ** m * r
        q[l + m, l - m] = 1j * (-1) ** m * r
    q[l, l] = 1.0
    return ((-1j) ** l) * q


@functools.lru_cache(maxsize=None)
def _w3j_cached(l1: int, l2: int, l3: int) -> np.ndarray:
    c = _su2_cg(l1, l2, l3).astype(np.complex128)
    q1, q2, q3 = _real_to_complex(l1), _real_to_complex(l2), _real_to_complex(l3)
    c = np.einsum("ij,kl,nm,ikn->jlm", q1, q2, np.conj(q3), c)
    assert np.abs(c.imag).max() < 1e-9, (l1, l2, l3)
    c = c.real
    return c / np.linalg.norm(c)


def wigner_3j(l1: int, l2: int, l3: int) -> np.ndarray:
    """Real CG tensor [2l1+1, 2l2+1, 2l3+1], Frobenius norm 1 (float64 copy)."""
    if not abs(l1 - l2) <= l3 <= l1 + l2:
        raise ValueError((l1, l2, l3))
    return _w3j_cached(l1, l2, l3).copy()


def nonzeros(c: np.ndarray, tol: float = 1e-12) -> List[Tuple[Tuple[int, ...], float]]:
    idx = np.argwhere(np.abs(c) > tol)
    return [(tuple(int(t) for t in i), float(c[tuple(i)])) for i in idx]


# --------------------------------------------------------------------------
# Spherical harmonics recursion
# --------------------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def sh_recursion(lmax: int) -> Tuple[Tuple[Tuple[int, int, int, float], ...], ...]:
    """For l = 1..lmax-1: nonzero (i, j, k, s_l*C[i,j,k]) with
    ``Y_{l+1}[k] = sum s_l C[i,j,k] Y_l[i] v[j]`` (norm-normalised on the sphere)."""
    v = np.array([0.37, -0.61, 0.7])
    v /= np.linalg.norm(v)
    ys = [np.ones(1), v.copy()]
    out = []
    for l in range(1, lmax):
        c = wigner_3j(l, 1, l + 1)
        nxt = np.einsum("ijk,i,j->k", c, ys[l], ys[1])
        s = 1.0 / np.linalg.norm(nxt)
        ys.append(nxt * s)
        out.append(tuple((i, j, k, s * val) for (i, j, k), val in nonzeros(c)))
    return tuple(out)


def spherical_harmonics_np(lmax: int, vec: np.ndarray) -> np.ndarray:
    """Reference evaluation (component normalisation) for host-side checks."""
    n = np.linalg.norm(vec, axis=-1, keepdims=True)
    v = vec / np.maximum(n, 1e-12)
    ys = [np.ones(v.shape[:-1] + (1,)), v]
    for l, terms in enumerate(sh_recursion(lmax), start=1):
        y = np.zeros(v.shape[:-1] + (2 * l + 3,))
        for i, j, k, c in terms:
            y[..., k] += c * ys[l][..., i] * v[..., j]
        ys.append(y)
    return np.concatenate([math.sqrt(2 * l + 1) * y for l, y in enumerate(ys[: lmax + 1])], -1)


# --------------------------------------------------------------------------
# Tensor-product instruction table
# --------------------------------------------------------------------------
class TPPath(NamedTuple):
    slot: int        # output slot after sorting (== weight block index)
    i_in1: int       # index into node irreps
    i_in2: int       # index into SH irreps
    l1: int
    l2: int
    l3: int
    mul: int
    in1_off: int     # float offset of the node irreps block
    in2_off: int     # float offset of the SH block
    out_off: int     # float offset of the output slot
    coef: float      # sqrt(2 l3 + 1) (e3nn 'component' + 'element', mul2 == 1)


def tp_out_irreps_with_instructions(irreps1: Irreps, irreps2: Irreps, target: Irreps):
    """``gnn/mace.py:286-314``: returns (irreps_out, [(i1, i2, k, 'uvu', True)])."""
    outs, ins = [], []
    for i, (mul, ir_in) in enumerate(irreps1):
        for j, (_, ir_e) in enumerate(irreps2):
            for ir_o in ir_in.times(ir_e):
                if ir_o in target:
                    ins.append((i, j, len(outs), "uvu", True))
                    outs.append((mul, ir_o))
    irreps_out, perm = Irreps(outs).sort()
    ins = sorted([(a, b, perm[k], m, t) for a, b, k, m, t in ins], key=lambda x: x[2])
    return irreps_out, ins


def tp_paths(node_irreps: Irreps, sh_irreps: Irreps, target: Irreps) -> List[TPPath]:
    irreps_out, ins = tp_out_irreps_with_instructions(node_irreps, sh_irreps, target)
    o1, o2, oo = node_irreps.offsets(), sh_irreps.offsets(), irreps_out.offsets()
    paths = []
    for i1, i2, k, _, _ in ins:
        m1, ir1 = node_irreps[i1]
        m2, ir2 = sh_irreps[i2]
        assert m2 == 1
        ir3 = irreps_out[k].ir
        paths.append(TPPath(k, i1, i2, ir1.l, ir2.l, ir3.l, m1, o1[i1], o2[i2], oo[k],
                            math.sqrt(ir3.dim / m2)))
    return paths


# --------------------------------------------------------------------------
# MACE U matrices and their symmetrised sparse form
# --------------------------------------------------------------------------
# correlation 4: the reference couples through natural-parity irreps up to l = 11 only
# (``filter_ir_mid``, gnn/mace.py:444-458, applied at every coupling level, gnn/mace.py:392-393)
MID_FILTER_LMAX = 11


def _mid_ok(ir: Ir) -> bool:
    return ir.l <= MID_FILTER_LMAX and ir.p == (-1) ** ir.l


@functools.lru_cache(maxsize=None)
def _coupled(irs: Tuple[Ir, ...], nu: int, only=None, mid_filter: bool = False):
    """``_wigner_nj`` over ``nu`` copies of the (mul=1) coupling irreps.

    Returns [(ir_out, E)] with E of shape [ir_out.dim, D, ..., D] (nu copies of
    D = sum dims), stably sorted by irrep like ``gnn/mace.py:432``.  ``only``
    keeps just one output irrep at the last level (same relative order, since the
    sort is stable).  ``mid_filter``: the correlation-4 ``filter_ir_mid`` at every level."""
    D = sum(ir.dim for ir in irs)
    if nu == 1:
        eye, out, s = np.eye(D), [], 0
        for ir in irs:
            out.append((ir, eye[s: s + ir.dim]))
            s += ir.dim
        return tuple(x for x in out if only is None or x[0] == only)
    out = []
    for ir_l, c_l in _coupled(irs, nu - 1, None, mid_filter):
        s = 0
        for ir in irs:
            for ir_o in ir_l.times(ir):
                if only is not None and ir_o != only:
                    continue
                if mid_filter and not _mid_ok(ir_o):
                    continue
                w = wigner_3j(ir_o.l, ir_l.l, ir.l) * math.sqrt(ir_o.dim)
                t = np.einsum("jk,ijl->ikl", c_l.reshape(ir_l.dim, -1), w)
                e = np.zeros((ir_o.dim,) + (D,) * nu)
                e[..., s: s + ir.dim] = t.reshape((ir_o.dim,) + (D,) * (nu - 1) + (ir.dim,))
                out.append((ir_o, e))
            s += ir.dim
    return tuple(sorted(out, key=lambda x: x[0].order_key()))


@functools.lru_cache(maxsize=None)
def U_matrix(coupling: str, l_out: int, nu: int) -> np.ndarray:
    """U_nu for output irrep l_out (natural parity): [2l+1, D x nu, K_nu]."""
    irs = tuple(ir for _, ir in Irreps(coupling))
    target = Ir(l_out, (-1) ** l_out)
    # U_matrix_real(correlation=nu) filters the intermediate irreps iff nu == 4 (gnn/mace.py:444)
    mats = [e for ir, e in _coupled(irs, nu, target, nu == 4) if ir == target]
    return np.stack(mats, axis=-1)


class SymConPlan(NamedTuple):
    """Sparse polynomial form of MACE's SymmetricContraction for one irreps config.

    ``terms`` lists (degree, (a, b, c), out) with a<=b<=c (unused slots -1; correlation 4:
    four slots (a, b, c, d), ordered by ``out``) and
    ``out`` in 0..D-1 (the [L][M] output component).  ``ubig`` [nnz, K_total]
    maps the stacked weights (order: for L: W1, W2, W3 ... per ``weight_blocks``)
    to the per-term coefficients: coef[term, c] = (ubig @ W_all)[term, c]."""
    D: int
    ls: Tuple[int, ...]
    terms: Tuple[Tuple[int, Tuple[int, int, int], int], ...]
    ubig: np.ndarray
    weight_blocks: Tuple[Tuple[int, int, int], ...]   # (l_out, nu, K)


def _sym_classes(D: int, deg: int):
    return list(itertools.combinations_with_replacement(range(D), deg))


@functools.lru_cache(maxsize=None)
def symcon_plan(coupling: str, out_ls: Tuple[int, ...], correlation: int) -> SymConPlan:
    irs = tuple(ir for _, ir in Irreps(coupling))
    D = sum(ir.dim for ir in irs)
    ls_out_off = {}
    off = 0
    for l in out_ls:
        ls_out_off[l] = off
        off += 2 * l + 1
    Dout = off
    blocks, cols = [], {}
    kt = 0
    slots = max(3, correlation)    # monomial index slots of a term (unused: -1)
    for l in out_ls:
        for nu in range(1, correlation + 1):
            k = U_matrix(coupling, l, nu).shape[-1]
            blocks.append((l, nu, k))
            cols[(l, nu)] = (kt, k)
            kt += k
    rows: Dict[Tuple[int, Tuple[int, int, int], int], np.ndarray] = {}
    for l in out_ls:
        for nu in range(1, correlation + 1):
            u = U_matrix(coupling, l, nu)          # [2l+1, D..., K]
            k0, k = cols[(l, nu)]
            for cls in _sym_classes(D, nu):
                perms = set(itertools.permutations(cls))
                acc = np.zeros((2 * l + 1, k))
                for p in perms:
                    acc += u[(slice(None),) + p]
                for m in range(2 * l + 1):
                    if np.abs(acc[m]).max() > 1e-12:
                        key = (nu, tuple(cls) + (-1,) * (slots - nu), ls_out_off[l] + m)
                        r = np.zeros(kt)
                        r[k0: k0 + k] = acc[m]
                        rows[key] = r
    # canonical order: by (a, b) pair, then degree-2 term before degree-3 terms,
    # then c, then output component; degree-1 terms first
    def order(key):
        nu, (a, b, c), o = key
        if nu == 1:
            return (0, a, 0, 0, 0, o)
        return (1, a, b, 0 if nu == 2 else 1, c, o)

    def order_by_output(key):
        # correlation 4 (the generic kernels, csrc/eelg_scg.hip): grouped by output component
        nu, cls, o = key
        return (o, nu, cls)

    keys = sorted(rows, key=order if correlation <= 3 else order_by_output)
    ubig = np.stack([rows[k] for k in keys]) if keys else np.zeros((0, kt))
    return SymConPlan(Dout, tuple(out_ls), tuple(keys), ubig, tuple(blocks))


def reference_U_shape(coupling: str, l_out: int, nu: int) -> Tuple[int, ...]:
    """Shape of the reference's ``U_matrix_{nu}`` buffer (``gnn/mace.py:198-205``): the
    stacked [2l+1, D x nu, K] tensor with ``squeeze()`` applied per path before stacking
    (``:462-476``), so the leading 1 of l_out = 0 is dropped."""
    u = U_matrix(coupling, l_out, nu)
    return tuple(u.shape[1:]) if u.shape[0] == 1 else tuple(u.shape)


def symcon_block_from_U(plan: SymConPlan, l_out: int, nu: int, u: np.ndarray,
                        tol: float = 1e-6) -> Tuple[int, np.ndarray]:
    """(first column, [nterms, K] values) of the (l_out, nu) weight block of ``plan.ubig``,
    recomputed from a U tensor given in ANY basis of that block ([2l+1, D x nu, K], or the
    reference's squeezed shape).

    The symmetric contraction only sees U through its symmetrisation over the nu input
    slots, summed per monomial class: ``row(cls, m) = sum over distinct permutations p of
    cls of U[m, p]`` (``symcon_plan``).  Raises ValueError when the symmetrised U has weight
    on a (class, component) the generated kernels have no term for: such a basis is not
    representable, and silently dropping it would change the model."""
    m_dim = 2 * l_out + 1
    u = np.asarray(u, dtype=np.float64)
    if u.ndim == nu + 1:                       # squeezed l_out = 0 form
        u = u[None]
    if u.shape[0] != m_dim or u.ndim != nu + 2:
        raise ValueError(f"U for l={l_out}, nu={nu}: unexpected shape {u.shape}")
    D = u.shape[1]
    k = u.shape[-1]
    kt0 = 0
    for l, n, kk in plan.weight_blocks:
        if (l, n) == (l_out, nu):
            if kk != k:
                raise ValueError(f"U for l={l_out}, nu={nu}: {k} basis columns, expected {kk}")
            break
        kt0 += kk
    else:
        raise ValueError(f"no weight block (l={l_out}, nu={nu}) in the plan")
    sym = np.zeros_like(u)
    for p in itertools.permutations(range(1, nu + 1)):
        sym += np.transpose(u, (0,) + p + (nu + 1,))
    fact = math.factorial(nu)
    off = 0
    for l in plan.ls:
        if l == l_out:
            break
        off += 2 * l + 1
    want = {(cls[:nu], o - off): i for i, (n, cls, o) in enumerate(plan.terms)
            if n == nu and off <= o < off + m_dim}
    block = np.zeros((len(plan.terms), k))
    scale = max(np.abs(u).max(), 1e-300)
    for cls in _sym_classes(D, nu):
        n_distinct = len(set(itertools.permutations(cls)))
        acc = sym[(slice(None),) + cls] * (n_distinct / fact)      # [2l+1, K]
        for m in range(m_dim):
            i = want.get((tuple(cls), m))
            if i is not None:
                block[i] = acc[m]
            elif np.abs(acc[m]).max() > tol * scale:
                raise ValueError(f"U for l={l_out}, nu={nu} has a symmetric component on monomial "
                                 f"{cls} -> m={m}, which the generated kernels do not evaluate")
    return kt0, block


# --------------------------------------------------------------------------
# Rank-4 stiffness change of basis ('2x0e+2x2e+1x4e' -> 3x3x3x3)
# --------------------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def stiffness_change_of_basis() -> np.ndarray:
    """[21, 3, 3, 3, 3] orthonormal rows spanning tensors with ij, kl and (ij)<->(kl)
    symmetry, ordered 0e, 0e, 2e(5), 2e(5), 4e(9).  Within a multiplicity the
    basis is our own Gram-Schmidt choice (e3nn's is unpinned; the preceding
    ``o3.Linear`` absorbs it)."""
    perms = [(0, 1, 2, 3, 4), (0, 2, 1, 3, 4), (0, 1, 2, 4, 3), (0, 2, 1, 4, 3),
             (0, 3, 4, 1, 2), (0, 4, 3, 1, 2), (0, 3, 4, 2, 1), (0, 4, 3, 2, 1)]
    keep = {0: [], 2: [], 4: []}
    for la in (0, 1, 2):
        for lb in (0, 1, 2):
            for L in range(abs(la - lb), la + lb + 1):
                if L not in keep:
                    continue
                t = np.einsum("ija,klb,abm->mijkl", wigner_3j(1, 1, la), wigner_3j(1, 1, lb),
                              wigner_3j(la, lb, L))
                t = sum(np.transpose(t, p) for p in perms) / len(perms)
                for u in keep[L]:
                    t = t - (t * u).sum() / (u * u).sum() * u
                n = np.linalg.norm(t)
                if n > 1e-8:
                    keep[L].append(t / n * math.sqrt(2 * L + 1))
    assert [len(keep[L]) for L in (0, 2, 4)] == [2, 2, 1]
    return np.concatenate([t for L in (0, 2, 4) for t in keep[L]], axis=0)


@functools.lru_cache(maxsize=None)
def silu_normalize2mom() -> float:
    """e3nn ``normalize2mom(silu)``: 1/sqrt(mean(silu(z)^2)), z = 1e6 N(0,1) draws, seed 0.

    Reproduced from the published constant-estimation procedure; the value is
    baked here (computed once with torch's CPU generator) to keep the product
    free of Monte-Carlo at import time."""
    return 1.6791767923989418


# --------------------------------------------------------------------------
# structural signatures (checked against the built library at load time)
# --------------------------------------------------------------------------
def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def tp_signature(node: Irreps, sh: Irreps, target: Irreps) -> str:
    paths = tp_paths(node, sh, target)
    return "tp|" + str(node) + "|" + str(sh) + "|" + ";".join(
        f"{p.slot},{p.l1},{p.l2},{p.l3},{p.in1_off},{p.in2_off},{p.out_off}" for p in paths)


def sc_signature(coupling: str, ls, corr: int) -> str:
    plan = symcon_plan(coupling, tuple(ls), corr)
    return "sc|" + coupling + f"|{corr}|" + ";".join(
        f"{nu},{a},{b},{c},{o}" for nu, (a, b, c), o in plan.terms)
