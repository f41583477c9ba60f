"""Correlation 4 (VERDICT r4 gap 3; the reference's ``U_matrix_real`` couples four copies
through natural-parity intermediate irreps up to l = 11, ``filter_ir_mid``, gnn/mace.py:435-477).
It runs the table-driven contraction kernels (``csrc/eelg_scg.hip``) over the same sparse
symmetrised polynomial as the generated correlation-1..3 kernels.  CPU checks: the filtered U
matrices against the oracle's restatement, the 4-slot polynomial against the oracle's dense
U.W contraction, and the kernels' table encoding (``gnn.ops.ScgTable``: packed component
indices, output ranges, row layout) evaluated by a numpy model of the kernel loops."""
import numpy as np
import pytest
import torch

import oracle.mace as omace
import oracle.o3 as oo3
from gnn import cg, kernel_sets


def _coupling(lmax):
    return "+".join(f"{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))


def _hidden(lmax, mul):
    return "+".join(f"{mul}x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))


@pytest.mark.parametrize("lmax", [1, 2])
def test_correlation4_u_matrices_match_oracle(lmax):
    coup = _coupling(lmax)
    for l in range(lmax + 1):
        ir = oo3.Irreps(str(oo3.Irrep(l, (-1) ** l)))
        a = cg.U_matrix(coup, l, 4)
        b = omace.U_matrix_real(oo3.Irreps(coup), ir, 4)[-1].numpy()
        assert a.size == b.size
        assert np.abs(a.reshape(b.shape) - b).max() < 1e-12


def test_correlation4_filter_drops_unnatural_intermediates():
    """Without the filter the four-fold coupling of 0e+1o has more paths (through 1e, 0o ...):
    the filtered basis is a strict subset, as the reference's."""
    irs = tuple(ir for _, ir in cg.Irreps("0e+1o"))
    full = [ir for ir, _ in cg._coupled(irs, 4, cg.Ir(0, 1), False)]
    filt = [ir for ir, _ in cg._coupled(irs, 4, cg.Ir(0, 1), True)]
    assert 0 < len(filt) < len(full)
    assert cg.U_matrix("0e+1o", 0, 4).shape[-1] == len(filt)


def _oracle_sc(lmax, mul, seed=0):
    torch.manual_seed(seed)
    h = oo3.Irreps(_hidden(lmax, mul))
    return omace.SymmetricContraction(h, h, 4).double()


def _weights(sc, plan, mul):
    ws = []
    for l, nu, k in plan.weight_blocks:
        w = sc.contractions[f"{mul}x{oo3.Irrep(l, (-1) ** l)}"].weights[str(nu)]
        assert w.shape == (k, mul)
        ws.append(w.detach())
    return torch.cat(ws).numpy()


@pytest.mark.parametrize("lmax", [1, 2])
def test_correlation4_polynomial_equals_dense_contraction(lmax):
    plan = cg.symcon_plan(_coupling(lmax), tuple(range(lmax + 1)), 4)
    assert {nu for nu, _, _ in plan.terms} == {1, 2, 3, 4}
    assert all(len(cls) == 4 for _, cls, _ in plan.terms)
    outs = [o for _, _, o in plan.terms]
    assert outs == sorted(outs)                       # the table kernels' output ranges
    sc = _oracle_sc(lmax, 4)
    coef = plan.ubig @ _weights(sc, plan, 4)
    x = np.random.default_rng(1).normal(size=(5, 4, plan.D))
    out = np.zeros((5, 4, plan.D))
    for t, (nu, cls, o) in enumerate(plan.terms):
        m = np.ones((5, 4))
        for i in cls[:nu]:
            m = m * x[:, :, i]
        out[:, :, o] += coef[t] * m
    with torch.no_grad():
        ref = sc(torch.tensor(x)).numpy()
    mine = np.concatenate([out[:, :, l * l:(l + 1) ** 2].reshape(5, -1) for l in range(lmax + 1)], 1)
    # the oracle holds U as the default dtype (fp32) buffers, as the reference
    assert np.abs(mine - ref).max() < 1e-6 * np.abs(ref).max()


def _table_model(tab, x_rows, coef, g_rows):
    """numpy model of eelg_scg_fwd / _bwd_x / _bwd_coef (the kernels' loops, fp64)."""
    d = tab.desc
    D, Dout, mul = d.D, d.Dout, d.mul
    terms = tab._terms.numpy().astype(np.int64) & 0xffffffff
    outs = tab._outs.numpy()
    n = x_rows.shape[0]
    col = np.ones((n, mul, D + 1))
    for a in range(D):
        for c in range(mul):
            col[:, c, a] = x_rows[:, d.xb[a] + c * d.xs[a]]
    idx = np.stack([(terms >> (8 * k)) & 0xff for k in range(4)], 1)
    out = np.zeros((n, mul * Dout))
    gx_col = np.zeros((n, mul, D + 1))
    gcoef = np.zeros((mul, tab.ldc))
    gq = np.zeros((n, mul, Dout + 1))
    for q in range(Dout):
        for c in range(mul):
            gq[:, c, q] = g_rows[:, d.ob[q] + c * d.os[q]]
    for q in range(Dout):
        for t in range(d.orow[q], d.orow[q + 1]):
            f = col[:, :, idx[t]]                     # [n, mul, 4]
            v = f.prod(-1)
            for c in range(mul):
                out[:, d.ob[q] + c * d.os[q]] += coef[c, t] * v[:, c]
            cg_ = coef[None, :, t] * gq[:, :, q]
            for k in range(4):
                gx_col[:, :, idx[t, k]] += cg_ * np.prod(np.delete(f, k, axis=-1), -1)
    for t in range(tab.ldc):
        gcoef[:, t] = (gq[:, :, outs[t]] * col[:, :, idx[t]].prod(-1)).sum(0)
    gx = np.zeros_like(x_rows)
    for a in range(D):
        for c in range(mul):
            gx[:, d.xb[a] + c * d.xs[a]] = gx_col[:, c, a]
    return out, gx, gcoef


def test_correlation4_table_encoding_matches_oracle():
    """The ScgTable the kernels read (packed indices, constant-1 slot, zero-output padding,
    mul-major row layout) reproduces the oracle's contraction, its input gradient and the
    coefficient gradient that autograd gives through coef = U_sym W."""
    from gnn import ops
    lmax, mul, n = 1, 4, 6
    plan = cg.symcon_plan(_coupling(lmax), tuple(range(lmax + 1)), 4)
    tab = ops.ScgTable(plan, tuple(range(lmax + 1)), tuple(range(lmax + 1)), mul)
    assert tab.ldc % 64 == 0 and tab.ldc >= len(plan.terms)
    assert tab.desc.orow[tab.desc.Dout] == len(plan.terms)
    sc = _oracle_sc(lmax, mul)
    w = torch.tensor(_weights(sc, plan, mul), requires_grad=True)
    coef = torch.zeros(mul, tab.ldc, dtype=torch.float64)
    coef_live = (torch.tensor(plan.ubig) @ w).t()
    rng = np.random.default_rng(3)
    x = torch.tensor(rng.normal(size=(n, mul * plan.D)), requires_grad=True)
    g = rng.normal(size=(n, mul * plan.D))
    with torch.no_grad():
        coef[:, :len(plan.terms)] = coef_live
    out, gx, gcoef = _table_model(tab, x.detach().numpy(), coef.numpy(), g)
    # oracle on the same rows ([N, mul, D] per the reference's reshape_irreps)
    xr = omace.reshape_irreps(oo3.Irreps(_hidden(lmax, mul)), x)
    ref = sc(xr)
    assert np.abs(out - ref.detach().numpy()).max() < 1e-6 * ref.abs().max().item()
    ref.backward(torch.tensor(g))
    assert np.abs(gx - x.grad.numpy()).max() < 1e-6 * x.grad.abs().max().item()
    # coefficient gradient -> weight gradient through U_sym, against autograd's
    gw = plan.ubig.T @ gcoef[:, :len(plan.terms)].T
    ws = [sc.contractions[f"{mul}x{oo3.Irrep(l, (-1) ** l)}"].weights[str(nu)].grad
          for l, nu, _ in plan.weight_blocks]
    ref_gw = torch.cat(ws).numpy()
    assert np.abs(gw - ref_gw).max() < 1e-6 * np.abs(ref_gw).max()
    assert np.abs(gcoef[:, len(plan.terms):]).max() == 0.0


def test_correlation4_constructs_up_to_lmax3_and_raises_at_lmax4():
    from argparse import Namespace
    from helpers import params
    from gnn.model import EnergyEquivGNN
    for lmax in (1, 2, 3):
        p = Namespace(**{**vars(params(2)), "lmax": lmax, "correlation": 4,
                         "hidden_irreps": kernel_sets.hidden_irreps_str(lmax),
                         "readout_irreps": kernel_sets.hidden_irreps_str(lmax, 16)})
        m = EnergyEquivGNN(p)
        assert any(getattr(mod, "_table", None) is not None for mod in m.modules())
    with pytest.raises(NotImplementedError, match="table-driven"):
        EnergyEquivGNN(Namespace(**{**vars(params(2)), "correlation": 4}))
