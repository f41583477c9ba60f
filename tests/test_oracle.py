"""Pinning the oracle (CPU, no GPU): known answers derivable from reference code and
basis-independent invariants of the full model."""
import math

import numpy as np
import pytest
import torch

import oracle.blocks as ob
import oracle.mace as omace
import oracle.model as omodel
import oracle.o3 as oo3
from oracle.train import stiffness_loss

from helpers import batch, batch_to, params
from helpers_mandel import rotate_mandel

F64 = torch.float64


def small_params(**kw):
    """A fast configuration exercising the same code paths (lmax 2, mul 8)."""
    from argparse import Namespace
    p = Namespace(lmax=2, hidden_irreps="8x0e+8x1o+8x2e", readout_irreps="4x0e+4x1o+4x2e",
                  num_edge_bases=6, interaction_reduction="sum", interaction_bias=True,
                  agg_norm_const=4.0, inter_MLP_dim=16, inter_MLP_layers=3, correlation=3,
                  global_reduction="mean", message_passes=2, positive_function="matrix_power_2",
                  max_edge_radius=0.05)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


# ---------------------------------------------------------------- known answers
def test_cart4_to_mandel_isotropic():
    """gnn/blocks.py:395-425 on lambda d_ij d_kl + mu (d_ik d_jl + d_il d_jk)."""
    lam, mu = 1.7, 0.6
    d = torch.eye(3, dtype=F64)
    c = lam * torch.einsum("ij,kl->ijkl", d, d) + mu * (torch.einsum("ik,jl->ijkl", d, d)
                                                        + torch.einsum("il,jk->ijkl", d, d))
    m = ob.Cart_4_to_Mandel().double()(c.unsqueeze(0))[0]
    ref = torch.zeros(6, 6, dtype=F64)
    ref[:3, :3] = lam
    ref[:3, :3] += 2 * mu * torch.eye(3, dtype=F64)
    ref[3:, 3:] = 2 * mu * torch.eye(3, dtype=F64)
    assert torch.allclose(m, ref, atol=1e-12)


def test_edge_vectors_formula():
    pos = torch.tensor([[0.0, 0.0, 0.0], [1.0, 2.0, 3.0]], dtype=F64)
    ei = torch.tensor([[0, 1], [1, 0]])
    shifts = torch.tensor([[0.5, 0.0, 0.0], [-0.5, 0.0, 0.0]], dtype=F64)
    v, ln = omace.get_edge_vectors_and_lengths(pos, ei, shifts)
    assert torch.allclose(v, torch.tensor([[1.5, 2.0, 3.0], [-1.5, -2.0, -3.0]], dtype=F64))
    assert torch.allclose(ln[:, 0], torch.full((2,), math.sqrt(1.5 ** 2 + 13), dtype=F64))


def test_positive_layer_and_unknown_function():
    c = torch.randn(3, 6, 6, dtype=F64)
    c = c + c.transpose(1, 2)
    pl = ob.PositiveLayer(small_params())
    assert torch.allclose(pl(c), c @ c)
    with pytest.raises(ValueError):
        ob.PositiveLayer(small_params(positive_function="nope"))


def test_loss_formula():
    """scripts/train_utils.py:54-60."""
    t = torch.randn(4, 6, 6, dtype=F64)
    p = torch.randn(4, 6, 6, dtype=F64)
    ref = 100 * np.mean([((p[i] - t[i]) ** 2).mean().item() / (t[i] ** 2).mean().item() for i in range(4)])
    assert abs(stiffness_loss(p, t).item() - ref) < 1e-10


def test_irreps_bookkeeping_counts():
    """SURVEY.md 3.3 / A.3 / A.4 numbers."""
    hid = oo3.Irreps("32x0e+32x1o+32x2e+32x3o+32x4e")
    sh = oo3.Irreps.spherical_harmonics(4)
    target = (sh * 32).sort()[0].simplify()
    assert str(target) == "32x0e+32x1o+32x2e+32x3o+32x4e"
    mid0, ins0 = omace.tp_out_irreps_with_instructions(oo3.Irreps("32x0e"), sh, target)
    mid1, ins1 = omace.tp_out_irreps_with_instructions(hid, sh, target)
    assert len(ins0) == 5 and mid0.dim == 800
    assert len(ins1) == 42 and mid1.dim == 7360
    assert str(mid1.simplify()) == "160x0e+256x1o+320x2e+320x3o+288x4e"
    dense = sum(oo3.wigner_3j(hid[i1].ir.l, sh[i2].ir.l, mid1[k].ir.l).numel() for i1, i2, k, *_ in ins1)
    assert dense == 7194
    ks = {}
    for l in range(5):
        ir = oo3.Irreps(str(oo3.Irrep(l, (-1) ** l)))
        ks[l] = [omace.U_matrix_real(oo3.Irreps("0e+1o+2e+3o+4e"), ir, nu)[-1].shape[-1] for nu in (1, 2, 3)]
    assert ks == {0: [1, 5, 42], 1: [1, 8, 99], 2: [1, 10, 139], 3: [1, 10, 155], 4: [1, 9, 150]}


def test_parameter_counts():
    """552,210 (4 layers) / 223,186 (2 layers), SURVEY.md A.3."""
    for layers, count in ((2, 223186), (4, 552210)):
        m = omodel.EnergyEquivGNN(params(layers))
        assert sum(p.numel() for p in m.parameters()) == count


# ---------------------------------------------------------------- basis consistency
def _rand_rot(seed=0):
    g = torch.Generator().manual_seed(seed)
    q, _ = torch.linalg.qr(torch.randn(3, 3, generator=g, dtype=F64))
    if torch.det(q) < 0:
        q[:, 0] = -q[:, 0]
    return q


def test_sh_norm_and_cg_intertwine_sh_rotations():
    rot = _rand_rot(1)
    pts = torch.randn(300, 3, generator=torch.Generator().manual_seed(2), dtype=F64)
    pts = pts / pts.norm(dim=-1, keepdim=True)
    ya = oo3.spherical_harmonics_norm(4, pts)
    yb = oo3.spherical_harmonics_norm(4, pts @ rot.T)
    for l in range(5):
        assert torch.allclose(ya[l].norm(dim=-1), torch.ones(300, dtype=F64), atol=1e-12)
    D = [torch.linalg.lstsq(ya[l], yb[l]).solution.T for l in range(5)]
    assert torch.allclose(D[1], rot, atol=1e-10)          # l=1 basis is (x, y, z)
    for l1 in range(5):
        for l2 in range(5):
            for l3 in range(abs(l1 - l2), min(4, l1 + l2) + 1):
                c = oo3.wigner_3j(l1, l2, l3)
                assert abs(c.norm().item() - 1) < 1e-12
                lhs = torch.einsum("ijk,ia,jb->abk", c, D[l1], D[l2])
                rhs = torch.einsum("abc,kc->abk", c, D[l3])
                assert torch.allclose(lhs, rhs, atol=1e-9), (l1, l2, l3)


def test_stiffness_change_of_basis():
    q = oo3.stiffness_change_of_basis().reshape(21, 81)
    assert torch.allclose(q @ q.T, torch.eye(21, dtype=F64), atol=1e-12)
    t = q.reshape(21, 3, 3, 3, 3)
    for perm in [(0, 2, 1, 3, 4), (0, 1, 2, 4, 3), (0, 3, 4, 1, 2)]:
        assert torch.allclose(t, t.permute(*perm), atol=1e-12)


# ---------------------------------------------------------------- model invariants
@pytest.fixture(scope="module")
def small_model():
    torch.manual_seed(0)
    b, rmax = batch(3, 30, 120, seed=11)
    m = omodel.EnergyEquivGNN(small_params(max_edge_radius=rmax)).double()
    return m, batch_to(b, "cpu", torch.float64)


def test_rotation_equivariance(small_model):
    m, b = small_model
    q = _rand_rot(5)
    with torch.no_grad():
        c = m(b)["stiffness"]
        b2 = batch_to(b, "cpu", torch.float64)
        b2.positions = b.positions @ q.T
        b2.shifts = b.shifts @ q.T
        c2 = m(b2)["stiffness"]
    # constants (U, Q) are stored in fp32 like the reference buffers -> ~1e-8 relative
    assert torch.allclose(c2, rotate_mandel(c, q), rtol=1e-6, atol=1e-6 * c.abs().max())


def test_translation_invariance_and_psd(small_model):
    m, b = small_model
    with torch.no_grad():
        c = m(b)["stiffness"]
        b2 = batch_to(b, "cpu", torch.float64)
        b2.positions = b.positions + torch.tensor([0.3, -1.2, 2.0], dtype=F64)
        c2 = m(b2)["stiffness"]
    assert torch.allclose(c, c2, atol=1e-10 * c.abs().max())
    ev = torch.linalg.eigvalsh(c)
    assert (ev > -1e-10 * ev.abs().max()).all()


def test_batching_invariance(small_model):
    m, b = small_model
    from gnn.synthetic import SyntheticLattices
    from gnn.data import collate
    ds = SyntheticLattices(3, 30, 120, 11)
    with torch.no_grad():
        cb = m(b)["stiffness"]
        cs = torch.cat([m(batch_to(collate([ds[g]]), "cpu", torch.float64))["stiffness"] for g in range(3)])
    assert torch.allclose(cb, cs, atol=1e-10 * cb.abs().max())


def test_oracle_gradcheck_interaction():
    """fp64 gradcheck of the TP interaction block (the kernel's backward target)."""
    torch.manual_seed(3)
    blk = ob.TensorProductInteractionBlock("4x0e+4x1o", oo3.Irreps.spherical_harmonics(2), "4x0e",
                                           "4x0e+4x1o+4x2e", 4.0, MLP_dim=8).double()
    x = torch.randn(5, 16, dtype=F64, requires_grad=True)
    v = torch.randn(7, 3, dtype=F64)
    sh = oo3.spherical_harmonics(2, v)
    ef = torch.randn(7, 4, dtype=F64)
    ei = torch.tensor([[0, 1, 2, 3, 4, 0, 2], [1, 2, 3, 4, 0, 3, 1]])
    assert torch.autograd.gradcheck(lambda xx: blk(xx, sh, ef, ei)[0], (x,))
